#!/bin/bash
# round 5, call T: how much of the one-launch FFN kernel is its LayerNorm + GELU epilogue
set -o pipefail
O=$PWD/gpurun_out/r05t; mkdir -p $O
A=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_lnabl.so
for i in 1 2; do
  timeout -k 10 200 python tools/linear_ab.py 16 1024 cat 1 b >> $O/lab_prod.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$A timeout -k 10 200 python tools/linear_ab.py 16 1024 cat 1 >> $O/lab_abl.jsonl 2>&1 || exit 1
done
