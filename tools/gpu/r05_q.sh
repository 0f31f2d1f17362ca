#!/bin/bash
# round 5, call Q: counters of the rewritten head-major epilogues and of the one-launch FFN kernel
set -o pipefail
O=$PWD/gpurun_out/r05q; mkdir -p $O
rm -rf gpurun_out/linpmc
OPS="qkv split2 cat_ln" timeout -k 10 700 bash tools/linear_pmc.sh > $O/linear_pmc.log 2>&1 || exit 1
timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 b > $O/lab.jsonl 2>&1 || exit 1
NT=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_nt.so
for i in 1 2; do
  MHA_HD64_LIB=$NT timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_nt_$i.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_prod_$i.jsonl 2>&1 || exit 1
done
