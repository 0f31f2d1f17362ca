#!/bin/bash
# round 5, call AA: one-launch FFN kernel with its A operand from L2-hot rows (diagnostic) vs production
set -o pipefail
O=$PWD/gpurun_out/r05aa; mkdir -p $O
V=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_ahot.so
for i in 1 2 3; do
  timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_prod.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$V timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_ahot.jsonl 2>&1 || exit 1
done
