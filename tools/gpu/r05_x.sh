#!/bin/bash
# round 5, call X: one-launch FFN kernel with 64-row tiles (two per workgroup at P = 16) vs 128-row
set -o pipefail
O=$PWD/gpurun_out/r05x; mkdir -p $O
V=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_ln64.so
MHA_HD64_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "ln_gelu or batched or sweep" --timeout 200 --timeout-method thread > $O/tests_ln64.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_prod.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$V timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_ln64.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/linear_ab.py 32 1024 cat_ln 1 >> $O/lab_prod.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$V timeout -k 10 200 python tools/linear_ab.py 32 1024 cat_ln 1 >> $O/lab_ln64.jsonl 2>&1 || exit 1
done
for P in 16 32; do
  for i in 1 2; do
    timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_prod.txt 2>&1 || exit 1
    MHA_HD64_LIB=$V timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_ln64.txt 2>&1 || exit 1
  done
done
