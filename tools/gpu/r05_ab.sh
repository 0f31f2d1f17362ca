#!/bin/bash
# round 5, call AB: one-launch FFN kernel with per-workgroup rotated K order (W reads spread) vs production
set -o pipefail
O=$PWD/gpurun_out/r05ab; mkdir -p $O
V=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_krot.so
MHA_HD64_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "ln_gelu" --timeout 200 --timeout-method thread > $O/tests_krot.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_prod.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$V timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 >> $O/lab_krot.jsonl 2>&1 || exit 1
done
