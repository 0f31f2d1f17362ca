#!/bin/bash
# round 5, call D: loader / storer roles in the tile forms: parity, timing, ablations, P = 16 forward
set -o pipefail
O=$PWD/gpurun_out/r05e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "wide_projections or glue_kernels or batched_pairs" --timeout 150 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
timeout -k 10 150 python tools/linear_ab.py 16 1024 "" 0123 b > $O/linear_ab.jsonl 2>&1 || exit 1
timeout -k 10 150 python tools/linear_ab.py 4 1024 "" 0123 >> $O/linear_ab.jsonl 2>&1 || exit 1
for v in 1 6; do
  MHA_HD64_LIB=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_abl$v.so timeout -k 10 120 python tools/linear_ab.py 16 1024 "" 1 > $O/linear_abl$v.jsonl 2>&1 || exit 1
done
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof.txt 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 4 1024 20 >> $O/mprof.txt 2>&1 || exit 1
