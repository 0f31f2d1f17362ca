#!/bin/bash
# round 5, call AE: one-launch FFN form by size with the 64-row tiles in the middle range: tests, forwards vs HEAD
set -o pipefail
O=$PWD/gpurun_out/r05ae; mkdir -p $O
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_base.so
timeout -k 10 600 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
for P in 4 8 16; do
  for i in 1 2; do
    MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_base.txt 2>&1 || exit 1
    timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_new.txt 2>&1 || exit 1
  done
done
