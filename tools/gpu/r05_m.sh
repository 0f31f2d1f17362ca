#!/bin/bash
# round 5, call M: head-major epilogue with wave-uniform part / head and stepped rows, fp16 rotary
# (A/B against the HEAD build in lib/ab/libmha_hd64_base.so, and the row-step fast path in
# lib/ab/libmha_hd64_rowstep.so), matcher tests, pairs/s
set -o pipefail
O=$PWD/gpurun_out/r05m; mkdir -p $O
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_base.so
R=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_rowstep.so
for i in 1 2; do
  MHA_HD64_LIB=$B timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 b > $O/lab_base_$i.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_new_$i.jsonl 2>&1 || exit 1
  MHA_HD64_LIB=$R timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_rowstep_$i.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python tools/linear_ab.py 4 1024 "" 01 > $O/lab_new_p4.jsonl 2>&1 || exit 1
MHA_HD64_LIB=$R timeout -k 10 200 python tools/linear_ab.py 4 1024 "" 01 > $O/lab_rowstep_p4.jsonl 2>&1 || exit 1
MHA_HD64_LIB=$B timeout -k 10 200 python tools/linear_ab.py 4 1024 "" 01 > $O/lab_base_p4.jsonl 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 150 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
MHA_HD64_LIB=$R timeout -k 10 500 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "wide or batched or fused" --timeout 150 --timeout-method thread > $O/matcher_tests_rowstep.log 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof.txt 2>&1 || exit 1
MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof_base.txt 2>&1 || exit 1
MHA_HD64_LIB=$R timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof_rowstep.txt 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 >> $O/mprof.txt 2>&1 || exit 1
