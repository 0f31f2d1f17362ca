#!/bin/bash
# round 5, call C: tile-form ablations, matcher tests with the new bounds, P = 16 forward kernel trace
set -o pipefail
O=$PWD/gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "batched_pairs or sweep" --timeout 150 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
for v in 1 2 4 6; do
  MHA_HD64_LIB=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_abl$v.so timeout -k 10 120 python tools/linear_ab.py 16 1024 "" 1 > $O/linear_abl$v.jsonl 2>&1 || exit 1
done
timeout -k 10 120 python tools/linear_ab.py 16 1024 "" 1 > $O/linear_abl0.jsonl 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mtrace -o m -- python3 $R/tools/matcher_profile.py 16 1024 10 > $O/mprof_traced.txt 2>&1 || exit 1
