#!/bin/bash
# round 5, call A: plan-23 fixture tests, matcher error sources, projection yardsticks + ablations
set -o pipefail
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -q -k "reference_fixtures" --timeout 120 --timeout-method thread > $O/stream_fixture_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/matcher_plan_errors.py float16 > $O/matcher_plan_errors.jsonl 2> $O/mpe.err || exit 1
timeout -k 10 300 python -u tools/matcher_plan_errors.py float32 >> $O/matcher_plan_errors.jsonl 2>> $O/mpe.err || exit 1
timeout -k 10 120 python tools/linear_ab.py 16 1024 "" 12 b > $O/linear_yardsticks.jsonl 2>&1 || exit 1
for v in 1 2 4 3 6; do
  MHA_HD64_LIB=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_abl$v.so timeout -k 10 120 python tools/linear_ab.py 16 1024 "" 12 > $O/linear_abl$v.jsonl 2>&1 || exit 1
done
