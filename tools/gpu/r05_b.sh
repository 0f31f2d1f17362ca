#!/bin/bash
# round 5, call B: the LDS-staged projection tile forms: parity, A/B timing, matcher forward
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "wide_projections or glue_kernels or batched_pairs or sweep" --timeout 150 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
timeout -k 10 150 python tools/linear_ab.py 16 1024 "" 0123 b > $O/linear_ab.jsonl 2>&1 || exit 1
timeout -k 10 150 python tools/linear_ab.py 4 1024 "" 0123 >> $O/linear_ab.jsonl 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/matcher_plan_errors.py float16 > $O/matcher_plan_errors.jsonl 2> $O/mpe.err || exit 1
