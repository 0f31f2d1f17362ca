#!/bin/bash
# round 5, call P: one-launch Linear -> LayerNorm -> GELU by size as the default: matcher tests, forwards
set -o pipefail
O=$PWD/gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
for P in 8 16 32; do timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/mprof.txt 2>&1 || exit 1; done
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 >> $O/mprof.txt 2>&1 || exit 1
