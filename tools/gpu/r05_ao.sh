#!/bin/bash
# round 5, call AO: tile form 4 as the by-size default for the non-gather projections: matcher GPU
# tests, forms 0 / 1 / 4 at P = 2 / 4 (the threshold), forwards default vs form 1 forced at P = 4..32
set -o pipefail
O=$PWD/gpurun_out/r05ao; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for P in 2 4; do timeout -k 10 200 python tools/linear_ab.py $P 1024 "" 014 >> $O/lab.jsonl 2>&1 || exit 1; done &&
timeout -k 10 300 python tools/form_fwd_ab.py 4,8,16,32 1 > $O/fwd.jsonl 2>&1
