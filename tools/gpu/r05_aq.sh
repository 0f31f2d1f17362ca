#!/bin/bash
# round 5, call AQ: the tile-form rule with the 8,192-row floor: matcher GPU tests, forwards default vs
# forms 1 / 0 forced at P = 1..32
set -o pipefail
O=$PWD/gpurun_out/r05aq; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python tools/form_fwd_ab.py 1,2,4,8,16,32 10 > $O/fwd.jsonl 2>&1
