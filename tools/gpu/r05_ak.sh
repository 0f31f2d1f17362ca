#!/bin/bash
# round 5, call AK: the whole FFN in one launch (lg_linear_cat_ffn / ffn_kernel): its parity tests and
# the matcher GPU tests, then the op alone vs the two calls and P = 8 / 16 / 32 forwards (tools/ffn_ab.py)
set -o pipefail
O=$PWD/gpurun_out/r05ak; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/ffn_ab.py > $O/ffn_ab.jsonl 2>&1
