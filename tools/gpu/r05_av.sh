#!/bin/bash
# round 5, call AV: matcher GPU tests with the larger ragged form-equality case
set -o pipefail
O=$PWD/gpurun_out/r05av; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
