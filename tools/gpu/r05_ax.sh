#!/bin/bash
# round 5, call AX: the random-shape parity sweep widened to 400 / 400 / 300 cases
set -o pipefail
O=$PWD/gpurun_out/r05ax; mkdir -p $O
LG_FUZZ_CASES=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread > $O/fuzz400.log 2>&1
