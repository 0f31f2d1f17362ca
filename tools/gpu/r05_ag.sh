#!/bin/bash
# round 5, call AG: seeded random-shape parity sweep through the plugin, batched and grouped launchers
set -o pipefail
O=$PWD/gpurun_out/r05ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -v --timeout 120 --timeout-method thread > $O/fuzz.log 2>&1
