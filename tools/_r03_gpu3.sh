#!/bin/bash
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nonfinite or nan_inputs or grouped_past" tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nf_tests.log 2>&1 || exit 1
bash tools/_r03_gpu1.sh
