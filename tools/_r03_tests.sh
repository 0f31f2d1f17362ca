#!/bin/bash
# full GPU suite (as the driver runs it, with per-test timeouts)
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r03.log 2>&1
