#!/bin/bash
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r03b.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r03.log 2>&1 || exit 1
true
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err || exit 1
