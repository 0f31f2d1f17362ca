#!/bin/bash
# round-3 bench + profiles (run on the GPU box from the repo root)
set -o pipefail
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r03.json 2> gpurun_out/bench_r03.err || exit 1
timeout -k 10 640 bash tools/profile_round.sh r03 || exit 1
