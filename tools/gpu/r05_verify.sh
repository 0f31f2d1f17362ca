#!/bin/bash
# round 5: full GPU suite, smoke, the driver's bench command, then the round profile
set -o pipefail
O=gpurun_out/${OUT:-r05v}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 900 bash tools/profile_round.sh r05 > $O/profile_round.log 2>&1 || exit 1
