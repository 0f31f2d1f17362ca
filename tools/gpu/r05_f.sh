#!/bin/bash
# round 5, call F: FFN input projection with LayerNorm + GELU in its epilogue
set -o pipefail
O=$PWD/gpurun_out/r05j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_matcher.py -x -q -s -m gpu --timeout 150 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 16 1024 20 > $O/mprof.txt 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 8 1024 20 >> $O/mprof.txt 2>&1 || exit 1
timeout -k 10 150 python tools/matcher_profile.py 32 1024 10 >> $O/mprof.txt 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mtrace -o m -- python3 $R/tools/matcher_profile.py 16 1024 10 > $O/mprof_traced.txt 2>&1 || exit 1
