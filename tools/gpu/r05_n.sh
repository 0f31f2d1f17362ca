#!/bin/bash
# round 5, call N: the new form-equality cases; kernel timelines of single-pair forwards (configs[3])
set -o pipefail
O=$PWD/gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -x -q -m gpu -k "wide_projections" --timeout 150 --timeout-method thread > $O/wide_tests.log 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
for n in 512 1024 2048; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p1_$n -o m -- python3 $R/tools/matcher_profile.py 1 $n 10 > $O/p1_$n.txt 2>&1 || exit 1
done
