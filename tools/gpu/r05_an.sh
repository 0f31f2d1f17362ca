#!/bin/bash
# round 5, call AN: projection tile forms 4 / 5 (128 x 128 on 4 waves, two workgroups per CU) against
# form 1 (256 x 128, 8 waves): form equality tests, then tools/linear_ab.py at P = 8 / 16 / 32
set -o pipefail
O=$PWD/gpurun_out/r05an; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -m gpu -q -k "wide_projections or linear_cat" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for P in 8 16 32; do timeout -k 10 200 python tools/linear_ab.py $P 1024 "" 145 >> $O/lab.jsonl 2>&1 || exit 1; done
