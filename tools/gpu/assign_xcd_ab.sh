#!/bin/bash
# A/B of assign_lse_kernel's block order (LG_ASSIGN_XCD=0 grid order / 1 XCD-contiguous; the option existed only in
# the round-6 A/B build, measured and dropped: profiles/r06/assign_xcd_order_ab.txt). The steps:
# assignment-head tests, matcher forwards at P = 1 / 16 (interleaved), and a kernel trace each way.
#   bash tools/gpu/assign_xcd_ab.sh <tag>
set -o pipefail
T=${1:-r06ax}; R=$PWD; O=$R/gpurun_out/$T; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "assign or head or sweep or batched" > "$O/tests.log" 2>&1 || { tail -5 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for rep in 1 2 3; do for X in 0 1; do for P in 1 16; do
    LG_ASSIGN_XCD=$X timeout -k 10 120 python -u tools/matcher_profile.py $P 1024 50 > "$O/fwd_${X}_${P}_$rep.log" 2>&1 || exit $?
    echo "xcd=$X $(grep 'per forward' "$O/fwd_${X}_${P}_$rep.log")"
done; done; done | tee "$O/forwards.txt"
cd /tmp && export TMPDIR=/tmp
for X in 0 1; do
    LG_ASSIGN_XCD=$X timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$X" -o m -- \
        python3 "$R/tools/matcher_profile.py" 16 1024 20 > "$O/kt_$X.log" 2>&1 || exit $?
    grep -h "assign" $(find "$O/kt_$X" -name "m_kernel_stats.csv") | cut -c1-200
done
