#!/bin/bash
# Per-kernel HBM traffic of the fp16 matcher forward (P pairs of n keypoints, graph replays of
# tools/matcher_profile.py): a kernel trace, then one --pmc pass each for FETCH_SIZE and WRITE_SIZE
# (never beside trace domains), summarised by tools/matcher_traffic.py.
#   bash tools/gpu/matcher_pmc.sh <P> <n> <tag>      (run on the GPU box from the repo root)
set -o pipefail
P=$1; N=$2; TAG=${3:-r06}
R=$PWD; O=$R/gpurun_out/mpmc_${TAG}_${P}x${N}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/kt" -o m -- \
    python3 "$R/tools/matcher_profile.py" "$P" "$N" 10 > "$O/kt.log" 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_$C" -o m -- \
        python3 "$R/tools/matcher_profile.py" "$P" "$N" 3 > "$O/pmc_$C.log" 2>&1 || exit $?
done
cd "$R" && python3 tools/matcher_traffic.py "$O" "$P" "$N" > "$O/summary.json" && tail -c 2000 "$O/summary.json"
