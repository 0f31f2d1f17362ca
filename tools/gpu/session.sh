#!/bin/bash
# One GPU session: named steps run in order, each under its own time limit, stopping at the first
# failure (no GPU step runs after a fault, abort or timeout). Logs in gpurun_out/<tag>/.
#   bash tools/gpu/session.sh <tag> <step> [<step> ...]
# steps: tests[:<pytest -k expr>]  gpu  ffn_ab[:<args>]  bench[:<args>]  smoke  prof_fwd:<P>x<n>
set -o pipefail
tag=$1; shift
O=$PWD/gpurun_out/$tag; mkdir -p "$O"
export PYTHONUNBUFFERED=1
run() {  # run <seconds> <log> <cmd...>
    local t=$1 log=$2; shift 2
    echo "[$(date +%T)] $*" | tee -a "$O/steps.txt"
    timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
    local rc=$?
    echo "[$(date +%T)] rc=$rc" | tee -a "$O/steps.txt"
    tail -5 "$O/$log"
    return $rc
}
for step in "$@"; do
    name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
    case $name in
        tests)  run 900 "tests_${arg//[^a-zA-Z0-9_]/_}.log" python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${arg:+-k "$arg"} || exit $? ;;
        gpu)    run 1100 gpu_suite.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $? ;;
        ffn_ab) run 600 "ffn_ab.log" python -u tools/ffn_ab.py $arg || exit $? ;;
        bench)  run 900 "bench.log" python -u bench.py $arg || exit $? ;;
        smoke)  run 300 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        prof_fwd)  # kernel trace of P x n forwards (graph replays), then one forward's timeline
            P=${arg%x*}; n=${arg#*x}; R=$PWD
            (cd /tmp && TMPDIR=/tmp run 300 "prof_fwd_${P}x${n}.log" rocprofv3 --kernel-trace --output-format csv \
                -d "$O/fwd_${P}x${n}" -o m -- python3 "$R/tools/matcher_profile.py" "$P" "$n" 10) || exit $?
            f=$(find "$O/fwd_${P}x${n}" -name "m_kernel_trace.csv" | head -1)
            python3 tools/forward_timeline.py "$f" > "$O/timeline_${P}x${n}.txt" 2>&1; cat "$O/timeline_${P}x${n}.txt" | head -20 ;;
        *) echo "unknown step $name"; exit 2 ;;
    esac
done
