#!/bin/bash
# One GPU session: named steps run in order, each under its own time limit, stopping at the first
# failure (no GPU step runs after a fault, abort or timeout). Logs in gpurun_out/<tag>/.
#   bash tools/gpu/session.sh <tag> <step> [<step> ...]
# steps: tests[:<pytest -k expr>]  gpu  ffn_ab[:<args>]  bench[:<args>]  smoke  prof_fwd:<P>x<n>
#        pmc_ffn:<P>:<n>:<mode>  "tool:<tools/NAME.py> [args...]" (one quoted word)
#        "frstamps:<P> <n> <kind>" (FFN segment stamps; build lib/ab/libmha_hd64_frstamps.so first with
#        tools/build_linear_variant.sh frstamps -DLG_FR_STAMPS)
# (the round-start check: gpu smoke "bench:--steps 20 --warmup 5"; round 5's 50 tools/gpu/r05_*.sh
# sessions were each one such list of steps, folded into this script in round 6)
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
        bench)  b=${arg//[^a-zA-Z0-9]/_}; run 900 "bench${b:+_${b:0:60}}.log" python -u bench.py $arg || exit $? ;;
        tool)   # one diagnostic script of tools/ (its stdout in <name>.log)
            read -r -a ta <<< "$arg"; tn=${ta[0]}; sfx=$(basename -a "${ta[@]:1}" 2>/dev/null | tr -c 'a-zA-Z0-9\n' '_' | tr '\n' '_')
            run 600 "${tn}_${sfx:0:60}.log" python -u "tools/${tn}.py" "${ta[@]:1}" || exit $? ;;
        frstamps)
            run 120 "frstamps_${arg// /_}.log" env MHA_HD64_LIB=$PWD/lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_frstamps.so \
                python -u tools/fr_stamps.py $arg || exit $?
            grep '^{' "$O/frstamps_${arg// /_}.log" >> "$O/stamps.jsonl" ;;
        smoke)  run 300 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        prof_fwd)  # kernel trace of P x n forwards (graph replays), then one forward's timeline (arg PxN[:fp32])
            sz=${arg%%:*}; dt=fp16; [ "$sz" != "$arg" ] && dt=${arg#*:}
            P=${sz%x*}; n=${sz#*x}; R=$PWD; t=${P}x${n}${dt/fp16/}
            (cd /tmp && TMPDIR=/tmp run 300 "prof_fwd_${t}.log" rocprofv3 --kernel-trace --output-format csv \
                -d "$O/fwd_${t}" -o m -- python3 "$R/tools/matcher_profile.py" "$P" "$n" 10 "$dt") || exit $?
            f=$(find "$O/fwd_${t}" -name "m_kernel_trace.csv" | head -1)
            python3 tools/forward_timeline.py "$f" > "$O/timeline_${t}.txt" 2>&1; cat "$O/timeline_${t}.txt" | head -20 ;;
        pmc_ffn)  # counter passes over lg_linear_cat_ffn at P x n (arg P:n:mode)
            IFS=: read -r P n mode <<< "$arg"; R=$PWD
            for pass in "A:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
                        "B:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
                        "C:FETCH_SIZE" "D:WRITE_SIZE" "E:SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
                pn=${pass%%:*}; ctr=${pass#*:}
                (cd /tmp && TMPDIR=/tmp run 120 "pmc_ffn_${P}_${mode}_$pn.log" rocprofv3 --pmc $ctr --output-format csv \
                    -d "$O/pmc_ffn_${P}_${mode}_$pn" -o p -- python3 "$R/tools/ffn_driver.py" "$P" "$n" "$mode" 20) || exit $?
            done ;;
        *) echo "unknown step $name"; exit 2 ;;
    esac
done
