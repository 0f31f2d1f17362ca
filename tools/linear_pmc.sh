#!/bin/bash
# PMC passes over the matcher projections (tools/linear_ab.py, P = 16, n = 1024, M = 32,768), one
# rocprofv3 run per counter group and op: OPS (op-name substrings, default all four) in form MODES
# (default 1 = the 256 x 128 tile form the planner takes at this size). Counter files land in
# gpurun_out/linpmc/pmc_<op>_<pass>/; tools/pmc_summary.py reduces them.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/linpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { op=$1; name=$2; shift 2; timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_${op}_$name -o p -- \
        python3 $R/tools/linear_ab.py 16 1024 "$op" ${MODES:-1} > $OUT/pmc_${op}_$name.log 2>&1; }
for op in ${OPS:-qkv split2 cat linear+res}; do
    run $op A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
    run $op B SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit 1
    run $op C FETCH_SIZE || exit 1
    run $op D WRITE_SIZE || exit 1
    run $op E SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
done
