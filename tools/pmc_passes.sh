#!/bin/bash
# rocprofv3 recipe for the MHAHeadDim64 kernels (run on the GPU box from the repo root):
#   bash tools/pmc_passes.sh <workload: call|batched> <tag>
# Counter passes are separate runs (gfx950 slot limits; no --pmc beside trace domains).
set -e
W=${1:-batched}
T=${2:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${T}_${W}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o p -- \
        python3 $R/bench.py --only $W --steps 40 --warmup 5 > $OUT/pmc_$name.log 2>&1; }
run A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
run B SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run C FETCH_SIZE
run D WRITE_SIZE
run E SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o k -- \
    python3 $R/bench.py --only $W --steps 100 --warmup 5 > $OUT/kt.log 2>&1
