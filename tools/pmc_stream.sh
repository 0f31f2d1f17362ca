#!/bin/bash
# rocprofv3 counter passes of one forced plan of a batched 1024^2 launch (run on the GPU box from
# the repo root):  bash tools/pmc_stream.sh <plan code> <batch> <tag>
# One pass per run (gfx950 slot limits; no --pmc beside trace domains), each under its own timeout.
set -e
P=${1:-23}
B=${2:-32}
T=${3:-stream}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${T}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o p -- \
        python3 $R/tools/pmc_driver.py $P 1024 1024 30 $B > $OUT/pmc_$name.log 2>&1; }
run A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
run B SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run E SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o k -- \
    python3 $R/tools/pmc_driver.py $P 1024 1024 30 $B > $OUT/kt.log 2>&1
