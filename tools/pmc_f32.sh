#!/bin/bash
# Float-boundary counters at 1x4xNQxNKV for set_f32_inkernel modes 0 (convert + fp16 kernel) and 2
# (the two-pass kernel rounding fp32 itself); one --pmc pass per run (run on the GPU box from the
# repo root):  bash tools/pmc_f32.sh [nq] [nkv]
set -e
NQ=${1:-1024}
NKV=${2:-2048}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_f32_${NQ}x${NKV}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for M in 0 2; do
  run() { name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/m${M}_$name -o p -- \
          python3 $R/tools/pmc_f32.py $M $NQ $NKV 30 > $OUT/m${M}_$name.log 2>&1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/m${M}_kt -o k -- \
      python3 $R/tools/pmc_f32.py $M $NQ $NKV 200 > $OUT/m${M}_kt.log 2>&1
  run F FETCH_SIZE
  run W WRITE_SIZE
  run A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
  run B SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
done
