#!/bin/bash
# scratch GPU runner: stream tests, extreme-logit comparison, MALL/FETCH_SIZE microbenchmark
set -o pipefail
mkdir -p gpurun_out/mall
true
true
timeout -k 10 60 ./tools/mb_mall_count > gpurun_out/mall/plain.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mall/kt -o kt -- $R/tools/mb_mall_count > $R/gpurun_out/mall/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/mall/fs -o fs -- $R/tools/mb_mall_count > $R/gpurun_out/mall/fs.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $R/gpurun_out/mall/dram -o dram -- $R/tools/mb_mall_count > $R/gpurun_out/mall/dram.log 2>&1 || exit 1
cd $R
for M in 0 1 2; do MHA_HD64_F32_INKERNEL=$M timeout -k 10 120 python -u tools/f32_probe.py 1024-2048 512-1536 2048-2048 1024-1024 >> gpurun_out/f32_modes.jsonl 2>gpurun_out/f32_probe_err.log || exit 1; done
timeout -k 10 600 bash tools/pmc_f32.sh 1024 2048 || exit 1
