#!/bin/bash
# scratch GPU runner: stream tests, extreme-logit comparison, MALL/FETCH_SIZE microbenchmark
set -o pipefail
mkdir -p gpurun_out/mall
timeout -k 10 200 python -u tools/_extreme_logits.py > gpurun_out/extreme.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stream_tests.log 2>&1 || exit 1
timeout -k 10 60 ./tools/mb_mall_count > gpurun_out/mall/plain.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mall/kt -o kt -- $R/tools/mb_mall_count > $R/gpurun_out/mall/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/mall/fs -o fs -- $R/tools/mb_mall_count > $R/gpurun_out/mall/fs.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $R/gpurun_out/mall/dram -o dram -- $R/tools/mb_mall_count > $R/gpurun_out/mall/dram.log 2>&1 || exit 1
