#!/bin/bash
# Round profiles (run on the GPU box from the repo root): the bench command under a kernel trace,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE; never combined with trace domains) of the
# single-call workload. Output under gpurun_out/prof_<tag>/; summaries copied to profiles/ by hand.
set -e
TAG=${1:-r02}
OUT=$PWD/gpurun_out/prof_$TAG
REPO=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 "$REPO/bench.py" --steps 20 --warmup 5 > "$OUT/bench_stdout.json" 2> "$OUT/bench_stderr.log"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o call -- \
      python3 "$REPO/bench.py" --only call --steps 50 --warmup 5 > /dev/null 2> "$OUT/pmc_$C.log"
done
python3 "$REPO/tools/pmc_summary.py" "$OUT/trace" "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" > "$OUT/summary.json"
