#!/bin/bash
# A/B timing of streaming-kernel library variants (forced plan 23, batched 1x4x1024^2 calls), one
# process per library, rounds interleaved:  bash tools/stream_ab.sh <lib.so> <lib.so> ...
set -o pipefail
for round in 1 2; do
  for L in "$@"; do
    echo -n "$(basename $L) r$round: "
    timeout -k 10 120 python3 tools/stream_check.py --no-parity --lib $L | python3 -c "
import sys, json
print(' '.join('%d:%s' % (d['calls_per_launch'], d['stream']['us_per_launch']) for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
