#!/bin/bash
# round 5, call Z: projection tile forms 1 (256 x 128) vs 3 (128 x 256) at P = 8, 16, 32
set -o pipefail
O=$PWD/gpurun_out/r05z; mkdir -p $O
for P in 8 16 32; do
  for i in 1 2; do
    timeout -k 10 200 python tools/linear_ab.py $P 1024 "" 13 >> $O/lab_13.jsonl 2>&1 || exit 1
  done
done
