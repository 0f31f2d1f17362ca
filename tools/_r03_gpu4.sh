#!/bin/bash
timeout -k 10 120 ./tools/mb_mfma_shape > gpurun_out/mfma_shape.txt 2>&1 || exit 1
for M in 0 1 0 1; do echo "mode $M" >> gpurun_out/bs_ab.jsonl; MHA_HD64_STREAM=$M timeout -k 10 200 python -u tools/batched_streams.py >> gpurun_out/bs_ab.jsonl 2>>gpurun_out/bs_ab.err || exit 1; done
