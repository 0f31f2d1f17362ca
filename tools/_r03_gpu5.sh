#!/bin/bash

# Float path past one round of 16-row blocks: convert + 32-row kernel (default) vs the ring kernel's convert-on-load
for C in 1 0 1 0; do MHA_HD64_F32_CONVERT=$C timeout -k 10 150 python -u tools/f32_probe.py 2x1024-1024 3x1024-1024 4x1024-1024 8x1024-1024 2x512-512 4x512-512 2x1000-777 2x2048-2048 >> gpurun_out/f32_conv_ab.jsonl 2>>gpurun_out/f32_conv_ab.err || exit 1; done

timeout -k 10 120 ./tools/mb_mfma_shape > gpurun_out/mfma_shape.txt 2>&1 || exit 1
for M in 0 1 0 1; do echo "mode $M" >> gpurun_out/bs_ab.jsonl; MHA_HD64_STREAM=$M timeout -k 10 200 python -u tools/batched_streams.py >> gpurun_out/bs_ab.jsonl 2>>gpurun_out/bs_ab.err || exit 1; done
