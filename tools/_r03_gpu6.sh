#!/bin/bash
timeout -k 10 300 python -u tools/f32_routes.py 1x1024-1024 2x1024-1024 4x1024-1024 8x1024-1024 2x512-512 4x512-512 1x1024-2048 1x2048-2048 2x2048-2048 1x512-1536 3x1000-777 > gpurun_out/f32_routes2.jsonl 2> gpurun_out/f32_routes.err || exit 1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "float or f32 or Float or grouped or batched" --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
