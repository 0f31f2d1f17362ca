#!/bin/bash
timeout -k 10 300 python -u tools/f32_routes.py 1x1024-1024 2x1024-1024 4x1024-1024 8x1024-1024 2x512-512 4x512-512 1x1024-2048 1x2048-2048 2x2048-2048 1x512-1536 > gpurun_out/f32_routes.jsonl 2> gpurun_out/f32_routes.err
