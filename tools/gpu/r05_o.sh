#!/bin/bash
# round 5, call O: one-launch Linear -> LayerNorm -> GELU by size (op alone; forwards at P = 8, 16, 32)
set -o pipefail
O=$PWD/gpurun_out/r05o; mkdir -p $O
timeout -k 10 500 python tools/ln_fused_ab.py 1024 8x1024,16x1024,32x1024 > $O/ln_fused_ab_p16.jsonl 2>&1 || exit 1
