#!/bin/bash
# round 5, call AD: 64-row one-launch FFN form by size (op alone at P = 1..32; forwards at P = 4, 8)
set -o pipefail
O=$PWD/gpurun_out/r05ad; mkdir -p $O
V=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_ln64.so
MHA_HD64_LIB=$V timeout -k 10 500 python tools/ln_fused_ab.py 1024 4x1024,8x1024 > $O/ln64_by_size.jsonl 2>&1 || exit 1
