#!/bin/bash
# round 5, call W: stamps of the one-launch FFN kernel (where the 37 us go)
set -o pipefail
O=$PWD/gpurun_out/r05w; mkdir -p $O
S=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_lnstamps.so
MHA_HD64_LIB=$S timeout -k 10 200 python tools/ln_stamps.py 16 1024 > $O/ln_stamps.jsonl 2>&1 || exit 1
MHA_HD64_LIB=$S timeout -k 10 200 python tools/ln_stamps.py 32 1024 >> $O/ln_stamps.jsonl 2>&1 || exit 1
