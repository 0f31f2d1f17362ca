#!/bin/bash
# round 5, call K: streaming kernel A/B (static priority for waves 4-7 of the 8-wave form)
set -o pipefail
O=$PWD/gpurun_out/r05k; mkdir -p $O
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
timeout -k 10 300 python tools/stream_check.py --no-parity --slope $L/libmha_hd64.so,$L/ab/libmha_hd64_prio.so,$L/libmha_hd64.so,$L/ab/libmha_hd64_prio.so > $O/slope_prio.jsonl 2>&1 || exit 1
