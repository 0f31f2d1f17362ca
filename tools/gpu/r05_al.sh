#!/bin/bash
# round 5, call AL: ffn_kernel ablations (-DLG_FFN_ABL=1/2/4/8) and prefetch depths (-DLG_FFN_PF=4/16)
# against the default build, the op alone at P = 16 / 32 (tools/ffn_ab.py <libs>)
set -o pipefail
O=$PWD/gpurun_out/r05al; mkdir -p $O
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
timeout -k 10 300 python tools/ffn_ab.py $L/libmha_hd64.so,$L/ab/libmha_hd64_ffnabl1.so,$L/ab/libmha_hd64_ffnabl2.so,$L/ab/libmha_hd64_ffnabl4.so,$L/ab/libmha_hd64_ffnabl8.so,$L/ab/libmha_hd64_pf4.so,$L/ab/libmha_hd64_pf16.so > $O/abl.jsonl 2>&1
