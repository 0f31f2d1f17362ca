#!/bin/bash
# round 5, call AT: the one-launch FFN input projection as 64-row tiles on 4 waves, two workgroups
# per CU (-DLG_LN_2WG=1 build) vs the shipped 128-row form: the op alone (interleaved), then forwards
# under each library (separate processes)
set -o pipefail
O=$PWD/gpurun_out/r05at; mkdir -p $O
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
timeout -k 10 200 python tools/ln_lib_ab.py $L/libmha_hd64.so,$L/ab/libmha_hd64_ln2wg.so 16,32 > $O/op.jsonl 2>&1 &&
timeout -k 10 200 python tools/form_fwd_ab.py 16,32 "" > $O/fwd_ship.jsonl 2>&1 &&
MHA_HD64_LIB=$PWD/$L/ab/libmha_hd64_ln2wg.so timeout -k 10 200 python tools/form_fwd_ab.py 16,32 "" > $O/fwd_2wg.jsonl 2>&1 &&
timeout -k 10 200 python tools/form_fwd_ab.py 16,32 "" > $O/fwd_ship2.jsonl 2>&1
