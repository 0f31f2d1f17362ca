#!/bin/bash
# round 5, call S: packed LayerNorm + GELU epilogues (one-launch FFN kernel and the standalone kernel)
set -o pipefail
O=$PWD/gpurun_out/r05s; mkdir -p $O
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_base.so
L=lightglue-with-flashattentionv2-tensorrt_amd/lib/libmha_hd64.so
timeout -k 10 600 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/ln_ab.py $B,$L,$B,$L > $O/ln_ab.jsonl 2>&1 || exit 1
for i in 1 2; do
  MHA_HD64_LIB=$B timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 > $O/lab_base_$i.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/linear_ab.py 16 1024 cat_ln 1 > $O/lab_new_$i.jsonl 2>&1 || exit 1
done
for P in 8 16 32; do
  for i in 1 2; do
    MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_base.txt 2>&1 || exit 1
    timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_new.txt 2>&1 || exit 1
  done
done
