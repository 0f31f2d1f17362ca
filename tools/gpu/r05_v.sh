#!/bin/bash
# round 5, call V: packed fp16 output arithmetic in the projection epilogues (v_fma_mix, v_pk_add_f16)
set -o pipefail
O=$PWD/gpurun_out/r05v3; mkdir -p $O
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_base.so
timeout -k 10 600 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
for i in 1 2; do
  MHA_HD64_LIB=$B timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_base_$i.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/linear_ab.py 16 1024 "" 1 > $O/lab_new_$i.jsonl 2>&1 || exit 1
done
for P in 4 16 32; do
  for i in 1 2; do
    MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_base.txt 2>&1 || exit 1
    timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_new.txt 2>&1 || exit 1
  done
done
