#!/bin/bash
# round 5, call Y2: the column pass with 16 groups; tests; single-pair forwards vs HEAD
set -o pipefail
O=$PWD/gpurun_out/r05y2; mkdir -p $O
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_base.so
timeout -k 10 600 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/matcher_tests.log 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
for n in 1024 2048; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/new_$n -o m -- python3 $R/tools/matcher_profile.py 1 $n 20 > $O/new_$n.txt 2>&1 || exit 1
done
cd $R
for n in 512 1024 2048; do
  for i in 1 2; do
    MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py 1 $n 50 >> $O/fwd_base.txt 2>&1 || exit 1
    timeout -k 10 150 python tools/matcher_profile.py 1 $n 50 >> $O/fwd_new.txt 2>&1 || exit 1
  done
done
for P in 2 4; do
  MHA_HD64_LIB=$B timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_base.txt 2>&1 || exit 1
  timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/fwd_new.txt 2>&1 || exit 1
done
