#!/bin/bash
# round 5, call R: non-temporal output stores in the 256-row projection forms, whole forwards
set -o pipefail
O=$PWD/gpurun_out/r05r; mkdir -p $O
NT=lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_nt.so
for P in 4 8 16 32; do
  for i in 1 2; do
    timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/prod.txt 2>&1 || exit 1
    MHA_HD64_LIB=$NT timeout -k 10 150 python tools/matcher_profile.py $P 1024 20 >> $O/nt.txt 2>&1 || exit 1
  done
done
