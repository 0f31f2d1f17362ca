#!/bin/bash
# round 6: ffn_rows_kernel segment stamps (lib/ab/libmha_hd64_frstamps.so) at several sizes (forced form 2)
set -o pipefail
O=$PWD/gpurun_out/${1:-r06f}; mkdir -p $O
for s in "1 512" "1 1024" "4 1024" "16 1024"; do
  MHA_HD64_LIB=$PWD/lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_frstamps.so timeout -k 10 120 python -u tools/fr_stamps.py $s >> $O/stamps.jsonl 2>> $O/err.log || exit 1
done
