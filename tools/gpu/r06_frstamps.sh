#!/bin/bash
# round 6: ffn_rows_kernel segment stamps (lib/ab/libmha_hd64_frstamps.so): "P n kind" cases
set -o pipefail
O=$PWD/gpurun_out/${1:-r06f}; mkdir -p $O; shift
for s in "${@:-1 1024 0}"; do
  MHA_HD64_LIB=$PWD/lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_frstamps.so timeout -k 10 120 python -u tools/fr_stamps.py $s >> $O/stamps.jsonl 2>> $O/err.log || exit 1
done
