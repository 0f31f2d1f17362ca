#!/bin/bash
# A/B of FFN library variants (lib/ab/libmha_hd64_<name>.so; "base" = the shipped build, measured
# first and last): tools/ffn_ab.py per library, then optional stamps builds.
#   bash tools/gpu/ffn_libs_ab.sh <tag> "<variant names>" "<ffn_ab args>" ["<stamps variant>" "<P n kind>"...]
set -o pipefail
tag=$1; vars=$2; args=$3; shift 3
O=$PWD/gpurun_out/$tag; mkdir -p "$O"; L=$PWD/lightglue-with-flashattentionv2-tensorrt_amd/lib
for v in base $vars base; do
    lib=$L/ab/libmha_hd64_$v.so; [ "$v" = base ] && lib=$L/libmha_hd64.so
    MHA_HD64_LIB=$lib timeout -k 10 300 python -u tools/ffn_ab.py $args >> "$O/$v.log" 2>&1 || exit 1
done
if [ $# -gt 0 ]; then
    sv=$1; shift
    for c in "$@"; do
        MHA_HD64_LIB=$L/ab/libmha_hd64_$sv.so timeout -k 10 120 python -u tools/fr_stamps.py $c >> "$O/stamps_$sv.log" 2>&1 || exit 1
    done
fi
