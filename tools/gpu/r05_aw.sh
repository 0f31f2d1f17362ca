#!/bin/bash
# round 5, call AW: counters of the projection tile form 4 (128 x 128, 4 waves, two workgroups per CU)
# for qkv and linear+res at P = 16, beside form 1 (same run)
set -o pipefail
O=$PWD/gpurun_out/r05aw; mkdir -p $O
rm -rf gpurun_out/linpmc
MODES=4 OPS="qkv linear+res" timeout -k 10 600 bash tools/linear_pmc.sh > $O/linear_pmc4.log 2>&1 &&
mv gpurun_out/linpmc $O/form4 &&
MODES=1 OPS="qkv linear+res" timeout -k 10 600 bash tools/linear_pmc.sh > $O/linear_pmc1.log 2>&1 &&
mv gpurun_out/linpmc $O/form1
