#!/bin/bash
# round 5, call AC: counters of the packed one-launch FFN kernel (final build)
set -o pipefail
O=$PWD/gpurun_out/r05ac; mkdir -p $O
rm -rf gpurun_out/linpmc
OPS="cat_ln" timeout -k 10 400 bash tools/linear_pmc.sh > $O/linear_pmc.log 2>&1 || exit 1
