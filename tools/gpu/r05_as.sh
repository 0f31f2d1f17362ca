#!/bin/bash
# round 5, call AS: kernel trace of P = 16 and P = 32 forwards on the final build (tile form 4)
set -o pipefail
O=$PWD/gpurun_out/r05as; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for P in 16 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$P -o m -- python3 $R/tools/matcher_profile.py $P 1024 10 > $O/p$P.txt 2>&1 || exit 1
done
