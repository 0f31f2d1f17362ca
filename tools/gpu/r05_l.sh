#!/bin/bash
# round 5, call L: LayerNorm + GELU persistent-form A/B (tools/ln_ab.py), then PMC passes over the
# four projections in the production tile form (tools/linear_pmc.sh)
set -o pipefail
O=$PWD/gpurun_out/r05l; mkdir -p $O
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
V=$L/libmha_hd64.so,$L/ab/libmha_hd64_f1d2b4.so,$L/ab/libmha_hd64_f1d2b8.so,$L/ab/libmha_hd64_f1d4b4.so,$L/ab/libmha_hd64_f1d1b8.so,$L/ab/libmha_hd64_f1d3b6.so
timeout -k 10 300 python tools/ln_ab.py $V > $O/ln_ab.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/ln_ab.py $V 8192 >> $O/ln_ab.jsonl 2>&1 || exit 1
timeout -k 10 950 bash tools/linear_pmc.sh > $O/linear_pmc.log 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/linpmc > $O/linear_pmc_summary.json 2>&1 || exit 1
