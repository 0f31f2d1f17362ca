#!/bin/bash
# Build diagnostic ablation variants of the current kernel into lib/exp/libmha_hd64_abl<N>.so
# (N = bitmask of ABL_* in mha_hd64_kernels.hip). Never shipped; results are wrong by design.
set -e
D="$(dirname "$0")"
for N in "$@"; do
  "$D/build_variant.sh" "$D/../lightglue-with-flashattentionv2-tensorrt_amd/csrc/mha_hd64_kernels.hip" abl$N -DMHA_ABL=$N &
done
wait
