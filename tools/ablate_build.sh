#!/bin/bash
# Build diagnostic ablation variants of the kernel library into lib/exp/libmha_hd64_abl<N>.so
# (N = bitmask of ABL_* in mha_hd64_kernels.hip). Never shipped; results are wrong by design.
set -e
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/exp
make -s lib/libmha_hd64.so
for N in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans -DMHA_ABL=$N \
        -I../include -Icsrc -c csrc/mha_hd64_kernels.hip -o lib/exp/k_abl$N.o &
done
wait
for N in "$@"; do
  hipcc --offload-arch=gfx950 -shared -fPIC lib/exp/k_abl$N.o lib/obj/mha_hd64_plugin.o -o lib/exp/libmha_hd64_abl$N.so
done
ls lib/exp
