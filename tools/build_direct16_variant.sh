#!/bin/bash
# Build a library variant of the 16-row single-pass kernel (A/B experiments; never shipped):
#   tools/build_direct16_variant.sh <name> [extra hipcc flags...]  -> lib/exp/libmha_hd64_<name>.so
# (run with MHA_HD64_LIB=lib/exp/libmha_hd64_<name>.so; WITH_DIRECT=1 builds the 32-row kernel with
# the same flags too)
set -e
NAME=$1; shift
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/exp
make -s lib/libmha_hd64.so
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans \
      -mllvm -amdgpu-kernarg-preload-count=12 "$@" -I../include -Icsrc -c csrc/mha_hd64_direct16.hip -o lib/exp/d16_$NAME.o
DOBJ=lib/obj/mha_hd64_direct.o
if [ "$WITH_DIRECT" = 1 ]; then
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans \
        "$@" -I../include -Icsrc -c csrc/mha_hd64_direct.hip -o lib/exp/d32_$NAME.o
  DOBJ=lib/exp/d32_$NAME.o
fi
hipcc --offload-arch=gfx950 -shared -fPIC lib/obj/mha_hd64_kernels.o $DOBJ lib/exp/d16_$NAME.o lib/obj/mha_hd64_stream.o \
      lib/obj/mha_hd64_plugin.o lib/obj/lightglue_glue.o lib/obj/lightglue_linear.o -o lib/exp/libmha_hd64_$NAME.so
rm -f lib/exp/d16_$NAME.o lib/exp/d32_$NAME.o
echo lib/exp/libmha_hd64_$NAME.so
