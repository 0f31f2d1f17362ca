#!/bin/bash
# Build a library variant of the persistent streaming kernel (A/B experiments; never shipped):
#   tools/build_stream_variant.sh <name> [extra hipcc flags...]  -> lib/exp/libmha_hd64_<name>.so
# (run with MHA_HD64_LIB=lib/exp/libmha_hd64_<name>.so or tools/stream_check.py --lib ...)
set -e
NAME=$1; shift
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/exp
make -s lib/libmha_hd64.so
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans \
      "$@" -I../include -Icsrc -c csrc/mha_hd64_stream.hip -o lib/exp/s_$NAME.o
hipcc --offload-arch=gfx950 -shared -fPIC lib/obj/mha_hd64_kernels.o lib/obj/mha_hd64_direct.o \
      lib/obj/mha_hd64_direct16.o lib/exp/s_$NAME.o lib/obj/mha_hd64_plugin.o lib/obj/lightglue_glue.o \
      lib/obj/lightglue_linear.o -o lib/exp/libmha_hd64_$NAME.so
rm -f lib/exp/s_$NAME.o
echo lib/exp/libmha_hd64_$NAME.so
