#!/bin/bash
# Build a library variant of the persistent streaming kernel (A/B experiments; never shipped; lib/ab/ travels to the GPU box, delete it afterwards):
#   tools/build_stream_variant.sh <name> [extra hipcc flags...]  -> lib/ab/libmha_hd64_<name>.so
# (run with MHA_HD64_LIB=lib/ab/libmha_hd64_<name>.so or tools/stream_check.py --lib ...)
set -e
NAME=$1; shift
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/ab
make -s lib/libmha_hd64.so
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans \
      "$@" -I../include -Icsrc -c csrc/mha_hd64_stream.hip -o lib/ab/s_$NAME.o
hipcc --offload-arch=gfx950 -shared -fPIC lib/obj/mha_hd64_kernels.o lib/obj/mha_hd64_direct.o \
      lib/obj/mha_hd64_direct16.o lib/ab/s_$NAME.o lib/obj/mha_hd64_plugin.o lib/obj/lightglue_glue.o \
      lib/obj/lightglue_linear.o -o lib/ab/libmha_hd64_$NAME.so
rm -f lib/ab/s_$NAME.o
echo lib/ab/libmha_hd64_$NAME.so
