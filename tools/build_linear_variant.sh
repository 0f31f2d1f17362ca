#!/bin/bash
# Build a library variant of the projection kernels, or (SRC=glue) of the glue kernels (A/B and
# ablation experiments; never shipped):
#   [SRC=glue] tools/build_linear_variant.sh <name> [extra hipcc flags, e.g. -DLG_ABL=1]  -> lib/ab/libmha_hd64_<name>.so
# lib/ab/ travels to the GPU box (lib/exp/ does not); delete it when the experiment is done.
set -e
NAME=$1; shift
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/ab
make -s lib/libmha_hd64.so
S=${SRC:-linear}
# (the Makefile's flags for each source: the glue kernels without the device flags)
if [ "$S" = glue ]; then SRCF=csrc/lightglue_glue.hip; KEEP=lib/obj/lightglue_linear.o; DEV=""
else SRCF=csrc/lightglue_linear.hip; KEEP=lib/obj/lightglue_glue.o; DEV="-mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans"; fi
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $DEV "$@" \
      -I../include -Icsrc -c $SRCF -o lib/ab/var_$NAME.o
OBJ="lib/obj/mha_hd64_kernels.o lib/obj/mha_hd64_plugin.o $KEEP lib/obj/mha_hd64_direct.o lib/obj/mha_hd64_direct16.o lib/obj/mha_hd64_stream.o"
hipcc --offload-arch=gfx950 -shared -fPIC lib/ab/var_$NAME.o $OBJ -o lib/ab/libmha_hd64_$NAME.so
rm -f lib/ab/var_$NAME.o
echo lib/ab/libmha_hd64_$NAME.so
