#!/bin/bash
# Build a library variant from a kernel source file (A/B experiments; never shipped; PLUGIN_SRC=
# an older shim source when the kernel source predates the current internal header):
#   tools/build_variant.sh <kernel.hip> <name> [extra hipcc flags...]  -> lib/exp/libmha_hd64_<name>.so
set -e
SRC=$(readlink -f "$1"); NAME=$2; shift 2
cd "$(dirname "$0")/../lightglue-with-flashattentionv2-tensorrt_amd"
mkdir -p lib/exp
make -s lib/libmha_hd64.so
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans "$@" \
      -I../include -Icsrc -c "$SRC" -o lib/exp/k_$NAME.o
PLUG="lib/obj/mha_hd64_plugin.o lib/obj/lightglue_glue.o lib/obj/lightglue_linear.o lib/obj/mha_hd64_direct.o lib/obj/mha_hd64_direct16.o lib/obj/mha_hd64_stream.o"
if [ -n "$PLUGIN_SRC" ]; then  # an older plugin shim for an older kernel source
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -c "$(readlink -f "$PLUGIN_SRC")" -o lib/exp/p_$NAME.o
  PLUG=lib/exp/p_$NAME.o
fi
hipcc --offload-arch=gfx950 -shared -fPIC lib/exp/k_$NAME.o $PLUG -o lib/exp/libmha_hd64_$NAME.so
rm -f lib/exp/p_$NAME.o
rm -f lib/exp/k_$NAME.o
echo lib/exp/libmha_hd64_$NAME.so
