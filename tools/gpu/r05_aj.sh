#!/bin/bash
# round 5, call AJ: counters of the streaming kernel at 32 calls, shipped (lazy) form and the
# speculative-max A/B build (tools/build_stream_variant.sh spec -DMHA_STREAM_SPEC=1), then the
# full verification (GPU suite, smoke, bench, round profile) into gpurun_out/r05v5
set -o pipefail
R=$PWD
timeout -k 10 400 bash tools/pmc_stream.sh 23 32 r05ship > /dev/null 2>&1 &&
MHA_HD64_LIB=$R/lightglue-with-flashattentionv2-tensorrt_amd/lib/ab/libmha_hd64_spec.so timeout -k 10 400 bash tools/pmc_stream.sh 23 32 r05spec > /dev/null 2>&1 &&
rm -rf lightglue-with-flashattentionv2-tensorrt_amd/lib/ab &&
OUT=r05v5 bash tools/gpu/r05_verify.sh
