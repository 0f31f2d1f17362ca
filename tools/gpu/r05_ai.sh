#!/bin/bash
# round 5, call AI: speculative max with the MFMA rare path: parity suites, rare-path cost, slope A/B
# (run with the SPEC build as lib/libmha_hd64.so and the then-default lazy form as lib/ab/libmha_hd64_lazy.so;
#  the default is now the lazy form: rebuild the pair with tools/build_stream_variant.sh spec -DMHA_STREAM_SPEC=1)
set -o pipefail
O=$PWD/gpurun_out/r05ai; mkdir -p $O
P=lightglue-with-flashattentionv2-tensorrt_amd/lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/spec_rare_cost.py $P/libmha_hd64.so,$P/ab/libmha_hd64_lazy.so 32 > $O/rare_cost.jsonl 2>&1 &&
timeout -k 10 300 python tools/stream_check.py --slope $P/libmha_hd64.so,$P/ab/libmha_hd64_lazy.so > $O/slope1.jsonl 2>&1
