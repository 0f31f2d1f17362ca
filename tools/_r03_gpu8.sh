#!/bin/bash
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
export GT_CASES="c1024:1:1024:1024:22:0:0;c512:1:512:512:22:0:0;c768:1:768:768:22:0:0;c1k2k:1:1024:2048:22:0:0;c2k:1:2048:2048:22:0:0"
timeout -k 10 300 python -u tools/graph_time.py $L/libmha_hd64.so $L/exp/libmha_hd64_st2.so $L/exp/libmha_hd64_st3.so $L/exp/libmha_hd64_st4.so > gpurun_out/stage16.json 2> gpurun_out/stage16.err || exit 1
MHA_HD64_LIB=$L/exp/libmha_hd64_st3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "direct_kernel or planner_default or full_tensor or nan or nonfinite" --timeout 120 --timeout-method thread > gpurun_out/stage16_tests.log 2>&1
