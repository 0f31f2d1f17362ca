#!/bin/bash
L=lightglue-with-flashattentionv2-tensorrt_amd/lib
for lib in $L/libmha_hd64.so $L/exp/libmha_hd64_prio1.so $L/exp/libmha_hd64_prio2.so $L/exp/libmha_hd64_nofence.so $L/libmha_hd64.so; do
  echo "$lib" >> gpurun_out/prio_ab.jsonl
  timeout -k 10 200 python -u tools/stream_check.py --lib $lib --quick --no-timing > gpurun_out/prio_parity.log 2>>gpurun_out/prio_ab.err || exit 1
  timeout -k 10 200 python -u tools/stream_check.py --lib $lib --no-parity >> gpurun_out/prio_ab.jsonl 2>>gpurun_out/prio_ab.err || exit 1
done
