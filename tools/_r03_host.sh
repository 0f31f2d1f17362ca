#!/bin/bash
B=lightglue-with-flashattentionv2-tensorrt_amd/lib/mha_hd64_host_bench
for a in "--nq 1024 --nkv 1024" "--nq 1024 --nkv 1024 --float" "--nq 2048 --nkv 2048" "--nq 2048 --nkv 2048 --float" "--nq 1024 --nkv 2048" "--nq 1536 --nkv 1536" "--nq 512 --nkv 512" "--nq 1024 --nkv 1024 --streams 4"; do
  timeout -k 10 120 $B --steps 2000 $a >> gpurun_out/host_bench_r03.jsonl 2>>gpurun_out/host_bench_r03.err || exit 1
done
