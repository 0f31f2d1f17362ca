# A/B of stream-kernel variant libraries (diagnostic): timing of B = 16 / 32 batched launches
rm -f gpurun_out/abl.jsonl
for W in 8; do for L in lib/exp/libmha_hd64_abl8.so lib/exp/libmha_hd64_abl7.so lib/exp/libmha_hd64_abl15.so lib/exp/libmha_hd64_abl23.so lib/exp/libmha_hd64_abl31.so; do
MHA_HD64_STREAM_WAVES=$W timeout -k 10 100 python -u -c "
import sys, json; sys.path.insert(0,'tools')
import stream_check as s, torch
print('$W', '$L', flush=True)
s.timing(s.load('lightglue-with-flashattentionv2-tensorrt_amd/$L'), torch.device('cuda:0'), False)" >> gpurun_out/abl.jsonl 2>>gpurun_out/abl.err || exit 1
done; done
