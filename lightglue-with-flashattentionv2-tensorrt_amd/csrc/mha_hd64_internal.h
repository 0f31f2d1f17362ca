// mha_hd64_internal.h — host-side launch plumbing shared by the kernels and the plugin shim.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

namespace mha_hd64 {

constexpr int kHeadDim = 64;
constexpr int kMaxSeqLen = 2048;
constexpr int kNumHeads = 4;

enum class InType { F16, F32 };
enum class OutType { F16, F32 };

// One attention call: Q [batch, heads, nq, 64], K/V [batch, heads, nkv, 64], O like Q.
// Contiguous row-major ("kLINEAR"), the layout the reference plugin receives
// (lightglue_attention_plugin.cpp:122-163, head stride N*64).
struct Call {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    int batch;
    int heads;
    int nq;
    int nkv;
};

// Launch-shape choice for one call (exposed so tests/bench can force a variant).
struct LaunchPlan {
    int q_waves;          // waves per workgroup that own distinct 32-row query slices
    int kv_waves;         // waves per workgroup that split the keys of every iteration
    int rows_per_wave;    // 32, or 64 (two query blocks per wave); 16: the 16-row single-pass kernel
    int splits;           // KV split across workgroups (1 = no combine pass)
    int tiles_per_split;  // KV super-tiles (64 * kv_waves keys) per split
    size_t ws_needed;     // workspace bytes the plan uses
    int direct_tiles;     // > 0: single-pass kernel, 8 waves x direct_tiles 64-key tiles (no split)
    int stream;           // 1: the persistent streaming kernel (128-row items, no split)
};

// Up to kGroupCalls calls share one launch (grouped launcher); larger groups are chunked.
constexpr int kGroupCalls = 4;

// Plan of one launch carrying n <= kGroupCalls calls: one workgroup shape, per-call KV split,
// per-call workspace offsets (split partials laid out call after call).
struct GroupPlan {
    int q_waves;
    int kv_waves;
    int rows_per_wave;  // 32 or 64 (two query blocks per wave share every K/V fragment read)
    int splits[kGroupCalls];
    int tiles_per_split[kGroupCalls];
    size_t ws_offset[kGroupCalls];
    size_t ws_needed;
    int direct_tiles;  // > 0: the single-pass kernel (mha_hd64_direct.hip), q_waves 1 x kv_waves 8
    int stream;        // 1: the persistent streaming kernel (mha_hd64_stream.hip), 128-row items
};
// force_q_waves = kForceDirect selects the single-pass kernel (fp16 input, nkv <= 1024).
constexpr int kForceDirect = 21;
// force_q_waves = kForceDirect16 selects the 16-row single-pass kernel (mha_hd64_direct16.hip).
constexpr int kForceDirect16 = 22;
// force_q_waves = kForceStream selects the persistent streaming kernel (mha_hd64_stream.hip).
constexpr int kForceStream = 23;
GroupPlan plan_group(const Call* calls, int n, size_t ws_bytes, int force_q_waves = 0, int force_kv_waves = 0,
                     int force_splits = 0, InType in = InType::F16);
hipError_t launch_group(const Call* calls, int n, InType in, OutType out, void* workspace, size_t ws_bytes,
                        hipStream_t stream, int force_q_waves = 0, int force_kv_waves = 0, int force_splits = 0,
                        int phase_mask = 3);
// Workspace bytes launch_group can use for these calls with inputs of type `in`: the largest
// chunk's need (chunks of kGroupCalls reuse the workspace in stream order) -- split partials, or
// for fp32 inputs the fp16 copies the convert launch writes when a single-pass kernel runs them.
size_t group_workspace_bytes(const Call* calls, int n, InType in = InType::F16);

// Workgroup shapes compiled: (q_waves, kv_waves) in {(4,1), (2,2), (1,2), (4,2)} with 32-row waves,
// and (2,2) with 64-row waves (forced as q_waves = 12).
LaunchPlan plan_call(const Call& c, size_t ws_bytes, int force_q_waves = 0, int force_kv_waves = 0,
                     int force_splits = 0, InType in = InType::F16);
size_t split_workspace_bytes(const Call& c, int splits);

// Returns hipSuccess or the launch error. phase_mask (measurement hook): bit 0 = main
// kernel, bit 1 = split-KV combine kernel.
hipError_t launch_attention(const Call& c, InType in, OutType out, void* workspace, size_t ws_bytes,
                            hipStream_t stream, int force_q_waves = 0, int force_kv_waves = 0,
                            int force_splits = 0, int phase_mask = 3);

// Record an error for mha_hd64_last_error() (and abort if abort-on-error is set); returns status.
int32_t report_error(int32_t status, const char* where, const char* what);

// Diagnostic builds (-DMHA_STAMPS): where the kernel writes its per-workgroup timestamps.
void set_stamp_buffer(void* p);
// In-launch split combine on/off (default on unless env MHA_HD64_FUSED_COMBINE=0).
void set_fused_combine(int enable);
int set_stream_mode(int mode);      // 1 = persistent streaming kernel for large fp16 launches; returns the previous
void set_f32_inkernel(int enable);  // fp32 inputs: 1 = rounded in the 16-row kernel, 0 = convert launch,
                                    // 2 = also the two-pass forms (diagnostic)
// How the calling thread's last launch merged its splits: 0 none, 1 in-launch, 2 combine kernel.
int last_combine_form();
// Concurrent enqueue streams the host keeps busy (mha_hd64_set_concurrency_hint); >= 1.
int concurrency_hint();
int set_concurrency_hint(int streams);

}  // namespace mha_hd64
