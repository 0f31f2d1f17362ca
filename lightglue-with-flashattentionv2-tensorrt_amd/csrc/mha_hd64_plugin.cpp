// mha_hd64_plugin.cpp — host side of the MHAHeadDim64 operator: a plugin object with the
// IPluginV2DynamicExt surface of the reference (lightglue_attention_plugin/lightglue_attention_plugin.h:28-159,
// .cpp:28-422) re-expressed without TensorRT, plus the extern "C" shim declared in include/mha_hd64.h.
//
// Behavioural contract kept from the reference:
//  * identity "MHAHeadDim64" / "1" / namespace "" , no fields, no serialized state (.cpp:19-20, 45-55, 363-367)
//  * getOutputDimensions = inputs[0] (.cpp:79-94); getOutputDataType = inputs_type[0] (.cpp:298-310)
//  * supportsFormatCombination: pos 0 FLOAT|HALF + LINEAR, pos 1..3 same type + LINEAR (.cpp:272-296)
//  * configurePlugin / enqueue validate B==1, H==4, N<=2048, Nk==Nv, No==Nq, D==64, one dtype, LINEAR
//    (.cpp:122-163, 330-358)
//  * getWorkspaceSize: fixed 3*(1*4*2048*64*2) + 1*4*2048*64*4 = 5,242,880 B (.cpp:96-112)
//  * enqueue: Half -> fp16 in/fp16 out; Float -> fp32 in (rounded to fp16), fp32 out (.cpp:177-267)
// Deliberate deviations:
//  * a failed assertion returns MHA_HD64_STATUS_BAD_PARAM (or aborts when mha_hd64_set_abort_on_error(1))
//    instead of cudaDeviceReset()+abort() (common/checkMacrosPlugin.cpp:118-128);
//  * enqueue reports launch errors (the reference always returns 0);
//  * no pad / unpad / convert launches: tails and the fp32->fp16 rounding happen inside the kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <vector>

#include "mha_hd64.h"
#include "mha_hd64_internal.h"

namespace {

constexpr const char* kPluginName = "MHAHeadDim64";
constexpr const char* kPluginVersion = "1";

thread_local std::string g_last_error;
bool g_abort_on_error = false;

int32_t fail(int32_t status, const char* file, int line, const char* what) {
    char buf[512];
    std::snprintf(buf, sizeof(buf), "mha_hd64: %s (%s:%d)", what, file, line);
    g_last_error = buf;
    if (g_abort_on_error) {
        std::fprintf(stderr, "%s\n", buf);
        std::abort();
    }
    return status;
}

#define MHA_CHECK(cond)                                                                      \
    do {                                                                                     \
        if (!(cond)) return fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__, "assertion failed: " #cond); \
    } while (0)

// Workspace layout constants of the reference (lightglue_attention_plugin.h:112-120).
constexpr size_t kWsQ = (size_t)MHA_HD64_BATCH * MHA_HD64_NUM_HEADS * MHA_HD64_MAX_SEQ_LEN * MHA_HD64_HEAD_DIM * 2;
constexpr size_t kWsO = (size_t)MHA_HD64_BATCH * MHA_HD64_NUM_HEADS * MHA_HD64_MAX_SEQ_LEN * MHA_HD64_HEAD_DIM * 4;
constexpr size_t kWorkspaceBytes = 3 * kWsQ + kWsO;  // 5,242,880

// Shape/type validation shared by configurePlugin and enqueue (reference .cpp:122-163 == .cpp:330-358).
int32_t validate(const mha_hd64_tensor_desc_t* in, const mha_hd64_tensor_desc_t* out) {
    MHA_CHECK(in != nullptr && out != nullptr);
    MHA_CHECK(in[0].dims.nb_dims == 4);
    MHA_CHECK(in[1].dims.nb_dims == 4);
    MHA_CHECK(in[2].dims.nb_dims == 4);
    MHA_CHECK(out[0].dims.nb_dims == 4);

    MHA_CHECK(in[0].dims.d[0] == MHA_HD64_BATCH);
    MHA_CHECK(in[0].dims.d[0] == in[1].dims.d[0]);
    MHA_CHECK(in[1].dims.d[0] == in[2].dims.d[0]);
    MHA_CHECK(in[0].dims.d[0] == out[0].dims.d[0]);

    MHA_CHECK(in[0].dims.d[1] == MHA_HD64_NUM_HEADS);
    MHA_CHECK(in[0].dims.d[1] == in[1].dims.d[1]);
    MHA_CHECK(in[1].dims.d[1] == in[2].dims.d[1]);
    MHA_CHECK(in[0].dims.d[1] == out[0].dims.d[1]);

    MHA_CHECK(in[0].dims.d[2] <= MHA_HD64_MAX_SEQ_LEN);
    MHA_CHECK(in[1].dims.d[2] <= MHA_HD64_MAX_SEQ_LEN);
    MHA_CHECK(in[1].dims.d[2] == in[2].dims.d[2]);
    MHA_CHECK(in[0].dims.d[2] == out[0].dims.d[2]);

    MHA_CHECK(in[0].dims.d[3] == MHA_HD64_HEAD_DIM);
    MHA_CHECK(in[0].dims.d[3] == in[1].dims.d[3]);
    MHA_CHECK(in[1].dims.d[3] == in[2].dims.d[3]);
    MHA_CHECK(in[0].dims.d[3] == out[0].dims.d[3]);

    MHA_CHECK(in[0].type == MHA_HD64_DT_FLOAT || in[0].type == MHA_HD64_DT_HALF);
    MHA_CHECK(in[1].type == in[0].type);
    MHA_CHECK(in[2].type == in[0].type);
    MHA_CHECK(out[0].type == in[0].type);

    MHA_CHECK(in[0].format == MHA_HD64_FMT_LINEAR);
    MHA_CHECK(in[1].format == MHA_HD64_FMT_LINEAR);
    MHA_CHECK(in[2].format == MHA_HD64_FMT_LINEAR);
    MHA_CHECK(out[0].format == MHA_HD64_FMT_LINEAR);
    // A softmax over zero keys is undefined (NaN in the PyTorch oracle); refuse it explicitly.
    MHA_CHECK(in[0].dims.d[2] == 0 || in[1].dims.d[2] >= 1);
    return MHA_HD64_STATUS_SUCCESS;
}

int32_t launch_status(hipError_t e, const char* file, int line) {
    if (e == hipSuccess) return MHA_HD64_STATUS_SUCCESS;
    char buf[256];
    std::snprintf(buf, sizeof(buf), "kernel launch failed: %s", hipGetErrorString(e));
    return fail(MHA_HD64_STATUS_LAUNCH_FAILED, file, line, buf);
}

int32_t run_launcher(const void* q, const void* k, const void* v, void* o, int32_t batch, int32_t heads,
                     int32_t nq, int32_t nkv, void* ws, size_t ws_bytes, hipStream_t stream,
                     mha_hd64::InType in, mha_hd64::OutType out) {
    MHA_CHECK(batch >= 0 && heads >= 0 && nq >= 0 && nkv >= 0);
    if (batch == 0 || heads == 0 || nq == 0) return MHA_HD64_STATUS_SUCCESS;
    MHA_CHECK(nkv >= 1);
    MHA_CHECK(q != nullptr && k != nullptr && v != nullptr && o != nullptr);
    MHA_CHECK(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16 == 0);
    const mha_hd64::Call c{q, k, v, o, batch, heads, nq, nkv};
    return launch_status(mha_hd64::launch_attention(c, in, out, ws, ws_bytes, stream), __FILE__, __LINE__);
}

}  // namespace

// The plugin object. Same members/methods as nvinfer1::plugin::LightGlueAttentionPlugin.
struct mha_hd64_plugin {
    std::string plugin_namespace;

    int32_t initialize() { return 0; }
    void terminate() {}
    size_t getSerializationSize() const { return 0; }
    void serialize(void*) const {}
    const char* getPluginType() const { return kPluginName; }
    const char* getPluginVersion() const { return kPluginVersion; }
    void setPluginNamespace(const char* ns) { plugin_namespace = ns ? ns : ""; }
    const char* getPluginNamespace() const { return plugin_namespace.c_str(); }
    int32_t getNbOutputs() const { return 1; }

    int32_t getOutputDimensions(int32_t output_index, const mha_hd64_dims_t* inputs, int32_t nb_inputs,
                                mha_hd64_dims_t* out) {
        MHA_CHECK(inputs != nullptr && out != nullptr && nb_inputs == 3 && output_index == 0);
        MHA_CHECK(inputs[0].nb_dims == 4 && inputs[1].nb_dims == 4 && inputs[2].nb_dims == 4);
        *out = inputs[0];
        return MHA_HD64_STATUS_SUCCESS;
    }

    size_t getWorkspaceSize(const mha_hd64_tensor_desc_t* in, int32_t nb_inputs,
                            const mha_hd64_tensor_desc_t* out, int32_t nb_outputs) const {
        if (!(in != nullptr && out != nullptr && nb_inputs == 3 && nb_outputs == 1)) {
            fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__,
                 "assertion failed: in != nullptr && out != nullptr && nb_inputs == 3 && nb_outputs == 1");
            return 0;
        }
        return kWorkspaceBytes;
    }

    int32_t supportsFormatCombination(int32_t pos, const mha_hd64_tensor_desc_t* io, int32_t nb_inputs,
                                      int32_t nb_outputs) {
        if (!(io != nullptr && nb_inputs == 3 && nb_outputs == 1 && pos >= 0 && pos <= 3)) {
            fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__, "assertion failed: supportsFormatCombination arguments");
            return -1;
        }
        if (pos == 0)
            return (io[0].type == MHA_HD64_DT_FLOAT || io[0].type == MHA_HD64_DT_HALF) &&
                   io[0].format == MHA_HD64_FMT_LINEAR;
        return io[pos].type == io[0].type && io[pos].format == MHA_HD64_FMT_LINEAR;
    }

    int32_t getOutputDataType(int32_t output_index, const int32_t* inputs_type, int32_t nb_inputs,
                              int32_t* out_type) const {
        MHA_CHECK(inputs_type != nullptr && out_type != nullptr && nb_inputs == 3 && output_index == 0);
        *out_type = inputs_type[0];
        return MHA_HD64_STATUS_SUCCESS;
    }

    int32_t configurePlugin(const mha_hd64_dynamic_tensor_desc_t* in, int32_t nb_inputs,
                            const mha_hd64_dynamic_tensor_desc_t* out, int32_t nb_outputs) {
        MHA_CHECK(in != nullptr && out != nullptr && nb_inputs == 3 && nb_outputs == 1);
        const mha_hd64_tensor_desc_t ins[3] = {in[0].desc, in[1].desc, in[2].desc};
        const mha_hd64_tensor_desc_t outs[1] = {out[0].desc};
        return validate(ins, outs);
    }

    int32_t enqueue(const mha_hd64_tensor_desc_t* in, const mha_hd64_tensor_desc_t* out,
                    const void* const* inputs, void* const* outputs, void* workspace, hipStream_t stream) {
        MHA_CHECK(in != nullptr && out != nullptr && inputs != nullptr && outputs != nullptr &&
                  workspace != nullptr);
        const int32_t st = validate(in, out);
        if (st != MHA_HD64_STATUS_SUCCESS) return st;
        const int nq = (int)in[0].dims.d[2];
        const int nkv = (int)in[1].dims.d[2];
        if (in[0].type == MHA_HD64_DT_HALF)
            return run_launcher(inputs[0], inputs[1], inputs[2], outputs[0], MHA_HD64_BATCH, MHA_HD64_NUM_HEADS,
                                nq, nkv, workspace, kWorkspaceBytes, stream, mha_hd64::InType::F16,
                                mha_hd64::OutType::F16);
        return run_launcher(inputs[0], inputs[1], inputs[2], outputs[0], MHA_HD64_BATCH, MHA_HD64_NUM_HEADS, nq,
                            nkv, workspace, kWorkspaceBytes, stream, mha_hd64::InType::F32, mha_hd64::OutType::F32);
    }
};

extern "C" {

// ---- creator ----
const char* mha_hd64_creator_plugin_name(void) { return kPluginName; }
const char* mha_hd64_creator_plugin_version(void) { return kPluginVersion; }
int32_t mha_hd64_creator_nb_fields(void) { return 0; }

mha_hd64_plugin_t* mha_hd64_create_plugin(const char* /*name*/) {
    try {
        auto* p = new mha_hd64_plugin();
        p->initialize();
        return p;
    } catch (const std::exception& e) {
        fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__, e.what());
    }
    return nullptr;
}

mha_hd64_plugin_t* mha_hd64_deserialize_plugin(const char* name, const void* /*data*/, size_t /*length*/) {
    return mha_hd64_create_plugin(name);
}

// ---- plugin ----
void mha_hd64_destroy(mha_hd64_plugin_t* p) { delete p; }

mha_hd64_plugin_t* mha_hd64_clone(const mha_hd64_plugin_t* p) {
    if (p == nullptr) return nullptr;
    try {
        auto* c = new mha_hd64_plugin();
        c->setPluginNamespace(p->getPluginNamespace());
        c->initialize();
        return c;
    } catch (const std::exception& e) {
        fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__, e.what());
    }
    return nullptr;
}

int32_t mha_hd64_initialize(mha_hd64_plugin_t* p) { return p ? p->initialize() : MHA_HD64_STATUS_BAD_PARAM; }
void mha_hd64_terminate(mha_hd64_plugin_t* p) { if (p) p->terminate(); }
size_t mha_hd64_get_serialization_size(const mha_hd64_plugin_t* p) { return p ? p->getSerializationSize() : 0; }
void mha_hd64_serialize(const mha_hd64_plugin_t* p, void* buffer) { if (p) p->serialize(buffer); }
const char* mha_hd64_get_plugin_type(const mha_hd64_plugin_t* p) { return p ? p->getPluginType() : kPluginName; }
const char* mha_hd64_get_plugin_version(const mha_hd64_plugin_t* p) {
    return p ? p->getPluginVersion() : kPluginVersion;
}
void mha_hd64_set_plugin_namespace(mha_hd64_plugin_t* p, const char* ns) { if (p) p->setPluginNamespace(ns); }
const char* mha_hd64_get_plugin_namespace(const mha_hd64_plugin_t* p) { return p ? p->getPluginNamespace() : ""; }
void mha_hd64_attach_to_context(mha_hd64_plugin_t*) {}
void mha_hd64_detach_from_context(mha_hd64_plugin_t*) {}
int32_t mha_hd64_get_nb_outputs(const mha_hd64_plugin_t* p) { return p ? p->getNbOutputs() : 1; }

int32_t mha_hd64_get_output_dimensions(mha_hd64_plugin_t* p, int32_t output_index, const mha_hd64_dims_t* inputs,
                                       int32_t nb_inputs, mha_hd64_dims_t* out) {
    MHA_CHECK(p != nullptr);
    return p->getOutputDimensions(output_index, inputs, nb_inputs, out);
}

int32_t mha_hd64_supports_format_combination(mha_hd64_plugin_t* p, int32_t pos, const mha_hd64_tensor_desc_t* io,
                                             int32_t nb_inputs, int32_t nb_outputs) {
    if (p == nullptr) return -1;
    return p->supportsFormatCombination(pos, io, nb_inputs, nb_outputs);
}

int32_t mha_hd64_get_output_data_type(const mha_hd64_plugin_t* p, int32_t output_index, const int32_t* inputs_type,
                                      int32_t nb_inputs, int32_t* out_type) {
    MHA_CHECK(p != nullptr);
    return p->getOutputDataType(output_index, inputs_type, nb_inputs, out_type);
}

int32_t mha_hd64_configure_plugin(mha_hd64_plugin_t* p, const mha_hd64_dynamic_tensor_desc_t* in, int32_t nb_inputs,
                                  const mha_hd64_dynamic_tensor_desc_t* out, int32_t nb_outputs) {
    MHA_CHECK(p != nullptr);
    return p->configurePlugin(in, nb_inputs, out, nb_outputs);
}

size_t mha_hd64_get_workspace_size(const mha_hd64_plugin_t* p, const mha_hd64_tensor_desc_t* in, int32_t nb_inputs,
                                   const mha_hd64_tensor_desc_t* out, int32_t nb_outputs) {
    if (p == nullptr) return 0;
    return p->getWorkspaceSize(in, nb_inputs, out, nb_outputs);
}

int32_t mha_hd64_enqueue(mha_hd64_plugin_t* p, const mha_hd64_tensor_desc_t* in, const mha_hd64_tensor_desc_t* out,
                         const void* const* inputs, void* const* outputs, void* workspace, hipStream_t stream) {
    MHA_CHECK(p != nullptr);
    return p->enqueue(in, out, inputs, outputs, workspace, stream);
}

// ---- L0 launchers ----
int32_t mha_hd64_launch_fp16in_fp16out(const void* q, const void* k, const void* v, void* o, int32_t batch,
                                       int32_t heads, int32_t nq, int32_t nkv, void* workspace, size_t ws_bytes,
                                       hipStream_t stream) {
    return run_launcher(q, k, v, o, batch, heads, nq, nkv, workspace, ws_bytes, stream, mha_hd64::InType::F16,
                        mha_hd64::OutType::F16);
}

int32_t mha_hd64_launch_fp16in_fp32out(const void* q, const void* k, const void* v, void* o, int32_t batch,
                                       int32_t heads, int32_t nq, int32_t nkv, void* workspace, size_t ws_bytes,
                                       hipStream_t stream) {
    return run_launcher(q, k, v, o, batch, heads, nq, nkv, workspace, ws_bytes, stream, mha_hd64::InType::F16,
                        mha_hd64::OutType::F32);
}

int32_t mha_hd64_launch_fp32in_fp32out(const void* q, const void* k, const void* v, void* o, int32_t batch,
                                       int32_t heads, int32_t nq, int32_t nkv, void* workspace, size_t ws_bytes,
                                       hipStream_t stream) {
    return run_launcher(q, k, v, o, batch, heads, nq, nkv, workspace, ws_bytes, stream, mha_hd64::InType::F32,
                        mha_hd64::OutType::F32);
}

size_t mha_hd64_launch_workspace_bytes(int32_t batch, int32_t heads, int32_t nq, int32_t nkv) {
    if (batch <= 0 || heads <= 0 || nq <= 0 || nkv <= 0) return 0;
    const mha_hd64::Call c{nullptr, nullptr, nullptr, nullptr, batch, heads, nq, nkv};
    // Plan with an unbounded workspace to learn what the preferred split needs.
    return mha_hd64::plan_call(c, (size_t)-1).ws_needed;
}

size_t mha_hd64_launch_workspace_bytes_typed(int32_t batch, int32_t heads, int32_t nq, int32_t nkv, int32_t in_type) {
    if (in_type != MHA_HD64_DT_HALF && in_type != MHA_HD64_DT_FLOAT) return 0;
    if (batch <= 0 || heads <= 0 || nq <= 0 || nkv <= 0) return 0;
    const mha_hd64::Call c{nullptr, nullptr, nullptr, nullptr, batch, heads, nq, nkv};
    return mha_hd64::group_workspace_bytes(&c, 1, in_type == MHA_HD64_DT_FLOAT ? mha_hd64::InType::F32
                                                                              : mha_hd64::InType::F16);
}

// ---- grouped launcher ----
static int32_t to_calls(const mha_hd64_call_t* calls, int32_t n, std::vector<mha_hd64::Call>& out) {
    MHA_CHECK(n >= 0 && (n == 0 || calls != nullptr));
    out.clear();
    for (int32_t i = 0; i < n; ++i) {
        const mha_hd64_call_t& c = calls[i];
        MHA_CHECK(c.batch >= 0 && c.heads >= 0 && c.nq >= 0 && c.nkv >= 0);
        if (c.batch == 0 || c.heads == 0 || c.nq == 0) continue;
        MHA_CHECK(c.nkv >= 1);
        MHA_CHECK(c.q != nullptr && c.k != nullptr && c.v != nullptr && c.o != nullptr);
        MHA_CHECK(((uintptr_t)c.q | (uintptr_t)c.k | (uintptr_t)c.v | (uintptr_t)c.o) % 16 == 0);
        out.push_back(mha_hd64::Call{c.q, c.k, c.v, c.o, c.batch, c.heads, c.nq, c.nkv});
    }
    return MHA_HD64_STATUS_SUCCESS;
}

int32_t mha_hd64_launch_grouped(const mha_hd64_call_t* calls, int32_t n_calls, int32_t in_type, int32_t out_type,
                                void* workspace, size_t ws_bytes, hipStream_t stream) {
    MHA_CHECK(in_type == MHA_HD64_DT_HALF || in_type == MHA_HD64_DT_FLOAT);
    MHA_CHECK(out_type == MHA_HD64_DT_HALF || out_type == MHA_HD64_DT_FLOAT);
    std::vector<mha_hd64::Call> v;
    const int32_t st = to_calls(calls, n_calls, v);
    if (st != MHA_HD64_STATUS_SUCCESS || v.empty()) return st;
    return launch_status(
        mha_hd64::launch_group(v.data(), (int)v.size(),
                               in_type == MHA_HD64_DT_HALF ? mha_hd64::InType::F16 : mha_hd64::InType::F32,
                               out_type == MHA_HD64_DT_HALF ? mha_hd64::OutType::F16 : mha_hd64::OutType::F32,
                               workspace, workspace ? ws_bytes : 0, stream),
        __FILE__, __LINE__);
}

size_t mha_hd64_grouped_workspace_bytes(const mha_hd64_call_t* calls, int32_t n_calls) {
    return mha_hd64_grouped_workspace_bytes_typed(calls, n_calls, MHA_HD64_DT_HALF);
}

size_t mha_hd64_grouped_workspace_bytes_typed(const mha_hd64_call_t* calls, int32_t n_calls, int32_t in_type) {
    if (in_type != MHA_HD64_DT_HALF && in_type != MHA_HD64_DT_FLOAT) return 0;
    std::vector<mha_hd64::Call> v;
    if (to_calls(calls, n_calls, v) != MHA_HD64_STATUS_SUCCESS || v.empty()) return 0;
    return mha_hd64::group_workspace_bytes(v.data(), (int)v.size(),
                                           in_type == MHA_HD64_DT_FLOAT ? mha_hd64::InType::F32
                                                                        : mha_hd64::InType::F16);
}

// ---- diagnostics ----
const char* mha_hd64_last_error(void) { return g_last_error.c_str(); }
void mha_hd64_set_abort_on_error(int32_t enable) { g_abort_on_error = enable != 0; }
int32_t mha_hd64_set_concurrency_hint(int32_t streams) { return mha_hd64::set_concurrency_hint(streams); }
const char* mha_hd64_build_info(void) {
    return "mha_hd64: gfx950 (CDNA4) HIP kernels, v_mfma_f32_32x32x16_f16 / 16x16x32_f16 + ds_read_b64_tr_b16; "
           "variants fp16->fp16, fp16->fp32, fp32->fp32; single-pass kernels (16 or 32 rows x all keys per workgroup, "
           "K/V by LDS-DMA, L2 prefetch of late rows; fp32 inputs rounded in the 16-row kernel) "
           "for launches of <= 256 blocks with nkv <= 2048; LDS-ring kernel with workgroups (q,kv waves) 4x1 2x2 1x2 4x2 2x4 1x4 1x8, "
           "2x2 with 64-row waves; software-pipelined QK(t+1)|softmax(t); split-KV combine (in-launch or kernel)";
}

// Test/bench hook (not part of include/mha_hd64.h): launch with a forced plan
// (q_waves/kv_waves/splits 0 = planner's choice); phase_mask 1 = main kernel only, 2 = combine only, 3 = both.
int32_t mha_hd64_launch_forced(const void* q, const void* k, const void* v, void* o, int32_t batch, int32_t heads,
                               int32_t nq, int32_t nkv, int32_t in_f32, int32_t out_f32, int32_t q_waves,
                               int32_t kv_waves, int32_t splits, void* workspace, size_t ws_bytes,
                               hipStream_t stream, int32_t phase_mask) {
    MHA_CHECK(batch >= 0 && heads >= 0 && nq >= 0 && nkv >= 0);
    if (batch == 0 || heads == 0 || nq == 0) return MHA_HD64_STATUS_SUCCESS;
    MHA_CHECK(nkv >= 1);
    const mha_hd64::Call c{q, k, v, o, batch, heads, nq, nkv};
    const mha_hd64::LaunchPlan plan =
        mha_hd64::plan_call(c, workspace ? ws_bytes : 0, q_waves, kv_waves, splits,
                            in_f32 ? mha_hd64::InType::F32 : mha_hd64::InType::F16);
    const int plan_qw = plan.stream ? mha_hd64::kForceStream
                        : plan.direct_tiles > 0
                            ? (plan.rows_per_wave == 16 ? mha_hd64::kForceDirect16 : mha_hd64::kForceDirect)
                            : plan.q_waves + (plan.rows_per_wave == 64 ? 10 : 0);
    // (2,4), (1,4), (1,8) take one split per super-tile and fall back to (2,2) past 16 of them
    const bool single_tile = kv_waves >= 4;
    const bool fell_back = single_tile && plan_qw == 2 && plan.kv_waves == 2;
    // q_waves = 21 / 22 force the 32- / 16-row single-pass kernel (kv_waves / splits ignored)
    // q_waves = 23 forces the persistent streaming kernel (fp16 input)
    const bool direct = q_waves == mha_hd64::kForceDirect || q_waves == mha_hd64::kForceDirect16 ||
                        q_waves == mha_hd64::kForceStream;
    if (direct && plan_qw != q_waves)
        return fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__,
                    "single-pass / streaming kernel: fp16 input, nkv <= 1024 (16-row) / 2048 (32-row)");
    if (q_waves != 0 && !direct && !fell_back && (plan_qw != q_waves || plan.kv_waves != kv_waves))
        return fail(MHA_HD64_STATUS_BAD_PARAM, __FILE__, __LINE__, "forced workgroup shape is not compiled");
    if (splits > 1 && !single_tile && !direct && plan.splits != splits)
        return fail(MHA_HD64_STATUS_WORKSPACE, __FILE__, __LINE__, "forced split does not fit the workspace/keys");
    return launch_status(mha_hd64::launch_attention(c, in_f32 ? mha_hd64::InType::F32 : mha_hd64::InType::F16,
                                                    out_f32 ? mha_hd64::OutType::F32 : mha_hd64::OutType::F16,
                                                    workspace, ws_bytes, stream, q_waves, kv_waves, splits,
                                                    phase_mask),
                         __FILE__, __LINE__);
}

// Diagnostic hook: per-workgroup timestamp buffer for -DMHA_STAMPS builds (ignored otherwise).
void mha_hd64_set_stamp_buffer(void* p) { mha_hd64::set_stamp_buffer(p); }

// Test/bench hook: 1 = split calls combine inside the main launch (default), 0 = combine kernel.
void mha_hd64_set_fused_combine(int32_t enable) { mha_hd64::set_fused_combine(enable); }
// Test/bench hook: fp32 Q/K/V rounded to fp16 inside the 16-row kernel (1, default where it
// applies) or by a separate convert launch before the fp16 kernel (0); results are bitwise equal.
void mha_hd64_set_f32_inkernel(int32_t enable) { mha_hd64::set_f32_inkernel(enable); }
// 1 = the persistent streaming kernel for fp16 launches of > 256 128-row blocks (default),
// 0 = never (MHA_HD64_STREAM=0 sets 0 at first use). Returns the previous mode.
int32_t mha_hd64_set_stream_mode(int32_t mode) { return mha_hd64::set_stream_mode(mode); }
// Test hook: 0 = the calling thread's last launch had no split, 1 = in-launch combine, 2 = combine kernel.
int32_t mha_hd64_last_combine_form(void) { return mha_hd64::last_combine_form(); }

// Plan query hook for tests/bench: fills {q_waves, kv_waves, splits, tiles_per_split}; returns workspace bytes.
size_t mha_hd64_plan(int32_t batch, int32_t heads, int32_t nq, int32_t nkv, size_t ws_bytes, int32_t* out4) {
    const mha_hd64::Call c{nullptr, nullptr, nullptr, nullptr, batch, heads, nq, nkv};
    const mha_hd64::LaunchPlan p = mha_hd64::plan_call(c, ws_bytes);
    if (out4) {
        out4[0] = p.stream ? mha_hd64::kForceStream
                  : p.direct_tiles > 0 ? (p.rows_per_wave == 16 ? mha_hd64::kForceDirect16 : mha_hd64::kForceDirect)
                                       : p.q_waves + (p.rows_per_wave == 64 ? 10 : 0);
        out4[1] = p.kv_waves;
        out4[2] = p.splits;
        out4[3] = p.tiles_per_split;
    }
    return p.ws_needed;
}

}  // extern "C"

namespace mha_hd64 {
int32_t report_error(int32_t status, const char* where, const char* what) {
    char buf[256];
    std::snprintf(buf, sizeof(buf), "%s: %s", where, what);
    return fail(status, __FILE__, __LINE__, buf);
}
}  // namespace mha_hd64
