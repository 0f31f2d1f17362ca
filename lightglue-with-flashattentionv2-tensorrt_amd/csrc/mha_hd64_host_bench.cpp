// mha_hd64_host_bench — a C++ host over the C ABI only (include/mha_hd64.h; no Python, no torch).
//
// It plays the reference's TensorRT host role for this path: LightGlueTRT dlopens the plugin
// library, the engine calls configurePlugin / getWorkspaceSize / enqueue, and the demo captures
// enqueueV3 into a CUDA graph (demo/lightglue_trt.cpp:15, 283-285, 347-366). Here: create the
// "MHAHeadDim64" plugin through the creator, configure it for Q/K/V [1,4,Nq|Nkv,64], check one
// eager enqueue against a double-precision CPU attention on sampled rows (tolerance 1e-2, the
// north_star bar), then capture `steps` enqueues into a hipGraph and time its replay with HIP
// events. Prints one JSON line.
//
//   lib/mha_hd64_host_bench [--nq N] [--nkv N] [--steps K] [--float]
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mha_hd64.h"

#define HIP_OK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

static void plugin_ok(int32_t st, const char* what) {
    if (st != MHA_HD64_STATUS_SUCCESS) {
        std::fprintf(stderr, "%s failed (%d): %s\n", what, st, mha_hd64_last_error());
        std::exit(3);
    }
}

// splitmix64 -> uniform in [-2, 2): deterministic inputs with logits of order 1 after the 1/8 scale
static uint64_t g_state = 0x4C47;
static float next_value() {
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)((z >> 40) * (1.0 / 16777216.0)) * 4.f - 2.f;
}

static mha_hd64_dims_t dims4(int64_t n) {
    mha_hd64_dims_t d{};
    d.nb_dims = 4;
    d.d[0] = MHA_HD64_BATCH;
    d.d[1] = MHA_HD64_NUM_HEADS;
    d.d[2] = n;
    d.d[3] = MHA_HD64_HEAD_DIM;
    return d;
}

int main(int argc, char** argv) {
    int nq = 1024, nkv = 1024, steps = 2000;
    bool use_float = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--nq") && i + 1 < argc) nq = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--nkv") && i + 1 < argc) nkv = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--steps") && i + 1 < argc) steps = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--float")) use_float = true;
    }
    const int H = MHA_HD64_NUM_HEADS, D = MHA_HD64_HEAD_DIM;
    const int32_t dt = use_float ? MHA_HD64_DT_FLOAT : MHA_HD64_DT_HALF;
    const size_t esz = use_float ? 4 : 2;

    // inputs (the Half path sees fp16-rounded values; the reference below uses the same values)
    std::vector<float> hq((size_t)H * nq * D), hk((size_t)H * nkv * D), hv((size_t)H * nkv * D);
    for (auto* v : {&hq, &hk, &hv})
        for (float& x : *v) x = use_float ? next_value() : __half2float(__float2half(next_value()));
    auto upload = [&](const std::vector<float>& h) {
        void* d = nullptr;
        HIP_OK(hipMalloc(&d, h.size() * esz));
        if (use_float) {
            HIP_OK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        } else {
            std::vector<__half> t(h.size());
            for (size_t i = 0; i < h.size(); ++i) t[i] = __float2half(h[i]);
            HIP_OK(hipMemcpy(d, t.data(), t.size() * 2, hipMemcpyHostToDevice));
        }
        return d;
    };
    void* dq = upload(hq);
    void* dk = upload(hk);
    void* dv = upload(hv);
    void* dout = nullptr;
    HIP_OK(hipMalloc(&dout, (size_t)H * nq * D * esz));

    // plugin lifecycle as the engine drives it
    mha_hd64_plugin_t* p = mha_hd64_create_plugin("MHAHeadDim64");
    if (!p) plugin_ok(MHA_HD64_STATUS_BAD_PARAM, "create_plugin");
    plugin_ok(mha_hd64_initialize(p), "initialize");
    mha_hd64_tensor_desc_t in[3], out[1];
    const int64_t ns[3] = {nq, nkv, nkv};
    for (int i = 0; i < 3; ++i) in[i] = mha_hd64_tensor_desc_t{dims4(ns[i]), dt, MHA_HD64_FMT_LINEAR, 1.f};
    out[0] = mha_hd64_tensor_desc_t{dims4(nq), dt, MHA_HD64_FMT_LINEAR, 1.f};
    mha_hd64_dynamic_tensor_desc_t din[3], dout_desc[1];
    for (int i = 0; i < 3; ++i) din[i] = mha_hd64_dynamic_tensor_desc_t{in[i], in[i].dims, in[i].dims};
    dout_desc[0] = mha_hd64_dynamic_tensor_desc_t{out[0], out[0].dims, out[0].dims};
    plugin_ok(mha_hd64_configure_plugin(p, din, 3, dout_desc, 1), "configure_plugin");
    const size_t ws_bytes = mha_hd64_get_workspace_size(p, in, 3, out, 1);
    void* ws = nullptr;
    HIP_OK(hipMalloc(&ws, ws_bytes));
    hipStream_t stream;
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const void* inputs[3] = {dq, dk, dv};
    void* outputs[1] = {dout};

    // one eager enqueue (also warms this stream's in-launch-combine tickets before capture)
    plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    HIP_OK(hipStreamSynchronize(stream));
    std::vector<float> ho((size_t)H * nq * D);
    if (use_float) {
        HIP_OK(hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost));
    } else {
        std::vector<__half> t(ho.size());
        HIP_OK(hipMemcpy(t.data(), dout, t.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < t.size(); ++i) ho[i] = __half2float(t[i]);
    }
    // double-precision reference (lightglue_pytorch_no_plugin/lightglue.py:82-84) on sampled rows
    double max_err = 0.0;
    std::vector<double> s(nkv);
    for (int h = 0; h < H; ++h)
        for (int r = 0; r < nq; r += std::max(1, nq / 16)) {
            const float* qr = &hq[((size_t)h * nq + r) * D];
            double m = -INFINITY, l = 0.0;
            for (int j = 0; j < nkv; ++j) {
                const float* kr = &hk[((size_t)h * nkv + j) * D];
                double dot = 0.0;
                for (int d = 0; d < D; ++d) dot += (double)qr[d] * kr[d];
                s[j] = dot / 8.0;
                m = std::max(m, s[j]);
            }
            for (int j = 0; j < nkv; ++j) l += (s[j] = std::exp(s[j] - m));
            for (int d = 0; d < D; ++d) {
                double o = 0.0;
                for (int j = 0; j < nkv; ++j) o += s[j] * hv[((size_t)h * nkv + j) * D + d];
                max_err = std::max(max_err, std::fabs(o / l - ho[((size_t)h * nq + r) * D + d]));
            }
        }

    // `steps` enqueues captured into one graph, replayed between events
    for (int i = 0; i < 20; ++i) plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    hipGraph_t graph;
    hipGraphExec_t exec;
    HIP_OK(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal));
    for (int i = 0; i < steps; ++i) plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    HIP_OK(hipStreamEndCapture(stream, &graph));
    HIP_OK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    HIP_OK(hipGraphLaunch(exec, stream));  // upload / first replay outside the timer
    HIP_OK(hipStreamSynchronize(stream));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, stream));
    HIP_OK(hipGraphLaunch(exec, stream));
    HIP_OK(hipEventRecord(e1, stream));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / steps;
    std::printf("{\"host\": \"c++ (C ABI only)\", \"dtype\": \"%s\", \"nq\": %d, \"nkv\": %d, \"steps\": %d, "
                "\"us_per_call\": %.3f, \"calls_per_s\": %.1f, \"max_abs_err_sampled_rows\": %.3e, \"tolerance\": 1e-2}\n",
                use_float ? "fp32" : "fp16", nq, nkv, steps, us, 1e6 / us, max_err);
    HIP_OK(hipGraphExecDestroy(exec));
    HIP_OK(hipGraphDestroy(graph));
    mha_hd64_terminate(p);
    mha_hd64_destroy(p);
    for (void* d : {dq, dk, dv, dout, ws}) HIP_OK(hipFree(const_cast<void*>(d)));
    HIP_OK(hipStreamDestroy(stream));
    return max_err <= 1e-2 ? 0 : 1;
}
