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
//   lib/mha_hd64_host_bench [--nq N] [--nkv N] [--steps K] [--float] [--devices D] [--streams S]
//
// --devices D --streams S: D x S host threads, S per device (hipSetDevice), each with its own plugin,
// stream, workspace and buffers, all replaying at once; outputs must agree bit for bit across them.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <algorithm>
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

// Simple reusable barrier (C++17): the workers start their timed replays together.
class Barrier {
   public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        const int gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen != gen_; });
        }
    }

   private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0, gen_ = 0;
};

struct Config {
    int nq = 1024, nkv = 1024, steps = 2000;
    bool use_float = false;
};

// One host thread per (device, stream): hipSetDevice, its own plugin instance, stream, workspace
// and Q/K/V/O (a pair stream per GPU; the per-enqueue workspace rule of
// lightglue_attention_plugin.cpp:172-175). Every worker uploads the same inputs, so every
// worker's output must be bitwise identical to every other's.
struct Worker {
    int device = 0, index = 0;
    double us = 0.0, max_err = 0.0;
    std::vector<uint16_t> out_bits;  // raw output bytes (fp16) or halves of fp32 words
    std::string error;
};

static void run_worker(Worker& w, const Config& cfg, const std::vector<float>& hq, const std::vector<float>& hk,
                       const std::vector<float>& hv, Barrier& bar) {
    const int H = MHA_HD64_NUM_HEADS, D = MHA_HD64_HEAD_DIM;
    const int nq = cfg.nq, nkv = cfg.nkv;
    const bool use_float = cfg.use_float;
    const int32_t dt = use_float ? MHA_HD64_DT_FLOAT : MHA_HD64_DT_HALF;
    const size_t esz = use_float ? 4 : 2;
    HIP_OK(hipSetDevice(w.device));
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
    const size_t out_bytes = (size_t)H * nq * D * esz;
    HIP_OK(hipMalloc(&dout, out_bytes));

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
    HIP_OK(hipMemset(dout, 0xFF, out_bytes));
    plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    HIP_OK(hipStreamSynchronize(stream));
    w.out_bits.resize(out_bytes / 2);
    HIP_OK(hipMemcpy(w.out_bits.data(), dout, out_bytes, hipMemcpyDeviceToHost));
    std::vector<float> ho((size_t)H * nq * D);
    if (use_float) {
        std::memcpy(ho.data(), w.out_bits.data(), out_bytes);
    } else {
        for (size_t i = 0; i < ho.size(); ++i) {
            __half_raw r;
            r.x = w.out_bits[i];
            ho[i] = __half2float(__half(r));
        }
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
    w.max_err = max_err;

    // `steps` enqueues captured into one graph, replayed between events; the workers' replays start together
    for (int i = 0; i < 20; ++i) plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    hipGraph_t graph;
    hipGraphExec_t exec;
    HIP_OK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < cfg.steps; ++i)
        plugin_ok(mha_hd64_enqueue(p, in, out, inputs, outputs, ws, stream), "enqueue");
    HIP_OK(hipStreamEndCapture(stream, &graph));
    HIP_OK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    HIP_OK(hipGraphLaunch(exec, stream));  // upload / first replay outside the timer
    HIP_OK(hipStreamSynchronize(stream));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    bar.wait();
    HIP_OK(hipEventRecord(e0, stream));
    HIP_OK(hipGraphLaunch(exec, stream));
    HIP_OK(hipEventRecord(e1, stream));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    w.us = 1e3 * ms / cfg.steps;
    // the graph's output equals the eager one (same inputs, deterministic kernels)
    std::vector<uint16_t> again(out_bytes / 2);
    HIP_OK(hipMemcpy(again.data(), dout, out_bytes, hipMemcpyDeviceToHost));
    if (again != w.out_bits) w.error = "graph replay output differs from the eager enqueue";
    HIP_OK(hipEventDestroy(e0));
    HIP_OK(hipEventDestroy(e1));
    HIP_OK(hipGraphExecDestroy(exec));
    HIP_OK(hipGraphDestroy(graph));
    mha_hd64_terminate(p);
    mha_hd64_destroy(p);
    for (void* d : {dq, dk, dv, dout, ws}) HIP_OK(hipFree(const_cast<void*>(d)));
    HIP_OK(hipStreamDestroy(stream));
}

int main(int argc, char** argv) {
    Config cfg;
    int devices = 1, streams = 1;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--nq") && i + 1 < argc) cfg.nq = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--nkv") && i + 1 < argc) cfg.nkv = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--steps") && i + 1 < argc) cfg.steps = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) devices = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--streams") && i + 1 < argc) streams = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--float")) cfg.use_float = true;
    }
    int visible = 0;
    HIP_OK(hipGetDeviceCount(&visible));
    if (devices < 1 || streams < 1 || devices > visible) {
        std::fprintf(stderr, "--devices %d --streams %d: %d GPU(s) visible\n", devices, streams, visible);
        return 2;
    }
    const int H = MHA_HD64_NUM_HEADS, D = MHA_HD64_HEAD_DIM;
    // inputs (the Half path sees fp16-rounded values; the reference below uses the same values)
    std::vector<float> hq((size_t)H * cfg.nq * D), hk((size_t)H * cfg.nkv * D), hv((size_t)H * cfg.nkv * D);
    for (auto* v : {&hq, &hk, &hv})
        for (float& x : *v) x = cfg.use_float ? next_value() : __half2float(__float2half(next_value()));

    std::vector<Worker> workers(devices * streams);
    Barrier bar((int)workers.size());
    std::vector<std::thread> threads;
    for (int i = 0; i < (int)workers.size(); ++i) {
        workers[i].device = i / streams;
        workers[i].index = i;
        threads.emplace_back(run_worker, std::ref(workers[i]), std::cref(cfg), std::cref(hq), std::cref(hk),
                             std::cref(hv), std::ref(bar));
    }
    for (auto& t : threads) t.join();

    double max_err = 0.0, calls_per_s = 0.0;
    bool identical = true, ok = true;
    std::string per;
    for (const Worker& w : workers) {
        max_err = std::max(max_err, w.max_err);
        calls_per_s += 1e6 / w.us;
        identical = identical && w.out_bits == workers[0].out_bits;
        if (!w.error.empty()) {
            std::fprintf(stderr, "worker %d (device %d): %s\n", w.index, w.device, w.error.c_str());
            ok = false;
        }
        char buf[96];
        std::snprintf(buf, sizeof buf, "%s{\"device\": %d, \"us_per_call\": %.3f}", per.empty() ? "" : ", ",
                      w.device, w.us);
        per += buf;
    }
    std::printf("{\"host\": \"c++ (C ABI only)\", \"dtype\": \"%s\", \"nq\": %d, \"nkv\": %d, \"steps\": %d, "
                "\"devices\": %d, \"streams_per_device\": %d, \"us_per_call\": %.3f, \"calls_per_s\": %.1f, "
                "\"calls_per_s_all_workers\": %.1f, \"workers\": [%s], \"outputs_bitwise_identical\": %s, "
                "\"max_abs_err_sampled_rows\": %.3e, \"tolerance\": 1e-2}\n",
                cfg.use_float ? "fp32" : "fp16", cfg.nq, cfg.nkv, cfg.steps, devices, streams, workers[0].us,
                1e6 / workers[0].us, calls_per_s, per.c_str(), identical ? "true" : "false", max_err);
    return (max_err <= 1e-2 && identical && ok) ? 0 : 1;
}
