// lightglue_glue.hip — gfx950 kernels for the matcher around MHAHeadDim64 (include/lightglue_glue.h).
//
// Memory-bound layout/normalisation kernels: one pass over the data each, 16-B accesses where the
// layout allows, one wave64 per row for row statistics (shuffle-xor reductions), fp32 math.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lightglue_glue.h"
#include "mha_hd64.h"
#include "mha_hd64_internal.h"

namespace {

typedef _Float16 f16;

template <typename T> __device__ __forceinline__ float ld(const T* p) { return (float)*p; }
template <typename T> __device__ __forceinline__ void st(T* p, float v) { *p = (T)v; }

constexpr int kD = 64;  // head dim

// Row n of the stacked rows (`pairs` image pairs, pair-major: n0 rows of image 0, then n1 rows of
// image 1) -> which image, and the offset of the row's head-h segment in that image's
// [pairs, heads, ni, 64] tensor. pairs = 1 is the single-pair layout.
struct ImgRow {
    bool first;
    size_t off;
};
__device__ __forceinline__ ImgRow img_row(int n, int n0, int n1, int heads, int h) {
    const int ntot = n0 + n1;
    const int p = n / ntot, l = n - p * ntot;
    const bool first = l < n0;
    const int row = first ? l : l - n0, nn = first ? n0 : n1;
    return {first, (((size_t)p * heads + h) * nn + row) * kD};
}

// ---- q/k/v split + rotary (thread = one (row, head, rotary pair)) ----
template <typename T>
__global__ __launch_bounds__(256) void qkv_rotary_split_kernel(const T* __restrict__ qkv, const T* __restrict__ cosv,
                                                               const T* __restrict__ sinv, int heads, int n0, int n1,
                                                               int rows, T* q0, T* k0, T* v0, T* q1, T* k1, T* v1) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)rows * heads * (kD / 2)) return;
    const int p = idx % (kD / 2);
    const int h = (idx / (kD / 2)) % heads;
    const int n = idx / ((long)(kD / 2) * heads);
    // channels (h*64 + 2p + t)*3 + j, t in {0,1}, j in {q,k,v}: six consecutive values
    const T* src = qkv + (size_t)n * heads * kD * 3 + (size_t)(h * kD + 2 * p) * 3;
    const float q_a = ld(src + 0), k_a = ld(src + 1), v_a = ld(src + 2);
    const float q_b = ld(src + 3), k_b = ld(src + 4), v_b = ld(src + 5);
    const float c = ld(cosv + (size_t)n * kD + 2 * p), s = ld(sinv + (size_t)n * kD + 2 * p);
    const ImgRow ir = img_row(n, n0, n1, heads, h);
    const bool first = ir.first;
    const size_t o = ir.off + 2 * p;
    T* qd = first ? q0 : q1;
    T* kd = first ? k0 : k1;
    T* vd = first ? v0 : v1;
    // (x0, x1) -> (x0 c - x1 s, x1 c + x0 s)   (t*cos + rotate_half(t)*sin)
    st(qd + o, q_a * c - q_b * s);
    st(qd + o + 1, q_b * c + q_a * s);
    st(kd + o, k_a * c - k_b * s);
    st(kd + o + 1, k_b * c + k_a * s);
    st(vd + o, v_a);
    st(vd + o + 1, v_b);
}

// 16-B vector of T
template <typename T> struct V16;
template <> struct V16<f16> { typedef unsigned int type __attribute__((ext_vector_type(4))); static constexpr int n = 8; };
template <> struct V16<float> { typedef unsigned int type __attribute__((ext_vector_type(4))); static constexpr int n = 4; };

// ---- [rows, heads*64] <-> per image [heads, ni, 64] (thread = one 16-B chunk) ----
template <typename T, bool SPLIT>
__global__ __launch_bounds__(256) void heads_kernel(const T* a, const T* b, T* a0, T* a1, T* b0, T* b1, int heads,
                                                    int n0, int n1, int rows, int ld) {
    typedef typename V16<T>::type vec;
    constexpr int E = V16<T>::n;
    constexpr int CH = kD / E;  // chunks per head row
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per = (long)rows * heads * CH;
    if (idx >= (b ? 2 : 1) * per) return;
    const bool second = idx >= per;
    const long i = second ? idx - per : idx;
    const int c = i % CH;
    const int h = (i / CH) % heads;
    const int n = i / ((long)CH * heads);
    const ImgRow ir = img_row(n, n0, n1, heads, h);
    const bool first = ir.first;
    const size_t rows_off = (size_t)n * ld + h * kD + c * E;  // row-major side: row stride ld
    const size_t head_off = ir.off + c * E;
    if (SPLIT) {
        const T* src = second ? b : a;
        T* dst = second ? (first ? b0 : b1) : (first ? a0 : a1);
        *reinterpret_cast<vec*>(dst + head_off) = *reinterpret_cast<const vec*>(src + rows_off);
    } else {  // merge: a = x0, b = x1 (head-major inputs), a0 = out
        const T* src = first ? a : b;
        *reinterpret_cast<vec*>(a0 + rows_off) = *reinterpret_cast<const vec*>(src + head_off);
    }
}

// [x | merge_heads(x0, x1)]: one 16-B chunk of a 2*heads*64-wide output row per thread; the left
// half copies x (the FFN's concatenation, lightglue.py:104/181), the right half gathers the
// head-major attention outputs.
template <typename T>
__global__ __launch_bounds__(256) void merge_cat_kernel(const T* x, const T* x0, const T* x1, T* out, int heads,
                                                        int n0, int n1, int rows) {
    typedef typename V16<T>::type vec;
    constexpr int E = V16<T>::n;
    constexpr int CH = kD / E;
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int half = CH * heads;  // chunks per half row
    if (idx >= (long)rows * 2 * half) return;
    const int cc = idx % (2 * half);
    const int n = idx / (2 * half);
    vec v;
    if (cc < half) {
        v = *reinterpret_cast<const vec*>(x + (size_t)n * heads * kD + cc * E);
    } else {
        const int c2 = cc - half, h = c2 / CH, c = c2 % CH;
        const ImgRow ir = img_row(n, n0, n1, heads, h);
        v = *reinterpret_cast<const vec*>((ir.first ? x0 : x1) + ir.off + c * E);
    }
    *reinterpret_cast<vec*>(out + (size_t)n * 2 * heads * kD + cc * E) = v;
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = fmaxf(x, __shfl_xor(x, m, 64));
    return x;
}

// ---- LayerNorm + exact GELU (one wave per row, dim / 64 values per lane) ----
template <typename T, int PER>
__global__ __launch_bounds__(256) void ln_gelu_kernel(const T* x, const T* __restrict__ g,
                                                      const T* __restrict__ bta, int rows, float eps, T* y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    constexpr int dim = PER * 64;
    const T* xr = x + (size_t)row * dim;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        v[i] = ld(xr + i * 64 + lane);
        s += v[i];
    }
    const float mean = wave_sum(s) * (1.f / dim);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        v[i] -= mean;
        q += v[i] * v[i];
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.f / dim) + eps);
    T* yr = y + (size_t)row * dim;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = i * 64 + lane;
        const float t = v[i] * rstd * ld(g + c) + ld(bta + c);
        st(yr + c, 0.5f * t * (1.f + erff(t * 0.70710678118654752f)));
    }
}

// Exact (erf) GELU for the fp16 FFN with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far
// below the fp16 rounding of the output), folded: with z = |x| / sqrt(2), r = 1 / (1 + p z) and
// erf(z) = 1 - y(r) e^{-z^2}, x Phi(x) = max(x, 0) - |x| (y / 2) e^{-x^2 / 2} for either sign of x (no
// 1 + erf cancellation for negative x); one v_rcp_f32 and one v_exp_f32, the 1/2 and 1/sqrt(2) in
// the constants. (lightglue_glue.hip and lightglue_linear.hip compute it alike.)
__device__ __forceinline__ float gelu_as(float x) {
    const float ax = fabsf(x);
    const float r = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.f));
    float p = fmaf(0.5f * 1.061405429f, r, 0.5f * -1.453152027f);
    p = fmaf(p, r, 0.5f * 1.421413741f);
    p = fmaf(p, r, 0.5f * -0.284496736f);
    p = fmaf(p, r, 0.5f * 0.254829592f);
    const float w = p * r * ax;
    const float e = __builtin_amdgcn_exp2f(x * x * (-0.5f * 1.4426950408889634f));
    return fmaf(-w, e, fmaxf(x, 0.f));
}
// The same on a pair of values, written on float2 so that the FMAs and products issue as packed
// v_pk_fma_f32 / v_pk_mul_f32 (two values per instruction: the vector pipe's full fp32 rate; the
// rcp, exp, abs and max stay per value)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_as2(f32x2 x) {
    const f32x2 ax = f32x2{fabsf(x[0]), fabsf(x[1])};
    const f32x2 den = ax * (0.3275911f * 0.70710678118654752f) + 1.f;
    const f32x2 r = f32x2{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    f32x2 p = r * (0.5f * 1.061405429f) + (0.5f * -1.453152027f);
    p = p * r + (0.5f * 1.421413741f);
    p = p * r + (0.5f * -0.284496736f);
    p = p * r + (0.5f * 0.254829592f);
    const f32x2 w = p * r * ax;
    const f32x2 a = x * x * (-0.5f * 1.4426950408889634f);
    const f32x2 e = f32x2{__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])};
    return f32x2{fmaxf(x[0], 0.f), fmaxf(x[1], 0.f)} - w * e;
}

// fp16, dim 512 (the matcher's FFN width): a lane owns 8 contiguous columns (one 16-B load of x,
// gamma and beta), sum and sum of squares reduced together (fp32, E[x^2] - mean^2).
__global__ __launch_bounds__(256) void ln_gelu_512_f16_kernel(const f16* x, const f16* __restrict__ g,
                                                              const f16* __restrict__ bta, int rows, float eps,
                                                              f16* y) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const f16x8 xv = *reinterpret_cast<const f16x8*>(x + (size_t)row * 512 + lane * 8);
    const f16x8 gv = *reinterpret_cast<const f16x8*>(g + lane * 8);
    const f16x8 bv = *reinterpret_cast<const f16x8*>(bta + lane * 8);
    float v[8], s = 0.f, q = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        v[e] = (float)xv[e];
        s += v[e];
        q += v[e] * v[e];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {  // two independent shuffle chains
        s += __shfl_xor(s, m, 64);
        q += __shfl_xor(q, m, 64);
    }
    const float mean = s * (1.f / 512);
    const float rstd = rsqrtf(fmaxf(q * (1.f / 512) - mean * mean, 0.f) + eps);
    f16x8 o;
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        const f32x2 t = (f32x2{v[e], v[e + 1]} - mean) * rstd * f32x2{(float)gv[e], (float)gv[e + 1]} +
                        f32x2{(float)bv[e], (float)bv[e + 1]};
        const f32x2 gl = gelu_as2(t);
        o[e] = (f16)gl[0];
        o[e + 1] = (f16)gl[1];
    }
    *reinterpret_cast<f16x8*>(y + (size_t)row * 512 + lane * 8) = o;
}

// A/B build only (SRC=glue tools/build_linear_variant.sh <name> -DLG_LN_FORM=1, tools/ln_ab.py): the
// same operator, persistent: wave w of W walks rows w, w + W, ... with the loads of its next DEPTH
// rows in flight while it computes one, gamma / beta converted once per wave, and GELU as
// max(t, 0) - |t| * (y / 2) * exp(-t^2 / 2) (gelu_as, written out: for t >= 0
// t * Phi(t) = t - t * (y e / 2), for t < 0 it is -|t| * (y e / 2); no 1 + erf cancellation).
// Measured no faster (16.9-19.2 vs 17.0 us at 32,768 rows, profiles/r05/ln_gelu_persistent_ab.jsonl):
// the per-row kernel is vector-issue bound, not latency bound.
#ifndef LG_LN_FORM
#define LG_LN_FORM 0
#endif
#if LG_LN_FORM == 1
#ifndef LG_LN_DEPTH
#define LG_LN_DEPTH 2
#endif
#ifndef LG_LN_BPC
#define LG_LN_BPC 4
#endif
constexpr int kLnDepth = LG_LN_DEPTH;  // rows in flight per wave beyond the one computed
constexpr int kLnBlocksPerCU = LG_LN_BPC;
__global__ __launch_bounds__(256) void ln_gelu_512_rows_kernel(const f16* x, const f16* __restrict__ g,
                                                               const f16* __restrict__ bta, int rows, float eps,
                                                               f16* y) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    const int lane = threadIdx.x & 63;
    const int w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int W = gridDim.x * 4;
    float gf[8], bf[8];
    {
        const f16x8 gv = *reinterpret_cast<const f16x8*>(g + lane * 8);
        const f16x8 bv = *reinterpret_cast<const f16x8*>(bta + lane * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) gf[e] = (float)gv[e], bf[e] = (float)bv[e];
    }
    auto load = [&](int row) {
        return row < rows ? *reinterpret_cast<const f16x8*>(x + (size_t)row * 512 + lane * 8) : f16x8{};
    };
    f16x8 buf[kLnDepth];
#pragma unroll
    for (int d = 0; d < kLnDepth; ++d) buf[d] = load(w0 + d * W);
    for (int base = w0; base < rows; base += kLnDepth * W) {
#pragma unroll
        for (int d = 0; d < kLnDepth; ++d) {
            const int row = base + d * W;
            if (row >= rows) return;
            const f16x8 xv = buf[d];
            buf[d] = load(row + kLnDepth * W);
            float v[8], s = 0.f, q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[e] = (float)xv[e];
                s += v[e];
                q = fmaf(v[e], v[e], q);
            }
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) {
                s += __shfl_xor(s, m, 64);
                q += __shfl_xor(q, m, 64);
            }
            const float mean = s * (1.f / 512);
            const float rstd = rsqrtf(fmaxf(q * (1.f / 512) - mean * mean, 0.f) + eps);
            const float nm = -mean * rstd;
            f16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float t = fmaf(fmaf(v[e], rstd, nm), gf[e], bf[e]);
                const float at = fabsf(t);
                const float r = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, at, 1.f));
                float p = fmaf(0.5f * 1.061405429f, r, 0.5f * -1.453152027f);
                p = fmaf(p, r, 0.5f * 1.421413741f);
                p = fmaf(p, r, 0.5f * -0.284496736f);
                p = fmaf(p, r, 0.5f * 0.254829592f);
                const float w = p * r * at;
                const float ex = __builtin_amdgcn_exp2f(t * t * (-0.5f * 1.4426950408889634f));
                o[e] = (f16)fmaf(-w, ex, fmaxf(t, 0.f));
            }
            *reinterpret_cast<f16x8*>(y + (size_t)row * 512 + lane * 8) = o;
        }
    }
}
#endif  // LG_LN_FORM == 1

// ---- dual log-softmax ----
// Pass 1 (lse_kernel): blocks [0, rb) -> row logsumexp (one wave per row); blocks [rb, ...) ->
// column partials: a block is 64 consecutive columns x one chunk of kColChunk rows, its 256
// threads = 64 columns x 4 interleaved rows (a wave reads 256 contiguous bytes of a row), online
// (max, sum) per thread, merged through LDS, one (max, sum) per (chunk, column) to the workspace.
// Pass 2 (dual_combine_kernel): a block is 8 rows x 256 columns; it first finishes the column
// logsumexp of its 256 columns from the chunk partials, then writes its rows.
constexpr int kColChunk = 128;  // rows per column-partial block
constexpr int kCombRows = 8;    // rows per combine block

__device__ __forceinline__ void lse_merge(float& mx, float& s, float m2, float s2) {
    if (m2 == -INFINITY) return;
    if (m2 > mx) {
        s = s * __expf(mx - m2) + s2;
        mx = m2;
    } else {
        s += s2 * __expf(m2 - mx);
    }
}

__global__ __launch_bounds__(256) void lse_kernel(const float* __restrict__ sim, int m, int n, int rb,
                                                  float* lse_row, float2* col_part, size_t ws_stride) {
    // blockIdx.y: the pair of a batched launch (its sim slice and workspace slice)
    sim += (size_t)blockIdx.y * m * n;
    lse_row = reinterpret_cast<float*>(reinterpret_cast<char*>(lse_row) + blockIdx.y * ws_stride);
    col_part = reinterpret_cast<float2*>(reinterpret_cast<char*>(col_part) + blockIdx.y * ws_stride);
    if ((int)blockIdx.x < rb) {
        const int lane = threadIdx.x & 63;
        const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
        if (row >= m) return;
        const float* r = sim + (size_t)row * n;
        float mx = -INFINITY;
        for (int j = lane; j < n; j += 64) mx = fmaxf(mx, r[j]);
        mx = wave_max(mx);
        float s = 0.f;
        for (int j = lane; j < n; j += 64) s += __expf(r[j] - mx);
        s = wave_sum(s);
        if (lane == 0) lse_row[row] = mx + __logf(s);
        return;
    }
    __shared__ float2 part[4][64];
    const int b = blockIdx.x - rb, cgroups = (n + 63) / 64;
    const int chunk = b / cgroups, col = (b % cgroups) * 64 + (threadIdx.x & 63);
    const int r4 = threadIdx.x >> 6;
    const int i0 = chunk * kColChunk, i1 = min(m, i0 + kColChunk);
    float mx = -INFINITY, s = 0.f;
    if (col < n) {
#pragma unroll 4
        for (int i = i0 + r4; i < i1; i += 4) {
            const float v = sim[(size_t)i * n + col];
            if (v > mx) {
                s = s * __expf(mx - v) + 1.f;
                mx = v;
            } else {
                s += __expf(v - mx);
            }
        }
    }
    part[r4][threadIdx.x & 63] = make_float2(mx, s);
    __syncthreads();
    if (r4 == 0 && col < n) {
#pragma unroll
        for (int k = 1; k < 4; ++k) lse_merge(mx, s, part[k][threadIdx.x].x, part[k][threadIdx.x].y);
        col_part[(size_t)chunk * n + col] = make_float2(mx, s);
    }
}

__device__ __forceinline__ float log_sigmoid(float z) { return fminf(z, 0.f) - log1pf(__expf(-fabsf(z))); }

// pass 2: scores = 2 sim - lse_row[i] - lse_col[j] + logsig(z0[i]) + logsig(z1[j])
__global__ __launch_bounds__(256) void dual_combine_kernel(const float* __restrict__ sim, const float* z0,
                                                           const float* z1, const float* lse_row,
                                                           const float2* col_part, int chunks, int m, int n,
                                                           float* out, size_t ws_stride) {
    sim += (size_t)blockIdx.y * m * n;
    out += (size_t)blockIdx.y * m * n;
    z0 += (size_t)blockIdx.y * m;
    z1 += (size_t)blockIdx.y * n;
    lse_row = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lse_row) + blockIdx.y * ws_stride);
    col_part = reinterpret_cast<const float2*>(reinterpret_cast<const char*>(col_part) + blockIdx.y * ws_stride);
    const int cblocks = (n + 255) / 256;
    const int j = (blockIdx.x % cblocks) * 256 + threadIdx.x;
    const int i0 = (blockIdx.x / cblocks) * kCombRows;
    if (j >= n) return;
    float mx = -INFINITY, s = 0.f;
    for (int c = 0; c < chunks; ++c) {
        const float2 p = col_part[(size_t)c * n + j];
        lse_merge(mx, s, p.x, p.y);
    }
    const float cterm = logf(s) + mx;
    const float zj = log_sigmoid(z1[j]);
    const int i1 = min(m, i0 + kCombRows);
    for (int i = i0; i < i1; ++i)
        out[(size_t)i * n + j] = 2.f * sim[(size_t)i * n + j] - lse_row[i] - cterm + log_sigmoid(z0[i]) + zj;
}

// ---- dual log-softmax on the fp16 similarity (round 5; the fp16 matcher's assignment head) ----
// The fp16 model computes sim = m0·m1ᵀ in fp16 and the reference takes .float() of it
// (lightglue.py:214-216); these kernels read the fp16 sim and the fp16 matchability logits (strided:
// one channel of the final projection's output) directly, so no fp32 copies exist. Pass 1: a block
// is 64 rows x all columns of one pair; each of its 8 waves loads a batch of 8 rows at once (a lane
// owns 16 columns, 16-B loads): the row logsumexp of each (wave max, then the exp sum) and, per
// column, the batch's max and one exponential per element into a running (max, sum), merged over
// the 8 waves through LDS into one partial per (64-row block, column). (Round 5: 115 -> 49.6 us at
// P = 16 against the fp32 kernels above on a .float() copy, profiles/r05/matcher_p16_kernel_stats_head.csv.)
// Pass 2: a block is 64 rows; it first closes the column logsumexp (+ log-sigmoid of z1) of every
// column from the partials into LDS, then writes its rows as fp32 with 16-B stores.
constexpr int kDsRows = 64;  // rows per block, both passes

struct DsArgs {
    const f16* sim;            // [batch, m, n]
    const f16* z0;             // row i of pair p at z0[p * zps + i * zrs]
    const f16* z1;             // column j of pair p at z1[p * zps + j * zrs]
    long zps, zrs;
    float* scores;             // [batch, m, n]
    float* lse_row;            // workspace: [batch][m]
    float2* col_part;          // workspace: [batch][rblocks][n]
    float* cterm;              // workspace (small launches): [batch][n] logsig(z1) - column logsumexp
    int m, n, rblocks;
};

__device__ __forceinline__ void lse_step(float& mx, float& s, float v) {  // online (max, sum) of exp
    if (v > mx) {
        s = s * __expf(mx - v) + 1.f;
        mx = v;
    } else {
        s += __expf(v - mx);
    }
}

constexpr int kDsBatch = 8;  // rows a wave loads at once (16 KiB in flight per wave at n = 1024)
constexpr int kDsWaves = 8;  // waves per block: kDsRows / kDsWaves = one batch of rows each

// W waves per block, kDsBatch rows each (W = kDsWaves: 64-row blocks; W = 1: 8-row blocks, the small
// launches' form: a single pair's 1024 rows as 128 blocks instead of 16)
template <int CPL, int W>  // columns per lane in units of 8 (n <= 512 CPL)
__global__ __launch_bounds__(64 * W) void lse16_kernel(DsArgs a) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    const int p = blockIdx.y, rb = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const f16* sim = a.sim + (size_t)p * a.m * a.n;
    float cm[CPL][8], cs[CPL][8];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) cm[c][e] = -INFINITY, cs[c][e] = 0.f;
    const int r0 = (rb * W + wave) * kDsBatch;
    const int r1 = min(r0 + kDsBatch, a.m);
    for (int i0 = r0; i0 < r1; i0 += kDsBatch) {
        // a batch of rows, every load issued first (rows past the block's end: -inf)
        f16x8 x[kDsBatch][CPL];
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b)
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = (c * 64 + lane) * 8;
                if (i0 + b < r1 && j < a.n) x[b][c] = *reinterpret_cast<const f16x8*>(sim + (size_t)(i0 + b) * a.n + j);
                else
#pragma unroll
                    for (int e = 0; e < 8; ++e) x[b][c][e] = (f16)-INFINITY;
            }
        // row logsumexp of each row of the batch (independent wave reductions)
        float mx[kDsBatch], s[kDsBatch];
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) {
            mx[b] = -INFINITY;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int e = 0; e < 8; ++e) mx[b] = fmaxf(mx[b], (float)x[b][c][e]);
        }
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) mx[b] = wave_max(mx[b]);
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) {
            s[b] = 0.f;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int e = 0; e < 8; ++e) s[b] += __expf((float)x[b][c][e] - mx[b]);
        }
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) s[b] = wave_sum(s[b]);
        if (lane < kDsBatch) {
            float l = 0.f;
#pragma unroll
            for (int b = 0; b < kDsBatch; ++b)
                if (lane == b) l = mx[b] + __logf(s[b]);
            if (i0 + lane < r1) a.lse_row[(size_t)p * a.m + i0 + lane] = l;
        }
        // per column: the batch's max, then one exponential per element
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float bm = (float)x[0][c][e];
#pragma unroll
                for (int b = 1; b < kDsBatch; ++b) bm = fmaxf(bm, (float)x[b][c][e]);
                const float nm = fmaxf(cm[c][e], bm);
                if (nm == -INFINITY) continue;  // (columns past n)
                float t = cs[c][e] * __expf(cm[c][e] - nm);
#pragma unroll
                for (int b = 0; b < kDsBatch; ++b) t += __expf((float)x[b][c][e] - nm);
                cm[c][e] = nm, cs[c][e] = t;
            }
    }
    // the waves' column partials -> one per (block, column)
    __shared__ float2 part[W][64 * 8];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
#pragma unroll
        for (int e = 0; e < 8; ++e) part[wave][lane * 8 + e] = make_float2(cm[c][e], cs[c][e]);
        __syncthreads();
        for (int t = threadIdx.x; t < 512; t += 64 * W) {
            const int j = c * 512 + t;
            float mx = part[0][t].x, s = part[0][t].y;
#pragma unroll
            for (int w = 1; w < W; ++w) lse_merge(mx, s, part[w][t].x, part[w][t].y);
            if (j < a.n) a.col_part[((size_t)p * a.rblocks + rb) * a.n + j] = make_float2(mx, s);
        }
        __syncthreads();
    }
}

// The small launches' column pass: a block is 64 columns of one pair x 16 groups of row-block
// partials (merged in a fixed order: group g takes partials g, g + 16, ...; then groups 0..15), written
// once as logsig(z1[j]) - lse_col[j] for combine16_kernel<PRE>.
constexpr int kColGroups = 16;
__global__ __launch_bounds__(64 * kColGroups) void col_lse_kernel(DsArgs a) {
    const int p = blockIdx.y, j = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
    float mx = -INFINITY, s = 0.f;
    if (j < a.n) {
        for (int b0 = g; b0 < a.rblocks; b0 += kColGroups * 8) {
            float2 q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int b = b0 + kColGroups * u;
                q[u] = b < a.rblocks ? a.col_part[((size_t)p * a.rblocks + b) * a.n + j] : make_float2(-INFINITY, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) lse_merge(mx, s, q[u].x, q[u].y);
        }
    }
    __shared__ float2 part[kColGroups][64];
    part[g][threadIdx.x & 63] = make_float2(mx, s);
    __syncthreads();
    if (g == 0 && j < a.n) {
#pragma unroll
        for (int w = 1; w < kColGroups; ++w) lse_merge(mx, s, part[w][threadIdx.x].x, part[w][threadIdx.x].y);
        a.cterm[(size_t)p * a.n + j] = log_sigmoid((float)a.z1[p * a.zps + j * a.zrs]) - (logf(s) + mx);
    }
}

// PRE: the column terms come from col_lse_kernel (a.cterm), else every block merges the partials
template <int CPL, int W, bool PRE>
__global__ __launch_bounds__(64 * W) void combine16_kernel(DsArgs a) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const int p = blockIdx.y, rb = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ float cterm[512 * CPL];  // logsig(z1[j]) - lse_col[j]
    if constexpr (PRE) {
        for (int j = threadIdx.x * 4; j < a.n; j += 64 * W * 4)
            *reinterpret_cast<float4*>(cterm + j) = *reinterpret_cast<const float4*>(a.cterm + (size_t)p * a.n + j);
    } else
    for (int j = threadIdx.x; j < a.n; j += 64 * W) {
        float2 q[16];
        float mx = -INFINITY, s = 0.f;
        for (int b0 = 0; b0 < a.rblocks; b0 += 16) {  // (16 partial loads in flight)
#pragma unroll
            for (int b = 0; b < 16; ++b)
                q[b] = b0 + b < a.rblocks ? a.col_part[((size_t)p * a.rblocks + b0 + b) * a.n + j] : make_float2(-INFINITY, 0.f);
#pragma unroll
            for (int b = 0; b < 16; ++b) lse_merge(mx, s, q[b].x, q[b].y);
        }
        cterm[j] = log_sigmoid((float)a.z1[p * a.zps + j * a.zrs]) - (logf(s) + mx);
    }
    __syncthreads();
    const f16* sim = a.sim + (size_t)p * a.m * a.n;
    float* out = a.scores + (size_t)p * a.m * a.n;
    const int r0 = (rb * W + wave) * kDsBatch;
    const int r1 = min(r0 + kDsBatch, a.m);
    for (int i0 = r0; i0 < r1; i0 += kDsBatch) {
        f16x8 x[kDsBatch][CPL];
        float rterm[kDsBatch];
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) {
            const int i = min(i0 + b, r1 - 1);
            rterm[b] = log_sigmoid((float)a.z0[p * a.zps + (long)i * a.zrs]) - a.lse_row[(size_t)p * a.m + i];
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = (c * 64 + lane) * 8;
                if (j < a.n) x[b][c] = *reinterpret_cast<const f16x8*>(sim + (size_t)i * a.n + j);
            }
        }
#pragma unroll
        for (int b = 0; b < kDsBatch; ++b) {
            if (i0 + b >= r1) break;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = (c * 64 + lane) * 8;
                if (j >= a.n) continue;
                f32x4 o0, o1;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    o0[e] = 2.f * (float)x[b][c][e] + rterm[b] + cterm[j + e];
                    o1[e] = 2.f * (float)x[b][c][e + 4] + rterm[b] + cterm[j + e + 4];
                }
                *reinterpret_cast<f32x4*>(out + (size_t)(i0 + b) * a.n + j) = o0;
                *reinterpret_cast<f32x4*>(out + (size_t)(i0 + b) * a.n + j + 4) = o1;
            }
        }
    }
}

// ---- the forward's inputs in the pair-major layout + the positional encoding (round 5) ----
// x [pairs * (n0 + n1), dim] from desc0 [pairs, n0, dim], desc1 [pairs, n1, dim] (the reference's
// torch.cat of the two images, lightglue.py:332-336, pairs stacked), and the rotary tables cos, sin
// [rows, 64] of FourierPositionalEncoding (lightglue.py:32-52): proj_k = Wr[k] · kpt rounded to fp16
// (the fp16 model's Linear(2, 32)), cos / sin of it rounded to fp16, each repeated for the two
// members of a rotary pair. A block is 8 rows; per row 32 threads copy the descriptor (16 B each,
// dim = 256) and compute one (cos, sin) pair each.
__global__ __launch_bounds__(256) void pair_inputs_kernel(const f16* __restrict__ d0, const f16* __restrict__ d1,
                                                          const f16* __restrict__ k0, const f16* __restrict__ k1,
                                                          const f16* __restrict__ wr, int n0, int n1, int rows,
                                                          f16* x, f16* cosv, f16* sinv) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    typedef f16 f16x2 __attribute__((ext_vector_type(2)));
    const int row = blockIdx.x * 8 + (threadIdx.x >> 5), t = threadIdx.x & 31;
    if (row >= rows) return;
    const int ntot = n0 + n1, p = row / ntot, l = row - p * ntot;
    const bool first = l < n0;
    const size_t src = first ? (size_t)p * n0 + l : (size_t)p * n1 + (l - n0);
    const f16* d = first ? d0 : d1;
    const f16* kp = (first ? k0 : k1) + src * 2;
    *reinterpret_cast<f16x8*>(x + (size_t)row * 256 + t * 8) = *reinterpret_cast<const f16x8*>(d + src * 256 + t * 8);
    const float proj = (float)(f16)((float)wr[2 * t] * (float)kp[0] + (float)wr[2 * t + 1] * (float)kp[1]);
    const f16 c = (f16)cosf(proj), s = (f16)sinf(proj);
    *reinterpret_cast<f16x2*>(cosv + (size_t)row * kD + 2 * t) = f16x2{c, c};
    *reinterpret_cast<f16x2*>(sinv + (size_t)row * kD + 2 * t) = f16x2{s, s};
}

inline unsigned blocks_for(long threads) { return (unsigned)((threads + 255) / 256); }

int32_t launched(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return MHA_HD64_STATUS_SUCCESS;
    return mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, what, hipGetErrorString(e));
}

bool bad_dtype(int32_t dt) { return dt != MHA_HD64_DT_HALF && dt != MHA_HD64_DT_FLOAT; }

}  // namespace

extern "C" {

int32_t lg_qkv_rotary_split(int32_t dtype, const void* qkv, const void* cosv, const void* sinv, int32_t heads,
                            int32_t n0, int32_t n1, int32_t pairs, void* q0, void* k0, void* v0, void* q1, void* k1,
                            void* v1, hipStream_t stream) {
    if (bad_dtype(dtype) || heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !qkv || !cosv || !sinv)
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_qkv_rotary_split", "bad arguments");
    const int rows = pairs * (n0 + n1);
    const long threads = (long)rows * heads * (kD / 2);
    if (threads == 0) return MHA_HD64_STATUS_SUCCESS;
    if (dtype == MHA_HD64_DT_HALF)
        hipLaunchKernelGGL(qkv_rotary_split_kernel<f16>, dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const f16*)qkv, (const f16*)cosv, (const f16*)sinv, heads, n0, n1, rows, (f16*)q0,
                           (f16*)k0, (f16*)v0, (f16*)q1, (f16*)k1, (f16*)v1);
    else
        hipLaunchKernelGGL(qkv_rotary_split_kernel<float>, dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const float*)qkv, (const float*)cosv, (const float*)sinv, heads, n0, n1, rows, (float*)q0,
                           (float*)k0, (float*)v0, (float*)q1, (float*)k1, (float*)v1);
    return launched("lg_qkv_rotary_split");
}

int32_t lg_split_heads2(int32_t dtype, const void* a, const void* b, int32_t heads, int32_t n0, int32_t n1,
                        int32_t pairs, void* a0, void* a1, void* b0, void* b1, hipStream_t stream) {
    return lg_split_heads2_ld(dtype, a, b, heads * kD, heads, n0, n1, pairs, a0, a1, b0, b1, stream);
}

int32_t lg_split_heads2_ld(int32_t dtype, const void* a, const void* b, int32_t ld, int32_t heads, int32_t n0,
                           int32_t n1, int32_t pairs, void* a0, void* a1, void* b0, void* b1, hipStream_t stream) {
    const int E = dtype == MHA_HD64_DT_HALF ? 8 : 4;
    if (bad_dtype(dtype) || heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !a || ld < heads * kD || ld % E != 0 ||
        (reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) % 16 != 0)
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_split_heads2", "bad arguments");
    const int rows = pairs * (n0 + n1);
    const long threads = (b ? 2 : 1) * (long)rows * heads * (kD / E);
    if (threads == 0) return MHA_HD64_STATUS_SUCCESS;
    if (dtype == MHA_HD64_DT_HALF)
        hipLaunchKernelGGL((heads_kernel<f16, true>), dim3(blocks_for(threads)), dim3(256), 0, stream, (const f16*)a,
                           (const f16*)b, (f16*)a0, (f16*)a1, (f16*)b0, (f16*)b1, heads, n0, n1, rows, ld);
    else
        hipLaunchKernelGGL((heads_kernel<float, true>), dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const float*)a, (const float*)b, (float*)a0, (float*)a1, (float*)b0, (float*)b1, heads,
                           n0, n1, rows, ld);
    return launched("lg_split_heads2");
}

int32_t lg_merge_heads(int32_t dtype, const void* x0, const void* x1, int32_t heads, int32_t n0, int32_t n1,
                       int32_t pairs, void* out, hipStream_t stream) {
    if (bad_dtype(dtype) || heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !out)
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_merge_heads", "bad arguments");
    const int E = dtype == MHA_HD64_DT_HALF ? 8 : 4;
    const int rows = pairs * (n0 + n1);
    const long threads = (long)rows * heads * (kD / E);
    if (threads == 0) return MHA_HD64_STATUS_SUCCESS;
    if (dtype == MHA_HD64_DT_HALF)
        hipLaunchKernelGGL((heads_kernel<f16, false>), dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const f16*)x0, (const f16*)x1, (f16*)out, nullptr, nullptr, nullptr, heads, n0, n1, rows,
                           heads * kD);
    else
        hipLaunchKernelGGL((heads_kernel<float, false>), dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const float*)x0, (const float*)x1, (float*)out, nullptr, nullptr, nullptr, heads, n0,
                           n1, rows, heads * kD);
    return launched("lg_merge_heads");
}

int32_t lg_merge_heads_cat(int32_t dtype, const void* x, const void* x0, const void* x1, int32_t heads, int32_t n0,
                           int32_t n1, int32_t pairs, void* out, hipStream_t stream) {
    if (bad_dtype(dtype) || heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !x || !out)
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_merge_heads_cat", "bad arguments");
    const int E = dtype == MHA_HD64_DT_HALF ? 8 : 4;
    const int rows = pairs * (n0 + n1);
    const long threads = (long)rows * 2 * heads * (kD / E);
    if (threads == 0) return MHA_HD64_STATUS_SUCCESS;
    if (dtype == MHA_HD64_DT_HALF)
        hipLaunchKernelGGL((merge_cat_kernel<f16>), dim3(blocks_for(threads)), dim3(256), 0, stream, (const f16*)x,
                           (const f16*)x0, (const f16*)x1, (f16*)out, heads, n0, n1, rows);
    else
        hipLaunchKernelGGL((merge_cat_kernel<float>), dim3(blocks_for(threads)), dim3(256), 0, stream,
                           (const float*)x, (const float*)x0, (const float*)x1, (float*)out, heads, n0, n1, rows);
    return launched("lg_merge_heads_cat");
}

int32_t lg_layernorm_gelu(int32_t dtype, const void* x, const void* gamma, const void* beta, int32_t rows,
                          int32_t dim, float eps, void* y, hipStream_t stream) {
    if (bad_dtype(dtype) || rows < 0 || dim <= 0 || dim % 64 != 0 || dim > 1024 || !x || !gamma || !beta || !y)
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_layernorm_gelu", "bad arguments");
    if (rows == 0) return MHA_HD64_STATUS_SUCCESS;
    const dim3 grid((rows + 3) / 4);
    if (dtype == MHA_HD64_DT_HALF && dim == 512 &&
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
          reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
#if LG_LN_FORM == 1
        const int cap = 256 * kLnBlocksPerCU;
        const int nb = (rows + 3) / 4 < cap ? (rows + 3) / 4 : cap;
        hipLaunchKernelGGL(ln_gelu_512_rows_kernel, dim3(nb), dim3(256), 0, stream, (const f16*)x, (const f16*)gamma,
                           (const f16*)beta, rows, eps, (f16*)y);
#else
        hipLaunchKernelGGL(ln_gelu_512_f16_kernel, grid, dim3(256), 0, stream, (const f16*)x, (const f16*)gamma,
                           (const f16*)beta, rows, eps, (f16*)y);
#endif
        return launched("lg_layernorm_gelu");
    }
#define LG_LN(PER)                                                                                              \
    case PER:                                                                                                   \
        if (dtype == MHA_HD64_DT_HALF)                                                                          \
            hipLaunchKernelGGL((ln_gelu_kernel<f16, PER>), grid, dim3(256), 0, stream, (const f16*)x,           \
                               (const f16*)gamma, (const f16*)beta, rows, eps, (f16*)y);                        \
        else                                                                                                    \
            hipLaunchKernelGGL((ln_gelu_kernel<float, PER>), grid, dim3(256), 0, stream, (const float*)x,       \
                               (const float*)gamma, (const float*)beta, rows, eps, (float*)y);                  \
        break;
    switch (dim / 64) {
        LG_LN(1) LG_LN(2) LG_LN(4) LG_LN(8) LG_LN(16)
        default:
            return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_layernorm_gelu",
                                          "dim must be 64, 128, 256, 512 or 1024");
    }
#undef LG_LN
    return launched("lg_layernorm_gelu");
}

namespace {
size_t dual_ws_stride(int32_t m, int32_t n) {  // one pair's workspace slice (256-B aligned)
    const size_t chunks = (size_t)(m + kColChunk - 1) / kColChunk;
    const size_t b = ((size_t)m * sizeof(float) + 15) / 16 * 16 + chunks * (size_t)n * sizeof(float2);
    return (b + 255) / 256 * 256;
}
}  // namespace

size_t lg_log_double_softmax_workspace(int32_t m, int32_t n, int32_t batch) {
    if (m <= 0 || n <= 0 || batch <= 0) return 0;
    return dual_ws_stride(m, n) * (size_t)batch;
}

int32_t lg_log_double_softmax(const float* sim, const float* z0, const float* z1, int32_t m, int32_t n,
                              int32_t batch, float* scores, void* workspace, hipStream_t stream) {
    if (m < 0 || n < 0 || batch < 0 || ((m > 0 && n > 0 && batch > 0) && (!sim || !z0 || !z1 || !scores || !workspace)))
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_log_double_softmax", "bad arguments");
    if (m == 0 || n == 0 || batch == 0) return MHA_HD64_STATUS_SUCCESS;
    const size_t ws_stride = dual_ws_stride(m, n);
    float* lse_row = reinterpret_cast<float*>(workspace);
    float2* col_part = reinterpret_cast<float2*>(reinterpret_cast<char*>(workspace) +
                                                 ((size_t)m * sizeof(float) + 15) / 16 * 16);
    const int rb = (m + 3) / 4;
    const int chunks = (m + kColChunk - 1) / kColChunk;
    const int cblocks = (n + 63) / 64;
    hipLaunchKernelGGL(lse_kernel, dim3(rb + chunks * cblocks, batch), dim3(256), 0, stream, sim, m, n, rb, lse_row,
                       col_part, ws_stride);
    hipLaunchKernelGGL(dual_combine_kernel, dim3(((m + kCombRows - 1) / kCombRows) * ((n + 255) / 256), batch),
                       dim3(256), 0, stream, sim, z0, z1, lse_row, col_part, chunks, m, n, scores, ws_stride);
    return launched("lg_log_double_softmax");
}

namespace {
// small launches (fewer than 64 blocks of 64 rows): 8-row one-wave blocks and a separate column pass
bool ds_small(int32_t m, int32_t batch) { return (long)((m + kDsRows - 1) / kDsRows) * batch < 64; }
int ds_rows(int32_t m, int32_t batch) { return ds_small(m, batch) ? kDsBatch : kDsRows; }
}  // namespace

size_t lg_log_double_softmax_f16_workspace(int32_t m, int32_t n, int32_t batch) {
    if (m <= 0 || n <= 0 || batch <= 0) return 0;
    const size_t rb = (size_t)(m + ds_rows(m, batch) - 1) / ds_rows(m, batch);
    return ((size_t)batch * m * sizeof(float) + 255) / 256 * 256 + ((size_t)batch * rb * n * sizeof(float2) + 255) / 256 * 256 +
           (ds_small(m, batch) ? (size_t)batch * n * sizeof(float) : 0);
}

int32_t lg_log_double_softmax_f16(const void* sim, const void* z0, const void* z1, int64_t z_pair_stride,
                                  int64_t z_row_stride, int32_t m, int32_t n, int32_t batch, float* scores,
                                  void* workspace, hipStream_t stream) {
    if (m < 0 || n < 0 || batch < 0 || n % 8 != 0 || n > 2048 ||
        ((m > 0 && n > 0 && batch > 0) &&
         (!sim || !z0 || !z1 || !scores || !workspace || (reinterpret_cast<uintptr_t>(sim) & 15) ||
          (reinterpret_cast<uintptr_t>(scores) & 15))))
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_log_double_softmax_f16", "bad arguments");
    if (m == 0 || n == 0 || batch == 0) return MHA_HD64_STATUS_SUCCESS;
    DsArgs a;
    a.sim = (const f16*)sim, a.z0 = (const f16*)z0, a.z1 = (const f16*)z1, a.zps = z_pair_stride, a.zrs = z_row_stride;
    const bool small = ds_small(m, batch);
    const int rows = ds_rows(m, batch);
    a.scores = scores, a.m = m, a.n = n, a.rblocks = (m + rows - 1) / rows;
    a.lse_row = reinterpret_cast<float*>(workspace);
    const size_t lse_bytes = ((size_t)batch * m * sizeof(float) + 255) / 256 * 256;
    a.col_part = reinterpret_cast<float2*>(reinterpret_cast<char*>(workspace) + lse_bytes);
    a.cterm = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + lse_bytes +
                                       ((size_t)batch * a.rblocks * n * sizeof(float2) + 255) / 256 * 256);
    const dim3 grid(a.rblocks, batch);
#define LG_DS(CPL)                                                                                       \
    if (small) {                                                                                         \
        hipLaunchKernelGGL((lse16_kernel<CPL, 1>), grid, dim3(64), 0, stream, a);                        \
        hipLaunchKernelGGL(col_lse_kernel, dim3((n + 63) / 64, batch), dim3(64 * kColGroups), 0, stream, a); \
        hipLaunchKernelGGL((combine16_kernel<CPL, 1, true>), grid, dim3(64), 0, stream, a);               \
    } else {                                                                                             \
        hipLaunchKernelGGL((lse16_kernel<CPL, kDsWaves>), grid, dim3(64 * kDsWaves), 0, stream, a);      \
        hipLaunchKernelGGL((combine16_kernel<CPL, kDsWaves, false>), grid, dim3(64 * kDsWaves), 0, stream, a); \
    }
    if (n <= 512) {
        LG_DS(1)
    } else if (n <= 1024) {
        LG_DS(2)
    } else {
        LG_DS(4)
    }
#undef LG_DS
    return launched("lg_log_double_softmax_f16");
}

int32_t lg_pair_inputs(const void* desc0, const void* desc1, const void* kpts0, const void* kpts1, const void* wr,
                       int32_t n0, int32_t n1, int32_t pairs, int32_t dim, void* x, void* cosv, void* sinv,
                       hipStream_t stream) {
    const long rows = (long)pairs * (n0 + n1);
    if (n0 < 0 || n1 < 0 || pairs < 0 || dim != 256 || (rows > 0 && (!x || !cosv || !sinv || !wr)) ||
        (n0 > 0 && (!desc0 || !kpts0)) || (n1 > 0 && (!desc1 || !kpts1)) ||
        ((reinterpret_cast<uintptr_t>(desc0) | reinterpret_cast<uintptr_t>(desc1) | reinterpret_cast<uintptr_t>(x)) & 15) ||
        ((reinterpret_cast<uintptr_t>(cosv) | reinterpret_cast<uintptr_t>(sinv)) & 3) || rows > (1L << 30))
        return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, "lg_pair_inputs", "bad arguments");
    if (rows == 0) return MHA_HD64_STATUS_SUCCESS;
    hipLaunchKernelGGL(pair_inputs_kernel, dim3((unsigned)((rows + 7) / 8)), dim3(256), 0, stream, (const f16*)desc0,
                       (const f16*)desc1, (const f16*)kpts0, (const f16*)kpts1, (const f16*)wr, n0, n1, (int)rows,
                       (f16*)x, (f16*)cosv, (f16*)sinv);
    return launched("lg_pair_inputs");
}

}  // extern "C"
