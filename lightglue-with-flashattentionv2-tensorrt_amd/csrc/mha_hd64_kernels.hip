// mha_hd64_kernels.hip — fused FlashAttention-v2 forward, head_dim = 64, for gfx950 (MI355X, CDNA4).
//
// Computes, per (batch, head):  O = softmax(Q·Kᵀ · 0.125) · V
// the operator of the reference's TensorRT plugin "MHAHeadDim64"
// (lightglue_attention_plugin/attention_headdim_64_fp16in_fp16out.cu:253-733 and
//  attention_headdim_64_fp16in_fp32out.cu:253-703; oracle
//  lightglue_pytorch_no_plugin/lightglue.py:75-85).
//
// Design (MI355X-first, not a translation of the CuTe/SM80 kernel):
//  * Workgroup = QW x KW wave64s. Each wave owns 32 query rows: QW waves split the query
//    block, KW waves split the keys of every iteration (intra-workgroup split-KV, merged
//    through LDS at the end). 8-wave workgroups put two waves on every SIMD so one wave's
//    softmax (VALU) runs beside the other's MFMAs. An optional cross-workgroup KV split
//    (`splits`) writes fp32 partials + (m, l) to the workspace and a combine kernel merges
//    them; this is what fills the 256 CUs for a single 1x4x1024x1024 call.
//  * Swapped QKᵀ on v_mfma_f32_32x32x16_f16: Sᵀ = K·Qᵀ puts one query per lane (column)
//    and 16 keys per lane in registers, so the softmax row max / row sum is an in-register
//    reduction plus one v_permlane32_swap.
//  * The score scale 0.125·log2(e) is folded into Q once (fp16), and the running row max
//    is folded into the MFMA's C operand (C = -m, a register block that only changes on a
//    rescale), so the MFMA emits s·c - m directly and a probability is ONE v_exp_f32.
//  * Lazy rescale (max moves only when a tile's max exceeds it by > 8 in log2 units, P
//    stays <= 256 which fp16 carries exactly as well as 1.0): the O accumulators are
//    untouched by VALU in the steady state.
//  * P never touches LDS: the Sᵀ accumulators, packed to f16, are directly the B operand
//    of Oᵀ = Vᵀ·Pᵀ (also 32x32x16 f16); Vᵀ comes from LDS with the gfx950 transposing
//    read ds_read_b64_tr_b16. Oᵀ keeps one query per lane, so alpha is per-lane.
//  * K/V tiles (64 keys x 64 dims fp16 = 8 KiB) are register-staged into a double-buffered
//    LDS ring: global loads for iteration t+1 are issued before the MFMAs of iteration t and
//    written to LDS after them (one barrier per iteration). XOR swizzles keep ds_read_b128
//    (K) and ds_read_b64_tr_b16 (V) conflict-free.
//  * Tails (N % 64 != 0) are masked inside the kernel: no pad / unpad launches (replaces
//    the reference's a4/a5/a7 helper kernels). fp32 inputs are rounded to fp16 (RN) on load
//    (replaces the reference's a6 convert kernel).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "mha_hd64_internal.h"

namespace mha_hd64 {
namespace {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float kScaleLog2 = 0.18033688011112042f;  // 0.125 * log2(e)
constexpr float kRescaleThr = 8.0f;                  // lazy-rescale threshold (log2 units)
constexpr int kTileKV = 64;                          // keys per LDS tile
constexpr int kTileBytes = kTileKV * kHeadDim * 2;   // 8 KiB fp16 tile

struct FwdArgs {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    float* part_o;   // [bh][splits][nq][64] fp32, unnormalised (splits > 1 only)
    float2* part_ml; // [bh][splits][nq] (m in log2 units, l)
    int nq;
    int nkv;
    int splits;
    int tiles_per_split;
};

// LDS images (byte offsets inside one 8 KiB [64 rows][128 B] tile; chunk = 16 B = 8 halfs).
// K is read row-wise by ds_read_b128 (lane = key row): XOR the chunk with (row>>1)&7
// so the 16 rows of every b128 lane group hit 16 distinct 16-B bank slots.
// V is read column-wise by ds_read_b64_tr_b16 (4 rows x 32 cols per half-wave): XOR
// the chunk with ((row>>1)&1)<<2 so rows r and r+2 use opposite 64-B halves of the bank row.
__device__ __forceinline__ int k_off(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int v_off(int row, int chunk) {
    return row * 128 + ((chunk ^ (((row >> 1) & 1) << 2)) << 4);
}

template <typename T> struct Raw8;
template <> struct Raw8<f16> { f16x8 x; };
template <> struct Raw8<float> { f32x4 a, b; };

__device__ __forceinline__ void load8(Raw8<f16>& r, const f16* p) {
    r.x = *reinterpret_cast<const f16x8*>(p);
}
__device__ __forceinline__ void load8(Raw8<float>& r, const float* p) {
    r.a = *reinterpret_cast<const f32x4*>(p);
    r.b = *reinterpret_cast<const f32x4*>(p + 4);
}
__device__ __forceinline__ f16x8 to_f16(const Raw8<f16>& r) { return r.x; }
__device__ __forceinline__ f16x8 to_f16(const Raw8<float>& r) {
    // Round-to-nearest-even, as the reference's __float22half2_rn (…fp32out.cu:706-768).
    const f16x4 lo = __builtin_convertvector(r.a, f16x4);
    const f16x4 hi = __builtin_convertvector(r.b, f16x4);
    return f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Cross-half (lane l <-> l^32) reductions via v_permlane32_swap.
__device__ __forceinline__ float xhalf_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // same order in both halves
}

__device__ __forceinline__ float tree_max(const f32x16& a, const f32x16& b) {
    float t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = fmaxf(a[i], b[i]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) t[i] = fmaxf(t[i], t[i + w]);
    return t[0];
}
__device__ __forceinline__ float tree_sum(const f32x16& a, const f32x16& b) {
    float t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = a[i] + b[i];
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) t[i] = t[i] + t[i + w];
    return t[0];
}

__device__ __forceinline__ f16x4 tr_read(const char* lds_base, int byte_off) {
    const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds_base + byte_off));
    return __builtin_bit_cast(f16x4, v);
}

__device__ __forceinline__ f16x8 cat8(f16x4 a, f16x4 b) {
    return f16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <typename TOut>
__device__ __forceinline__ void store4(TOut* dst, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void store4<float>(float* dst, float a, float b, float c, float d) {
    *reinterpret_cast<f32x4*>(dst) = f32x4{a, b, c, d};
}
template <>
__device__ __forceinline__ void store4<f16>(f16* dst, float a, float b, float c, float d) {
    *reinterpret_cast<f16x4*>(dst) = f16x4{(f16)a, (f16)b, (f16)c, (f16)d};
}

__device__ __forceinline__ f32x16 splat16(float x) {
    return f32x16{x, x, x, x, x, x, x, x, x, x, x, x, x, x, x, x};
}

// ----------------------------------------------------------------------------------------
// Main kernel. Grid: x = query blocks of 32*QW rows, y = batch*heads, z = KV splits.
// ----------------------------------------------------------------------------------------
template <typename TIn, typename TOut, int QW, int KW>
__global__ __launch_bounds__(64 * QW * KW, 1) void mha_hd64_fwd_kernel(FwdArgs a) {
    constexpr int NT = 64 * QW * KW;                // threads
    constexpr int BLOCK_M = 32 * QW;                // query rows per workgroup
    constexpr int SUPER = kTileKV * KW;             // keys per iteration
    constexpr int STAGE_BYTES = KW * 2 * kTileBytes;
    constexpr int NLOAD = (2 * KW * 512) / NT;      // 16-B chunks staged per thread per iteration
    static_assert(NLOAD * NT == 2 * KW * 512, "staging must divide evenly");
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave
    const int qw = wave % QW;
    const int kw = wave / QW;
    const int nq = a.nq, nkv = a.nkv;
    const int bh = blockIdx.y;
    const int split = blockIdx.z;

    const TIn* Qb = reinterpret_cast<const TIn*>(a.q) + (size_t)bh * nq * kHeadDim;
    const TIn* Kb = reinterpret_cast<const TIn*>(a.k) + (size_t)bh * nkv * kHeadDim;
    const TIn* Vb = reinterpret_cast<const TIn*>(a.v) + (size_t)bh * nkv * kHeadDim;
    const int q_row = blockIdx.x * BLOCK_M + qw * 32 + r;

    const int super_total = (nkv + SUPER - 1) / SUPER;
    const int st_begin = split * a.tiles_per_split;
    const int st_end = min(super_total, st_begin + a.tiles_per_split);
    const int n_iter = max(0, st_end - st_begin);

    // Staging: chunk i of this thread -> (tile, K|V) = id / 512, row = (id % 512) / 8, chunk = id % 8.
    Raw8<TIn> stg[NLOAD];
    auto issue = [&](int it) {
        const int kv_base = (st_begin + it) * SUPER;
#pragma unroll
        for (int i = 0; i < NLOAD; ++i) {
            const int id = i * NT + tid;
            const int tt = id >> 9;
            const int row = (id & 511) >> 3;
            const int g = min(kv_base + (tt >> 1) * kTileKV + row, nkv - 1);  // clamp: masked keys read a valid row
            load8(stg[i], ((tt & 1) ? Vb : Kb) + (size_t)g * kHeadDim + (tid & 7) * 8);
        }
    };
    auto write = [&](int stage) {
#pragma unroll
        for (int i = 0; i < NLOAD; ++i) {
            const int id = i * NT + tid;
            const int tt = id >> 9;
            const int row = (id & 511) >> 3;
            const int ch = tid & 7;
            char* dst = smem + stage * STAGE_BYTES + tt * kTileBytes + ((tt & 1) ? v_off(row, ch) : k_off(row, ch));
            *reinterpret_cast<f16x8*>(dst) = to_f16(stg[i]);
        }
    };

    if (n_iter > 0) issue(0);

    // Q fragments (B operand of Sᵀ = K·Qᵀ): lane holds Q[q_row][16s + 8hh .. +7] * 0.125*log2(e), fp16.
    f16x8 qf[4];
    {
        const int qr = min(q_row, nq - 1);  // rows past nq are computed on a valid row and never stored
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            Raw8<TIn> t;
            load8(t, Qb + (size_t)qr * kHeadDim + 16 * s + 8 * hh);
            const f16x8 h = to_f16(t);
#pragma unroll
            for (int e = 0; e < 8; ++e) qf[s][e] = (f16)((float)h[e] * kScaleLog2);
        }
    }

    if (n_iter > 0) write(0);
    __syncthreads();

    // Per-lane LDS addressing (compile-time parts are added as immediates).
    int k_addr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = k_off(r, 2 * s + hh);
    // V tr-read: lane (group g, idx 4qq+pp) supplies row (4hh + qq) + const, columns
    // 32dt + 16(g&1) + 4pp. Swizzle bit b = (qq>>1)&1 flips the 64-B half (dt).
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const int v_addr0 = v_lane + 64 * vb;        // dims 0..31
    const int v_addr1 = v_lane + 64 * (1 - vb);  // dims 32..63

    float m_run = 0.f;        // reference max of this lane's query, log2 units (s·c)
    float l_run = 0.f;        // running sum, in-lane partial (the two halves hold disjoint keys)
    f32x16 cinit = {};        // = -m_run in every element: C operand of the first QK MFMA
    f32x16 o0 = {}, o1 = {};  // Oᵀ tiles: dims 0..31 and 32..63, query on the lane

    for (int it = 0; it < n_iter; ++it) {
        if (it + 1 < n_iter) issue(it + 1);
        const int cur = it & 1;
        const char* Kt = smem + cur * STAGE_BYTES + (kw * 2) * kTileBytes;
        const char* Vt = Kt + kTileBytes;
        const int kv0 = (st_begin + it) * SUPER + kw * kTileKV;

        // ---- Sᵀ = K·Qᵀ·c - m for keys kv0..kv0+31 (s0) and kv0+32..kv0+63 (s1) ----
        f16x8 kf[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            kf[2 * s] = *reinterpret_cast<const f16x8*>(Kt + k_addr[s]);
            kf[2 * s + 1] = *reinterpret_cast<const f16x8*>(Kt + k_addr[s] + 32 * 128);
        }
        f32x16 s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[0], qf[0], cinit, 0, 0, 0);
        f32x16 s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[1], qf[0], cinit, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < 4; ++s) {
            s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s], qf[s], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + 1], qf[s], s1, 0, 0, 0);
        }

        // ---- tail mask (reference: last KV tile only, …fp16out.cu:475-494); wave-uniform ----
        if (kv0 + kTileKV > nkv) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int kk = kv0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                if (kk >= nkv) s0[i] = -INFINITY;
                if (kk + 32 >= nkv) s1[i] = -INFINITY;
            }
        }

        // ---- online softmax (per lane = per query), scores already relative to m_run ----
        // First tile: set the max exactly. Later tiles: move it only when some query's tile
        // max exceeds it by more than kRescaleThr (wave-uniform, rare).
        const float mx = xhalf_max(tree_max(s0, s1));
        const bool first = (it == 0);
        if (first || __builtin_amdgcn_ballot_w64(mx > kRescaleThr) != 0) {
            const float d = first ? ((mx == -INFINITY) ? 0.f : mx)  // a fully masked tile keeps m = 0
                                  : fmaxf(mx, 0.f);
            const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-d);
            o0 *= alpha;
            o1 *= alpha;
            l_run *= alpha;
            m_run += d;
            s0 -= d;
            s1 -= d;
            cinit = splat16(-m_run);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s0[i] = __builtin_amdgcn_exp2f(s0[i]);
            s1[i] = __builtin_amdgcn_exp2f(s1[i]);
        }
        l_run += tree_sum(s0, s1);

        // ---- P (f16) as the B operand: registers 8ss..8ss+7 of a 32x32 tile = k-step ss ----
        f16x8 p[2][2];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            p[0][0][e] = (f16)s0[e];
            p[0][1][e] = (f16)s0[8 + e];
            p[1][0][e] = (f16)s1[e];
            p[1][1][e] = (f16)s1[8 + e];
        }

        // ---- Oᵀ += Vᵀ·Pᵀ, Vᵀ fragments by transposing LDS reads ----
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const int rowc = 128 * (32 * j + 16 * ss);
                const f16x8 va = cat8(tr_read(Vt, v_addr0 + rowc), tr_read(Vt, v_addr0 + rowc + 8 * 128));
                const f16x8 vb8 = cat8(tr_read(Vt, v_addr1 + rowc), tr_read(Vt, v_addr1 + rowc + 8 * 128));
                o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(va, p[j][ss], o0, 0, 0, 0);
                o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vb8, p[j][ss], o1, 0, 0, 0);
            }

        if (it + 1 < n_iter) write((it + 1) & 1);
        __syncthreads();
    }

    // A wave that saw no key (all of its tiles past nkv) must not set the merged max.
    float m_eff = (l_run > 0.f) ? m_run : -INFINITY;

    // ---- merge the KW key-split waves of this workgroup through LDS ----
    if constexpr (KW > 1) {
        float* red_m = reinterpret_cast<float*>(smem);  // [KW][QW][64]
        float* red_o = red_m + KW * QW * 64;            // [KW-1][QW][33][64]
        red_m[(kw * QW + qw) * 64 + lane] = m_eff;
        __syncthreads();
        float M = -INFINITY;
#pragma unroll
        for (int k = 0; k < KW; ++k) M = fmaxf(M, red_m[(k * QW + qw) * 64 + lane]);
        const float w = (m_eff == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m_eff - M);
        o0 *= w;
        o1 *= w;
        l_run *= w;
        if (kw > 0) {
            float* dst = red_o + ((kw - 1) * QW + qw) * 33 * 64 + lane;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                dst[i * 64] = o0[i];
                dst[(16 + i) * 64] = o1[i];
            }
            dst[32 * 64] = l_run;
        }
        __syncthreads();
        if (kw == 0) {
#pragma unroll
            for (int k = 1; k < KW; ++k) {
                const float* src = red_o + ((k - 1) * QW + qw) * 33 * 64 + lane;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o0[i] += src[i * 64];
                    o1[i] += src[(16 + i) * 64];
                }
                l_run += src[32 * 64];
            }
        }
        m_eff = M;
    }

    if (kw != 0) return;
    const float L = xhalf_sum(l_run);
    if (q_row >= nq) return;

    if (a.splits == 1) {
        const float inv = 1.f / L;
        TOut* Ob = reinterpret_cast<TOut*>(a.o) + ((size_t)bh * nq + q_row) * kHeadDim;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d = 8 * g4 + 4 * hh;
            store4<TOut>(Ob + d, o0[4 * g4] * inv, o0[4 * g4 + 1] * inv, o0[4 * g4 + 2] * inv,
                         o0[4 * g4 + 3] * inv);
            store4<TOut>(Ob + 32 + d, o1[4 * g4] * inv, o1[4 * g4 + 1] * inv, o1[4 * g4 + 2] * inv,
                         o1[4 * g4 + 3] * inv);
        }
    } else {
        const size_t prow = ((size_t)bh * a.splits + split) * nq + q_row;
        float* Pb = a.part_o + prow * kHeadDim;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d = 8 * g4 + 4 * hh;
            store4<float>(Pb + d, o0[4 * g4], o0[4 * g4 + 1], o0[4 * g4 + 2], o0[4 * g4 + 3]);
            store4<float>(Pb + 32 + d, o1[4 * g4], o1[4 * g4 + 1], o1[4 * g4 + 2], o1[4 * g4 + 3]);
        }
        if (hh == 0) a.part_ml[prow] = make_float2(m_eff, L);
    }
}

// ----------------------------------------------------------------------------------------
// Split-KV combine: O = Σ_s w_s O_s / Σ_s w_s l_s with w_s = exp2(m_s - M) (m in log2 units).
// One thread per (row, 4-dim chunk).
// ----------------------------------------------------------------------------------------
template <typename TOut>
__global__ __launch_bounds__(256) void mha_hd64_combine_kernel(const float* __restrict__ part_o,
                                                               const float2* __restrict__ part_ml,
                                                               TOut* __restrict__ out, int rows, int nq,
                                                               int splits) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int row = idx >> 4;  // = bh * nq + q
    if (row >= rows) return;
    const int chunk = idx & 15;
    const int bh = row / nq, q = row - bh * nq;
    const size_t base = (size_t)bh * splits * nq + q;
    float M = -INFINITY;
    for (int s = 0; s < splits; ++s) M = fmaxf(M, part_ml[base + (size_t)s * nq].x);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
    for (int s = 0; s < splits; ++s) {
        const size_t pr = base + (size_t)s * nq;
        const float2 ml = part_ml[pr];
        const float w = (ml.x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml.x - M);
        L += w * ml.y;
        const f32x4 v = *reinterpret_cast<const f32x4*>(part_o + pr * kHeadDim + chunk * 4);
        acc += w * v;
    }
    const float inv = 1.f / L;
    store4<TOut>(out + (size_t)row * kHeadDim + chunk * 4, acc[0] * inv, acc[1] * inv, acc[2] * inv,
                 acc[3] * inv);
}

template <typename TIn, typename TOut, int QW, int KW>
hipError_t launch_fwd(const FwdArgs& a, int bh, hipStream_t stream) {
    const dim3 grid((a.nq + 32 * QW - 1) / (32 * QW), bh, a.splits);
    hipLaunchKernelGGL((mha_hd64_fwd_kernel<TIn, TOut, QW, KW>), grid, dim3(64 * QW * KW), 0, stream, a);
    return hipGetLastError();
}

template <typename TIn, typename TOut>
hipError_t launch_fwd_shape(const FwdArgs& a, int bh, int qw, int kw, hipStream_t stream) {
    switch (qw * 8 + kw) {
        case 4 * 8 + 1: return launch_fwd<TIn, TOut, 4, 1>(a, bh, stream);
        case 2 * 8 + 2: return launch_fwd<TIn, TOut, 2, 2>(a, bh, stream);
        case 1 * 8 + 4: return launch_fwd<TIn, TOut, 1, 4>(a, bh, stream);
        case 4 * 8 + 2: return launch_fwd<TIn, TOut, 4, 2>(a, bh, stream);
        case 2 * 8 + 4: return launch_fwd<TIn, TOut, 2, 4>(a, bh, stream);
        default: return hipErrorInvalidValue;
    }
}

template <typename TOut>
hipError_t launch_combine(const FwdArgs& a, int bh, hipStream_t stream) {
    const int rows = bh * a.nq;
    const int threads = rows * 16;
    const dim3 grid((threads + 255) / 256);
    hipLaunchKernelGGL((mha_hd64_combine_kernel<TOut>), grid, dim3(256), 0, stream, a.part_o, a.part_ml,
                       reinterpret_cast<TOut*>(a.o), rows, a.nq, a.splits);
    return hipGetLastError();
}

bool valid_shape(int qw, int kw) {
    return (qw == 4 && kw == 1) || (qw == 2 && kw == 2) || (qw == 1 && kw == 4) || (qw == 4 && kw == 2) ||
           (qw == 2 && kw == 4);
}

}  // namespace

size_t split_workspace_bytes(const Call& c, int splits) {
    if (splits <= 1) return 0;
    const size_t rows = (size_t)c.batch * c.heads * splits * c.nq;
    const size_t o_bytes = rows * kHeadDim * sizeof(float);
    return o_bytes + rows * sizeof(float2);
}

LaunchPlan plan_call(const Call& c, size_t ws_bytes, int force_q_waves, int force_kv_waves, int force_splits) {
    const int bh = c.batch * c.heads;
    int qw = force_q_waves, kw = force_kv_waves;
    if (!valid_shape(qw, kw)) {
        if (bh * ((c.nq + 127) / 128) >= 256) {
            qw = 4;  // enough 128-row query blocks to fill the chip: 8 waves, no cross-WG split
            kw = 2;
        } else {
            qw = 2;
            kw = 2;
        }
    }
    const int qtiles = (c.nq + 32 * qw - 1) / (32 * qw);
    const int super_total = (c.nkv + 64 * kw - 1) / (64 * kw);
    int want = force_splits > 0 ? force_splits : (256 + qtiles * bh - 1) / (qtiles * bh);
    want = std::max(1, std::min(want, super_total));
    LaunchPlan p{};
    p.q_waves = qw;
    p.kv_waves = kw;
    for (;;) {
        p.tiles_per_split = (super_total + want - 1) / want;
        p.splits = (super_total + p.tiles_per_split - 1) / p.tiles_per_split;
        p.ws_needed = split_workspace_bytes(c, p.splits);
        if (p.splits <= 1 || p.ws_needed <= ws_bytes) break;
        want = p.splits - 1;
    }
    if (p.splits <= 1) {
        p.splits = 1;
        p.tiles_per_split = std::max(1, super_total);
        p.ws_needed = 0;
    }
    return p;
}

hipError_t launch_attention(const Call& c, InType in, OutType out, void* workspace, size_t ws_bytes,
                            hipStream_t stream, int force_q_waves, int force_kv_waves, int force_splits,
                            int phase_mask) {
    if (c.nq <= 0 || c.batch <= 0 || c.heads <= 0) return hipSuccess;  // nothing to compute
    const LaunchPlan p = plan_call(c, workspace ? ws_bytes : 0, force_q_waves, force_kv_waves, force_splits);
    FwdArgs a{};
    a.q = c.q;
    a.k = c.k;
    a.v = c.v;
    a.o = c.o;
    a.nq = c.nq;
    a.nkv = c.nkv;
    a.splits = p.splits;
    a.tiles_per_split = p.tiles_per_split;
    if (p.splits > 1) {
        const size_t rows = (size_t)c.batch * c.heads * p.splits * c.nq;
        a.part_o = reinterpret_cast<float*>(workspace);
        a.part_ml = reinterpret_cast<float2*>(reinterpret_cast<char*>(workspace) + rows * kHeadDim * sizeof(float));
    }
    const int bh = c.batch * c.heads;
    hipError_t e = hipSuccess;
    if (phase_mask & 1) {
        if (in == InType::F16) {
            e = (out == OutType::F16) ? launch_fwd_shape<f16, f16>(a, bh, p.q_waves, p.kv_waves, stream)
                                      : launch_fwd_shape<f16, float>(a, bh, p.q_waves, p.kv_waves, stream);
        } else {
            e = (out == OutType::F16) ? launch_fwd_shape<float, f16>(a, bh, p.q_waves, p.kv_waves, stream)
                                      : launch_fwd_shape<float, float>(a, bh, p.q_waves, p.kv_waves, stream);
        }
    }
    if (e != hipSuccess || p.splits == 1 || !(phase_mask & 2)) return e;
    return (out == OutType::F16) ? launch_combine<f16>(a, bh, stream) : launch_combine<float>(a, bh, stream);
}

}  // namespace mha_hd64
