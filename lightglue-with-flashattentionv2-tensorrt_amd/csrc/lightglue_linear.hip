// lightglue_linear.hip — the matcher's projections as gfx950 MFMA kernels with their neighbours
// fused in (include/lightglue_glue.h, lg_linear_*). fp16 in/out, fp32 accumulation.
//
// The LightGlue layer (lightglue_pytorch_no_plugin/lightglue.py:88-194) is a chain of small
// GEMMs (M = both images' keypoints, K = 256 or 512, N = 256..768) separated by layout and
// elementwise steps; at matcher sizes every one of them is a few-microsecond, latency-bound
// launch. These kernels do the GEMM and the step either side in one launch:
//   * lg_linear           : out = A·Wᵀ + b (+ residual)                  (FFN layers, residual add)
//   * lg_linear_cat       : A = [x | merge_heads(ctx0, ctx1)] gathered on load (FFN input of
//                           both blocks, lightglue.py:104/181; the message projection is folded
//                           into W by the caller)
//   * lg_linear_qkv_rotary: SelfBlock Wqkv + rotary + per-image head-major q/k/v (:111-134; W's
//                           rows pre-permuted to [q|k|v][head][dim] order by the caller)
//   * lg_linear_split2    : CrossBlock to_qk | to_v as one GEMM + per-image head split (:158-166)
//
// Workgroup: 64 rows (m) x 64 output channels (n), 4 waves as 2 x 2 tiles of 32 x 32. The
// product is computed transposed, Cᵀ = W·Aᵀ on v_mfma_f32_32x32x16_f16 (A-operand = W rows,
// B-operand = activation rows, both K-contiguous), so a lane ends up owning one activation row
// and 4 runs of 4 consecutive output channels: epilogue stores are 8-B row segments and a rotary
// pair (2d, 2d+1) sits in one lane. Both 64 x K tiles reach LDS by LDS-DMA in 128-column
// chunks ([chunk][row][256 B], 16-B units XOR-swizzled by row & 15 on the source address:
// conflict-free ds_read_b128 of 16 rows at one k); the MFMAs of chunk c start once c has
// landed (counted vmcnt + barrier) while the later chunks stream in.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <cstdlib>

#include "lightglue_glue.h"
#include "mha_hd64.h"
#include "mha_hd64_internal.h"
#include "mha_hd64_device.h"  // (lds_dma16: the inline-asm LDS-DMA piece)

namespace {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) f16x8 lds_f16x8;

__device__ __forceinline__ void st_out(f16* dst, f16x8 v) { *reinterpret_cast<f16x8*>(dst) = v; }
constexpr int kBM = 64, kBN = 64, kKC = 128;
// tile rows, tile channels, K columns per LDS chunk
constexpr int kChunkBytes = 64 * kKC * 2;     // one [64 rows][128 k] fp16 chunk = 16 KiB
constexpr int kD = 64;                        // head dim

enum { EPI_BIAS = 0, EPI_QKV_ROTARY = 1, EPI_SPLIT2 = 2 };

struct LinArgs {
    const f16* a;      // [m, k] activations (A-gather: x [m, k/2])
    const f16* ctx0;   // A-gather: head-major attention outputs of image 0 / 1 [heads, ni, 64]
    const f16* ctx1;
    const f16* w;      // [n, k]
    const f16* bias;   // [n]
    const f16* res;    // [m, n] residual (EPI_BIAS, nullable)
    const f16* cosv;   // [m, 64] rotary tables (EPI_QKV_ROTARY)
    const f16* sinv;
    f16* out[6];       // EPI_BIAS: out[0] [m, n]; QKV: q0 k0 v0 q1 k1 v1; SPLIT2: a0 a1 b0 b1
    int m, n, k;
    int heads, n0, n1; // per-image split: m = pairs x (n0 + n1) rows, pair-major (n0 of image 0, n1 of image 1)
    int mtiles, total;
};

// Row `row` of the stacked rows -> its image and the offset of its head-h segment in that image's
// [pairs, heads, ni, 64] tensor
struct LinRow {
    bool first;
    size_t off;
};
__device__ __forceinline__ LinRow lin_row(const LinArgs& p, int row, int h) {
    const int ntot = p.n0 + p.n1;
    const int pr = row / ntot, l = row - pr * ntot;
    const bool first = l < p.n0;
    const int r = first ? l : l - p.n0, nn = first ? p.n0 : p.n1;
    return {first, (((size_t)pr * p.heads + h) * nn + r) * kD};
}

// global source of A row `row`, 16-B unit `gc` (8 k values)
template <bool GATHER>
__device__ __forceinline__ const f16* a_src(const LinArgs& p, int row, int gc) {
    if constexpr (!GATHER) {
        return p.a + (size_t)row * p.k + gc * 8;
    } else {
        const int half = p.k / 2, col = gc * 8;
        if (col < half) return p.a + (size_t)row * half + col;  // x
        const int c2 = col - half, h = c2 / kD, d = c2 % kD;
        const LinRow lr = lin_row(p, row, h);
        return (lr.first ? p.ctx0 : p.ctx1) + lr.off + d;
    }
}

// The projections' output arithmetic, shared by every form (so every form gives the same bits): the
// GEMM value plus bias is rounded to fp16 once (F.linear's fp16 output, lightglue.py:97-122); the
// residual add and the rotary (lightglue.py:124-134) then work from that value, as the reference's
// fp16 model does (x + ffn(...): fp32 with one rounding; q * cos + rotate(q) * sin: fp16 products
// and sum, rot_pair).
__device__ __forceinline__ f16 lin_val(float acc, f16 b) { return (f16)(acc + (float)b); }
__device__ __forceinline__ f16 res_add(f16 v, f16 r) { return (f16)((float)v + (float)r); }
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

// (x0, x1) of a rotary pair (d, d + 1) -> (x0 c0 - x1 s0, x1 c1 + x0 s1), elements e, e + 1 of v,
// in fp16 arithmetic as the reference's fp16 model evaluates t * cos + rotate_half(t) * sin
// (lightglue.py:124-134): each product and the sum rounded to fp16 (packed v_pk_mul_f16 /
// v_pk_add_f16, no contraction into an fma)
typedef f16 f16x2 __attribute__((ext_vector_type(2)));
template <typename V>
__device__ __forceinline__ void rot_pair(V& v, int e, f16 c0, f16 s0, f16 c1, f16 s1) {
#pragma clang fp contract(off)
    const f16x2 x = f16x2{v[e], v[e + 1]};
    const f16x2 xr = f16x2{-v[e + 1], v[e]};
    const f16x2 o = x * f16x2{c0, c1} + xr * f16x2{s0, s1};
    v[e] = o[0];
    v[e + 1] = o[1];
}

// Mixed-precision FMAs for the one-launch LayerNorm epilogue (fp16 operands read in place, halves
// chosen by op_sel): mixf(x, g, b) = x * g + b in fp32 with g, b the HI-th halves of packed fp16
// words; mixh(acc, b) = fp16(acc + b), rounded once (the two-launch path's lin_val rounds to fp32
// first: the forms agree within the rare double-rounding ulp, not in every bit).
template <int HI>
__device__ __forceinline__ float mixf(float x, unsigned g2, unsigned b2) {
    float r;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[0,1,1]" : "=v"(r) : "v"(x), "v"(g2), "v"(b2));
    else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(x), "v"(g2), "v"(b2));
    return r;
}
// The packed forms (round 6): h2 = (fp16(acc0 + b.lo), fp16(acc1 + b.hi)) in one register, each half
// rounded once as mixh does; mixn(h2, a, c) = h2's HI-th half * a + c in fp32 (the LayerNorm's
// normalisation read straight from the packed fp16 values)
__device__ __forceinline__ unsigned mixh2(float acc0, float acc1, unsigned b2) {
    unsigned h;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, %2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, 1.0, %2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(h)
        : "v"(acc0), "v"(b2), "v"(acc1));
    return h;
}
template <int HI>
__device__ __forceinline__ float mixn(unsigned h2, float a, float c) {
    float r;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(a), "v"(c));
    else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h2), "v"(a), "v"(c));
    return r;
}
// the row sums of one packed pair: s1 += h.lo + h.hi, s2 += h.lo^2 + h.hi^2 (v_dot2_f32_f16: the f16
// products exact in fp32)
__device__ __forceinline__ void row_sums2(unsigned h2, float& s1, float& s2) {
    const f16x2 h = __builtin_bit_cast(f16x2, h2);
    s1 = __builtin_amdgcn_fdot2(h, f16x2{(f16)1.f, (f16)1.f}, s1, false);
    s2 = __builtin_amdgcn_fdot2(h, h, s2, false);
}
template <int HI>
__device__ __forceinline__ float mixh(float acc, unsigned b2) {
    unsigned h;
    if constexpr (HI) asm("v_fma_mixlo_f16 %0, %1, 1.0, %2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(h) : "v"(acc), "v"(b2));
    else asm("v_fma_mixlo_f16 %0, %1, 1.0, %2 op_sel_hi:[0,0,1]" : "=v"(h) : "v"(acc), "v"(b2));
    return (float)__builtin_bit_cast(f16x2, h)[0];
}

template <int EPI, bool GATHER, int KC>
__global__ __launch_bounds__(256) void linear_kernel(LinArgs p) {
    static_assert(KC == 2 || KC == 4, "k = 256 or 512");
    __shared__ __attribute__((aligned(16))) char smem[2 * KC * kChunkBytes];  // W, A tiles (64 / 128 KiB)
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;  // this wave's 32 x 32 tile of the 64 x 64
    const int r = lane & 31, hh = lane >> 5;
    // XCD-aware order: consecutive j (one XCD) = consecutive m tiles of one n tile (W tile in L2)
    int j;
    {
        const int T = p.total, L = blockIdx.x, q8 = T >> 3, r8 = T & 7, xcd = L & 7;
        j = xcd * q8 + min(xcd, r8) + (L >> 3);
    }
    const int mt = j % p.mtiles, nt = j / p.mtiles;
    const int m0 = mt * kBM, n0 = nt * kBN;
    const unsigned wbase = 0, abase = KC * kChunkBytes;
    const int wrow = wn * 32 + r, arow = wm * 32 + r;
    const int m = min(m0 + arow, p.m - 1);  // this lane's output row (clamped; stores are guarded)

    // Epilogue operands first (plain loads, older than every DMA below, so the counted waits
    // of the main loop stay exact): bias, residual / rotary tables of the lane's 4 x 4 channels.
    f16x4 bias4[4], aux0[4], aux1[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 32 + 8 * g + 4 * hh;
        bias4[g] = *reinterpret_cast<const f16x4*>(p.bias + n);
        if constexpr (EPI == EPI_BIAS) {
            if (p.res) aux0[g] = *reinterpret_cast<const f16x4*>(p.res + (size_t)m * p.n + n);
        } else if constexpr (EPI == EPI_QKV_ROTARY) {
            aux0[g] = *reinterpret_cast<const f16x4*>(p.cosv + (size_t)m * kD + n % kD);
            aux1[g] = *reinterpret_cast<const f16x4*>(p.sinv + (size_t)m * kD + n % kD);
        }
    }

    __builtin_amdgcn_sched_barrier(0);  // (they stay ahead of the DMAs)

    // ---- loads: per chunk c, W rows n0.. and A rows m0.. ; one DMA = 4 rows x 256 B ----
    // lane -> (row 4i + lane/16, LDS unit lane%16 <- global unit (lane%16) ^ (row & 15))
    // Wave w issues DMA instructions i = w, w+4, w+8, w+12 of each 16-instruction chunk tile.
#pragma unroll
    for (int c = 0; c < KC; ++c) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int i = wave + 4 * s;
            const int row = 4 * i + (lane >> 4), pu = lane & 15;
            const int gc = c * (kKC / 8) + (pu ^ (row & 15));
            const int wr = min(n0 + row, p.n - 1);
            __builtin_amdgcn_global_load_lds((const void*)(p.w + (size_t)wr * p.k + gc * 8),
                                             (__attribute__((address_space(3))) void*)(smem + wbase + c * kChunkBytes + i * 1024),
                                             16, 0, 0);
            const int ar = min(m0 + row, p.m - 1);
            __builtin_amdgcn_global_load_lds((const void*)a_src<GATHER>(p, ar, gc),
                                             (__attribute__((address_space(3))) void*)(smem + abase + c * kChunkBytes + i * 1024),
                                             16, 0, 0);
        }
    }

    f32x16 acc = {};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
        // chunk c landed for this wave's DMAs (8 per chunk, in issue order), then for everyone's
        switch (KC - 1 - c) {
            case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
            case 1: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
            case 2: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        }
        __builtin_amdgcn_s_barrier();
        const unsigned wc = wbase + c * kChunkBytes + wrow * 256, ac = abase + c * kChunkBytes + arow * 256;
        // all 8 k-steps' fragments of the chunk first (one LDS latency per chunk, not per step)
        f16x8 wf[kKC / 16], af[kKC / 16];
#pragma unroll
        for (int s = 0; s < kKC / 16; ++s) {
            const int u = 2 * s + hh;  // 16-B unit of the k-step
            wf[s] = *(lds_f16x8*)(lds + wc + ((u ^ (wrow & 15)) << 4));
            af[s] = *(lds_f16x8*)(lds + ac + ((u ^ (arow & 15)) << 4));
        }
#pragma unroll
        for (int s = 0; s < kKC / 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[s], af[s], acc, 0, 0, 0);
    }

    // ---- epilogue: lane = activation row m; acc[4g + t] = channel n0 + wn*32 + 8g + 4hh + t ----
    if (m0 + arow >= p.m) return;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 32 + 8 * g + 4 * hh;  // 4 consecutive channels n..n+3
        f16x4 v;
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = lin_val(acc[4 * g + t], bias4[g][t]);
        if constexpr (EPI == EPI_BIAS) {
            if (p.res) {
#pragma unroll
                for (int t = 0; t < 4; ++t) v[t] = res_add(v[t], aux0[g][t]);
            }
            *reinterpret_cast<f16x4*>(p.out[0] + (size_t)m * p.n + n) = v;
        } else {
            const int hd = p.heads * kD;
            const int part = n / hd, h = (n % hd) / kD, d = n % kD;
            const LinRow lr = lin_row(p, m, h);
            const bool first = lr.first;
            if constexpr (EPI == EPI_QKV_ROTARY) {
                if (part < 2) {  // q, k: (x0, x1) -> (x0 c - x1 s, x1 c + x0 s), pairs (d, d+1)
                    const f16x4 cc = aux0[g], ss = aux1[g];
#pragma unroll
                    for (int t = 0; t < 4; t += 2) rot_pair(v, t, cc[t], ss[t], cc[t + 1], ss[t + 1]);
                }
            }
            f16* dst = p.out[(first ? 0 : (EPI == EPI_QKV_ROTARY ? 3 : 1)) + (EPI == EPI_QKV_ROTARY ? part : 2 * part)];
            *reinterpret_cast<f16x4*>(dst + lr.off + d) = v;
        }
    }
}

// ---- per-tile DMA sources of the 256-row forms: each wave's W and A pieces of a tile, computed once
// per tile (row clamps, the swizzled unit, the A-gather's image and head-major offset) so that a K
// step's DMA is one address add per piece. BK-deep steps: a 1-KiB piece is 1024 / (2 BK) rows; lane
// -> (row RP i + lane / U, LDS unit lane % U <- global unit (lane % U) ^ swz(row)), U = BK / 8 units a row
template <int NWP, int NAP>
struct TileSrc {
    const f16* w[NWP];
    const f16* a[NAP];  // A rows (the gather: x rows)
    const f16* c[NAP];  // the gather: head 0 of the row in its image's [pairs, heads, ni, 64] tensor
    int hs[NAP];        // the gather: elements between heads there (ni * 64)
};
template <int BK>
__device__ __forceinline__ int src_unit(int row, int pos) {
    return BK == 64 ? (pos ^ ((row >> 1) & 7)) : (pos ^ ((row >> 2) & 3));
}
// (LW waves issue a stage's DMA pieces: piece wave + LW h)
template <bool GATHER, int BK, int NWP, int NAP, int LW>
__device__ __forceinline__ TileSrc<NWP, NAP> tile_src(const LinArgs& p, int m0, int n0, int wave, int lane) {
    constexpr int U = BK / 8, RP = 1024 / (2 * BK);
    TileSrc<NWP, NAP> t;
#pragma unroll
    for (int h = 0; h < NWP; ++h) {
        const int row = RP * (wave + LW * h) + lane / U;
        const int wr = min(n0 + row, p.n - 1);
        t.w[h] = p.w + (size_t)wr * p.k + src_unit<BK>(row, lane % U) * 8;
    }
#pragma unroll
    for (int h = 0; h < NAP; ++h) {
        const int row = RP * (wave + LW * h) + lane / U;
        const int ar = min(m0 + row, p.m - 1);
        const int gu8 = src_unit<BK>(row, lane % U) * 8;
        if constexpr (!GATHER) {
            t.a[h] = p.a + (size_t)ar * p.k + gu8;
        } else {
            t.a[h] = p.a + (size_t)ar * (p.k / 2) + gu8;
            const LinRow lr = lin_row(p, ar, 0);
            t.c[h] = (lr.first ? p.ctx0 : p.ctx1) + lr.off + gu8;
            t.hs[h] = (lr.first ? p.n0 : p.n1) * kD;
        }
    }
    return t;
}
// K step ks (compile-time after unrolling; K = KS BK) of a tile into the stage at sb: W pieces
// wave + LW h at sb, A pieces at sb + BN BK 2
template <bool GATHER, int BK, int KS, int BN, int LW, int NWP, int NAP>
__device__ __forceinline__ void tile_issue(const TileSrc<NWP, NAP>& t, int ks, char* sb, int wave) {
#pragma unroll
    for (int h = 0; h < NWP; ++h)
        __builtin_amdgcn_global_load_lds((const void*)(t.w[h] + ks * BK),
                                         (__attribute__((address_space(3))) void*)(sb + (wave + LW * h) * 1024), 16, 0, 0);
#pragma unroll
    for (int h = 0; h < NAP; ++h) {
        const f16* src;
        if constexpr (!GATHER) {
            src = t.a[h] + ks * BK;
        } else {
            constexpr int half = KS * BK / 2;
            const int col = ks * BK;
            src = col < half ? t.a[h] + col : t.c[h] + ((col - half) / kD) * t.hs[h] + (col - half) % kD;
        }
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(sb + BN * BK * 2 + (wave + LW * h) * 1024),
                                         16, 0, 0);
    }
}

// ---- the 256-row forms, for launches with many rows (several image pairs per forward) ----
// Persistent tiles of MT rows x NT channels (256 x 128 or 256 x 256 on 8 waves, 128 x 128 on 4), NWV waves as WM (m) x
// WN (n) tiles of 64 rows x NT / WN channels (2 x NB MFMA blocks of 32 x 32), K in BK-deep steps through
// an NST-stage LDS-DMA ring (16-B units XOR-swizzled on the source address: conflict-free
// ds_read_b128), NST - 1 steps in flight; the ring runs on across tile seams, so the next tile's
// first steps load during the current tile's last ones. XCD-aware: the workgroups of XCD x walk the
// contiguous tile range [jb, je) (tile j = m tile j / ntiles, n tile j % ntiles: the n tiles of one
// m tile run side by side on one XCD and read its A rows through one L2).
//
// Epilogue (round 5): the MFMA layout puts one activation row on each lane, so stores straight from
// the accumulators write 32 rows x 16-32 B per wave instruction; measured (ablations of the round-4
// forms, profiles/r05/linear_ablations.jsonl) those stores cost more than the GEMM: lg_linear_qkv_rotary
// 53.6 us with them, 15.9 without. Here each wave rounds (acc + bias) to fp16 into its own 4 KiB
// region of the ring stage its tile's last K step has just freed (one barrier per tile), 32 rows x
// 64 channels a round, reads it back row-major and writes whole 128-B row segments: 8 rows x 128 B
// per wave instruction, the residual / rotary tables loaded in the same coalesced layout (prefetched
// at the tile's last K step). The stores stay in flight into the next tile: its first NST - 1 waits
// count them (every lane stores; rows past m are computed on the clamped last A row and write that
// row's own bytes again, so the count is exact).
// RES (EPI_BIAS): p.res is added (a compile-time form: its prefetch holds registers).
template <int EPI, bool GATHER, bool RES, int KS, int MT, int NT, int BK, int NST, int NWV = 8>
__global__ __launch_bounds__(64 * NWV, NWV == 4 ? 2 : 1) void linear_tile_kernel(LinArgs p) {
    constexpr int WM = MT / 64, WN = NWV / WM, WTN = NT / WN, NB = WTN / 32, NP = WTN / 64;
    constexpr int SB = (MT + NT) * BK * 2;                               // one ring stage
    constexpr int NWP = NT * BK * 2 / (NWV * 1024), NAP = MT * BK * 2 / (NWV * 1024);  // 1-KiB DMA pieces per wave, step
    constexpr int D = NWP + NAP;
    constexpr int SPW = 2 * NP * 4;                                      // output stores per wave and tile
    // epilogue operands loaded per wave and tile (at its first K step): bias, residual / cos + sin rows
    constexpr int PF = NB * 4 + (RES ? 2 * NP * 4 : 0) + (EPI == EPI_QKV_ROTARY ? 16 : 0);
    static_assert(SB >= NWV * 4096, "a staging region per wave inside one ring stage");
    static_assert(KS >= NST - 1 && NB % 2 == 0 && (NST - 2) * D + SPW + PF <= 63, "shape");
    static_assert(NB == 2 || (EPI != EPI_QKV_ROTARY && !RES), "64 x 128 wave tiles: no room for the prefetched tables");
    __shared__ __attribute__((aligned(16))) char smem[NST * SB];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int r = lane & 31, hh = lane >> 5;
    const int T = p.total, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8), je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    const int ntiles = p.n / NT;
    const int j0 = jb + loc;
    if (j0 >= je) return;
    const int ntile_w = (je - j0 + G - 1) / G;
    const int nsteps = ntile_w * KS;

    auto src_of = [&](int t) {
        const int jt = j0 + G * t, mt = jt / ntiles;
        return tile_src<GATHER, BK, NWP, NAP, NWV>(p, mt * MT, (jt - mt * ntiles) * NT, wave, lane);
    };
    TileSrc<NWP, NAP> cur = src_of(0), nxt = cur;
#pragma unroll
    for (int i = 0; i < NST - 1; ++i)
        tile_issue<GATHER, BK, KS, NT, NWV>(cur, i, smem + i * SB, wave);

    // fragment rows of this lane: W rows wn * WTN + 32 b + r, A rows wm * 64 + 32 b + r
    auto swz = [](int row) { return BK == 64 ? (row >> 1) & 7 : (row >> 2) & 3; };
    unsigned wro[NB], aro[2];
    int wsw[NB], asw[2];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int wrow = wn * WTN + 32 * b + r;
        wro[b] = (unsigned)(wrow * BK * 2), wsw[b] = swz(wrow);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int arow = wm * 64 + 32 * b + r;
        aro[b] = (unsigned)(NT * BK * 2 + arow * BK * 2), asw[b] = swz(arow);
    }
    // coalesced phase: lane -> (row 8 i + lane / 8 of a 32-row round, 16-B chunk lane % 8 of 64 channels)
    const int cr = lane >> 3, cc = lane & 7;
    int st = 0;
    for (int t = 0; t < ntile_w; ++t) {
        const int jt = j0 + G * t;
        const int mt = jt / ntiles, m0 = mt * MT, n0 = (jt - mt * ntiles) * NT;
        const int nw0 = n0 + wn * WTN;  // this wave's first channel
        const bool more = t + 1 < ntile_w;
        if (more) nxt = src_of(t + 1);
        f32x16 acc[NB][2] = {};
        f16x4 bias4[NB][4];
        f16x8 aux[2][NP][4];  // residual rows (EPI_BIAS) / cos rows (QKV) of the coalesced phase
        f16x8 aux2[2][4];     // sin rows (QKV)
        int st_last = 0;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int gs = t * KS + ks;
            // step gs landed (this wave's pieces: younger ones = the later steps' DMAs in flight,
            // plus the previous tile's output stores while they are younger), then everyone's; past
            // this barrier every wave is done with step gs - 1's stage
            // Younger than step gs's pieces: the later steps' DMA in flight; the previous tile's output
            // stores while issued after gs's DMA (ks < NST - 1); this tile's epilogue operands,
            // loaded at ks = 0 after that step's wait (1 <= ks <= NST - 2). (The workgroup's last
            // NST - 2 steps have fewer later steps in flight: drain all.)
            const bool pfk = ks >= 1 && ks <= NST - 2;  // (folded after unrolling)
            if (gs + NST - 2 > nsteps - 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else if (ks < NST - 1 && t > 0) {
                if (pfk) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D + SPW + PF) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D + SPW) : "memory");
            } else {
                if (pfk) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D + PF) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D) : "memory");
            }
            __builtin_amdgcn_s_barrier();
            if (ks == 0) {
                // the epilogue's operands, a whole tile ahead of their use (rows clamped to m - 1, as
                // the A rows are; the rotary tables for the v part too: a fixed count for the waits)
#pragma unroll
                for (int b = 0; b < NB; ++b)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        bias4[b][g] = *reinterpret_cast<const f16x4*>(p.bias + nw0 + 32 * b + 8 * g + 4 * hh);
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = min(m0 + wm * 64 + 32 * mb + 8 * i + cr, p.m - 1);
                        if constexpr (EPI == EPI_BIAS && RES) {
#pragma unroll
                            for (int np = 0; np < NP; ++np)
                                aux[mb][np][i] = *reinterpret_cast<const f16x8*>(p.res + (size_t)row * p.n + nw0 + 64 * np + 8 * cc);
                        } else if constexpr (EPI == EPI_QKV_ROTARY) {
                            aux[mb][0][i] = *reinterpret_cast<const f16x8*>(p.cosv + (size_t)row * kD + 8 * cc);
                            aux2[mb][i] = *reinterpret_cast<const f16x8*>(p.sinv + (size_t)row * kD + 8 * cc);
                        }
                    }
            }
            {
                char* const fb = smem + (st == 0 ? NST - 1 : st - 1) * SB;
                if (ks + NST - 1 < KS) tile_issue<GATHER, BK, KS, NT, NWV>(cur, ks + NST - 1, fb, wave);
                else if (more) tile_issue<GATHER, BK, KS, NT, NWV>(nxt, ks + NST - 1 - KS, fb, wave);
            }
            const unsigned sb = (unsigned)(st * SB);
            st_last = st;
            st = st == NST - 1 ? 0 : st + 1;
#pragma unroll
            for (int s = 0; s < BK / 16; ++s) {
                const int u = 2 * s + hh;
                f16x8 wf[NB], af[2];
#pragma unroll
                for (int b = 0; b < NB; ++b) wf[b] = *(lds_f16x8*)(lds + sb + wro[b] + ((u ^ wsw[b]) << 4));
#pragma unroll
                for (int b = 0; b < 2; ++b) af[b] = *(lds_f16x8*)(lds + sb + aro[b] + ((u ^ asw[b]) << 4));
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb)
                        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[nb], af[mb], acc[nb][mb], 0, 0, 0);
            }
        }

        // ---- epilogue: the operands loaded at ks = 0 landed (younger: this tile's KS DMA issues when
        // another tile follows; a count capped at 63 only waits for more); every wave's fragment reads
        // of the last stage done (barrier) ----
        if (more) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(KS * D < 63 ? KS * D : 63) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        lds_char* const stg = lds + st_last * SB + wave * 4096;
        const int hd = p.heads * kD;
        // Head-major outputs (QKV / SPLIT2): rows rb + 32 mb + 8 i of the coalesced phase, split
        // into (pair, row of the pair) with one division per tile and a step per row (pairs of
        // more than 56 rows here, tile_form: one wrap at most); rows past m take row m - 1's
        // place, as their A rows did.
        const int ntot = p.n0 + p.n1;
        const int rb = m0 + wm * 64 + cr;
        const int pr0 = rb / ntot, l0 = rb - pr0 * ntot;
        const int prl = (p.m - 1) / ntot, ll = p.m - 1 - prl * ntot;
        auto split_row = [&](int o, int& pr, int& l) {
            pr = pr0, l = l0 + o;
            if (l >= ntot) l -= ntot, ++pr;
            if (rb + o > p.m - 1) pr = prl, l = ll;
        };
        // (the common tile: no lane's rows rb .. rb + 56 cross an image, pair or m boundary, so row
        // o's offset is row 0's + 64 o in the same image: wave-uniform)
        const bool img0 = l0 < p.n0;
        const bool span = (img0 ? l0 + 56 < p.n0 : l0 + 56 < ntot) && rb + 56 <= p.m - 1;
        const bool easy = __builtin_amdgcn_ballot_w64(!span) == 0;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int np = 0; np < NP; ++np) {
                // (acc + bias) -> fp16, rows r of the round, 16-B chunk (4 nbl + g) ^ (r & 7), half hh
#pragma unroll
                for (int nbl = 0; nbl < 2; ++nbl)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f32x16& a = acc[2 * np + nbl][mb];
                        const f16x4 b4 = bias4[2 * np + nbl][g];
                        const f16x4 v = f16x4{lin_val(a[4 * g], b4[0]), lin_val(a[4 * g + 1], b4[1]),
                                              lin_val(a[4 * g + 2], b4[2]), lin_val(a[4 * g + 3], b4[3])};
                        *(__attribute__((address_space(3))) f16x4*)(stg + r * 128 + (((4 * nbl + g) ^ (r & 7)) << 4) + 8 * hh) = v;
                    }
                f16x8 o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rl = 8 * i + cr;
                    o[i] = *(lds_f16x8*)(stg + rl * 128 + ((cc ^ (rl & 7)) << 4));
                }
                if constexpr (EPI == EPI_BIAS) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = min(m0 + wm * 64 + 32 * mb + 8 * i + cr, p.m - 1);
                        const int n = nw0 + 64 * np + 8 * cc;  // 8 consecutive channels n..n+7
                        f16x8 v = o[i];
                        if constexpr (RES) {
#pragma unroll
                            for (int e = 0; e < 8; ++e) v[e] = res_add(v[e], aux[mb][np][i][e]);
                        }
                        st_out(p.out[0] + (size_t)row * p.n + n, v);
                    }
                } else {
                    // the wave's 64 channels lie in one head of one part (nw0 + 64 np and hd are
                    // multiples of 64): part, head and the two images' destinations are wave-uniform
                    const int nu = __builtin_amdgcn_readfirstlane(nw0 + 64 * np);
                    const int part = nu / hd, h = (nu - part * hd) / kD;
                    f16* d0;
                    f16* d1;
                    if constexpr (EPI == EPI_QKV_ROTARY) {
                        d0 = part == 0 ? p.out[0] : part == 1 ? p.out[1] : p.out[2];
                        d1 = part == 0 ? p.out[3] : part == 1 ? p.out[4] : p.out[5];
                    } else {
                        d0 = part == 0 ? p.out[0] : p.out[2];
                        d1 = part == 0 ? p.out[1] : p.out[3];
                    }
                    // element offsets in [pairs, heads, ni, 64]: pair stride, head h's first row + d
                    const unsigned ps0 = (unsigned)(p.heads * p.n0 * kD), ps1 = (unsigned)(p.heads * p.n1 * kD);
                    const unsigned hb0 = (unsigned)(h * p.n0 * kD + 8 * cc), hb1 = (unsigned)(h * p.n1 * kD + 8 * cc);
                    f16* const db = img0 ? d0 : d1;
                    const unsigned ob = img0 ? (unsigned)pr0 * ps0 + (unsigned)l0 * kD + hb0
                                             : (unsigned)pr0 * ps1 + (unsigned)(l0 - p.n0) * kD + hb1;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        f16x8 v = o[i];
                        if constexpr (EPI == EPI_QKV_ROTARY) {
                            if (part < 2) {
#pragma unroll
                                for (int e = 0; e < 8; e += 2)
                                    rot_pair(v, e, aux[mb][0][i][e], aux2[mb][i][e], aux[mb][0][i][e + 1], aux2[mb][i][e + 1]);
                            }
                        }
                        if (easy) {
                            st_out(db + ob + (unsigned)((32 * mb + 8 * i) * kD), v);
                            continue;
                        }
                        int pr, l;
                        split_row(32 * mb + 8 * i, pr, l);
                        const bool first = l < p.n0;
                        const unsigned off = first ? (unsigned)pr * ps0 + (unsigned)l * kD + hb0
                                                   : (unsigned)pr * ps1 + (unsigned)(l - p.n0) * kD + hb1;
                        st_out((first ? d0 : d1) + off, v);
                    }
                }
            }
        cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- the FFN input projection with LayerNorm + GELU in its epilogue (lg_linear_cat_ln_gelu) ----
// LightGlue's FFN (lightglue.py:101-106) is Linear(2d, 2d) -> LayerNorm(2d) -> GELU -> Linear(2d, d):
// lg_linear_cat writes h = [x | heads]·Wᵀ + b, a separate pass normalises it (17 us at P = 16, M =
// 32,768: 33.5 MB read, 33.5 MB written; profiles/r05/matcher_p16_kernel_stats_tile_forms_v1.csv).
// Here a workgroup owns whole rows: tiles of 128 rows x all 512 channels (8 waves as 2 (m) x 4 (n)
// tiles of 64 x 128; K in 32-deep steps through a 3-stage LDS-DMA ring of 40 KiB stages, the A-gather
// of lg_linear_cat), so the row statistics close inside the workgroup: h = fp16(acc + bias) as the
// unfused path rounds it, row sums per wave -> LDS -> mean; sums of (h - mean)^2 -> LDS -> variance
// (two passes over registers: the unfused kernel's E[h^2] - mean^2 cancels less well), then
// GELU(LN(h)) (the erf of A&S 7.1.26, as the unfused fp16 kernel) rounded to fp16, staged and
// stored as in linear_tile_kernel. bias, gamma and beta sit in LDS for the whole launch.
// Diagnostic build (-DLG_LN_STAMPS, tools/ln_stamps.py; never shipped): per wave, s_memtime cycles
// of linear_ln_kernel by chained segment (0 prologue, 1 K-step waits + barriers, 2 K-step DMA issue +
// fragment reads + MFMAs, 3 epilogue: h and row statistics, 4 epilogue: normalise, GELU, staging,
// stores), read back by lg_diag_ln_stamps.
#ifdef LG_LN_STAMPS
__device__ unsigned long long g_ln_stamps[256 * 8 * 8];
#define LN_SEG(k)                                                                                    \
    do {                                                                                             \
        unsigned long long t_;                                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        sg_[k] += t_ - last_;                                                                        \
        last_ = t_;                                                                                  \
    } while (0)
#else
#define LN_SEG(k) \
    do {          \
    } while (0)
#endif
constexpr int kLnN = 512;
// the one-launch form's two tiles: 128 rows with 32-deep K steps through 3 stages of 40 KiB, and
// 64 rows with 64-deep K steps through 2 stages of 72 KiB (twice the W bytes per row: it pays only
// while the 128-row tiles would leave CUs idle; see lg_linear_cat_ln_gelu)
template <int KS, int MT, int BK, int NST, int NWV = 8>
__global__ __launch_bounds__(64 * NWV, NWV == 4 ? 2 : 1) void linear_ln_kernel(LinArgs p, const f16* __restrict__ gamma,
                                                                              const f16* __restrict__ beta, float eps) {
    constexpr int NT = kLnN;
    constexpr int WM = MT / 64, WN = NWV / WM, WTN = NT / WN, NB = WTN / 32, NP = WTN / 64;
    constexpr int SB = (MT + NT) * BK * 2;                             // 40 KiB
    constexpr int NWP = NT * BK * 2 / (NWV * 1024), NAP = MT * BK * 2 / (NWV * 1024);  // pieces per wave and step
    constexpr int D = NWP + NAP;
    constexpr int SPW = 2 * NP * 4;
    constexpr int kPar = NST * SB;                  // vectors: bias, gamma, beta [512] fp16
    constexpr int kRed = kPar + 3 * NT * 2;         // row partials [2][MT][WN] fp32
    static_assert((NST - 2) * D + SPW <= 63 && KS >= NST - 1, "shape");
    __shared__ __attribute__((aligned(16))) char smem[kRed + 2 * MT * WN * 4];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int r = lane & 31, hh = lane >> 5;
    const int T = p.total, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8), je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    const int j0 = jb + loc;
    if (j0 >= je) return;
    const int ntile_w = (je - j0 + G - 1) / G;
    const int nsteps = ntile_w * KS;
#ifdef LG_LN_STAMPS
    unsigned long long sg_[5] = {0, 0, 0, 0, 0}, last_, t_entry_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry_)::"memory");
    last_ = t_entry_;
#endif

    auto src_of = [&](int t) { return tile_src<true, BK, NWP, NAP, NWV>(p, (j0 + G * t) * MT, 0, wave, lane); };
    // the vectors into LDS (loaded ahead of the first stages, written after them: the compiler's wait
    // counts the DMA pieces), visible after the first step's barrier
    f16x8 pv = {};
    const f16* const pvs = tid < 64 ? p.bias : tid < 128 ? gamma : beta;
    if (tid < 192) pv = *reinterpret_cast<const f16x8*>(pvs + (tid & 63) * 8);
    TileSrc<NWP, NAP> cur = src_of(0);  // (the next tile's sources are computed where used: registers)
#pragma unroll
    for (int i = 0; i < NST - 1; ++i) tile_issue<true, BK, KS, NT, NWV>(cur, i, smem + i * SB, wave);
    if (tid < 192) *(lds_f16x8*)(lds + kPar + tid * 16) = pv;

    auto swz = [](int row) { return BK == 64 ? (row >> 1) & 7 : (row >> 2) & 3; };
    unsigned wro[NB], aro[2];
    int wsw[NB], asw[2];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int wrow = wn * WTN + 32 * b + r;
        wro[b] = (unsigned)(wrow * BK * 2), wsw[b] = swz(wrow);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int arow = wm * 64 + 32 * b + r;
        aro[b] = (unsigned)(NT * BK * 2 + arow * BK * 2), asw[b] = swz(arow);
    }
    const int cr = lane >> 3, cc = lane & 7;
    float* const red = (float*)(void*)(smem + kRed);  // [pass][row][wn]
    auto red_sum = [&](int off) {  // the WN partials of a row, in a fixed order
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < WN; q += 4) {
            const f32x4 w4 = *(__attribute__((address_space(3))) f32x4*)(lds + kRed + (off + q) * 4);
            v += (w4[0] + w4[1]) + (w4[2] + w4[3]);
        }
        return v;
    };
    int st = 0;
    for (int t = 0; t < ntile_w; ++t) {
        const int m0 = (j0 + G * t) * MT;
        const bool more = t + 1 < ntile_w;
        f32x16 acc[NB][2] = {};
        int st_last = 0;
#pragma unroll 2
        for (int ks = 0; ks < KS; ++ks) {
            const int gs = t * KS + ks;
            if (ks == 0 && t == 0) LN_SEG(0);
            else LN_SEG(2);
            if (gs + NST - 2 > nsteps - 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            else if (ks < NST - 1 && t > 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D + SPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NST - 2) * D) : "memory");
            __builtin_amdgcn_s_barrier();
            LN_SEG(1);
            {
                char* const fb = smem + (st == 0 ? NST - 1 : st - 1) * SB;
                if (ks + NST - 1 < KS) tile_issue<true, BK, KS, NT, NWV>(cur, ks + NST - 1, fb, wave);
                else if (more) tile_issue<true, BK, KS, NT, NWV>(src_of(t + 1), ks + NST - 1 - KS, fb, wave);
            }
            const unsigned sb = (unsigned)(st * SB);
            st_last = st;
            st = st == NST - 1 ? 0 : st + 1;
#pragma unroll
            for (int s = 0; s < BK / 16; ++s) {
                const int u = 2 * s + hh;
                f16x8 wf[NB], af[2];
#pragma unroll
                for (int b = 0; b < NB; ++b) wf[b] = *(lds_f16x8*)(lds + sb + wro[b] + ((u ^ wsw[b]) << 4));
#pragma unroll
                for (int b = 0; b < 2; ++b) af[b] = *(lds_f16x8*)(lds + sb + aro[b] + ((u ^ asw[b]) << 4));
#pragma unroll
                for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb)
                        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[nb], af[mb], acc[nb][mb], 0, 0, 0);
            }
        }

        LN_SEG(2);
        // ---- epilogue: h = fp16(acc + bias) (lane: row wm*64 + 32 mb + r, 64 of the wave's channels) ----
        const int nw0 = wn * WTN;
        float rs[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            float s = 0.f;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const u32x2 b4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + (nw0 + 32 * nb + 8 * g + 4 * hh) * 2);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float a = acc[nb][mb][4 * g + u];
                        const float h = (u & 1) ? mixh<1>(a, b4[u >> 1]) : mixh<0>(a, b4[u >> 1]);
                        acc[nb][mb][4 * g + u] = h;
                        s += h;
                    }
                }
            rs[mb] = s + __shfl_xor(s, 32, 64);  // the wave's 128 channels of the row
        }
        // row sums across the 4 n-waves (this tile's partials: every wave is past the last K step's
        // reads once it reaches the barrier below, and past the previous tile's statistics reads)
        if (hh == 0) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) red[(wm * 64 + 32 * mb + r) * WN + wn] = rs[mb];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        float mean[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            mean[mb] = red_sum((wm * 64 + 32 * mb + r) * WN) * (1.f / kLnN);
            float q = 0.f;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float d = acc[nb][mb][e] - mean[mb];
                    acc[nb][mb][e] = d;  // (h - mean, reused by the normalisation)
                    q = __builtin_fmaf(d, d, q);
                }
            rs[mb] = q + __shfl_xor(q, 32, 64);
        }
        if (hh == 0) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) red[MT * WN + (wm * 64 + 32 * mb + r) * WN + wn] = rs[mb];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // (also: every wave is done reading the last stage)
        LN_SEG(3);
        lds_char* const stg = lds + st_last * SB + wave * 4096;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const float rstd = __builtin_amdgcn_rsqf(red_sum(MT * WN + (wm * 64 + 32 * mb + r) * WN) * (1.f / kLnN) + eps);
#pragma unroll
            for (int np = 0; np < NP; ++np) {
#pragma unroll
                for (int nbl = 0; nbl < 2; ++nbl)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int n = nw0 + 64 * np + 32 * nbl + 8 * g + 4 * hh;
                        const u32x2 g4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + NT * 2 + n * 2);
                        const u32x2 b4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + 2 * NT * 2 + n * 2);
                        f16x4 o;
#pragma unroll
                        for (int u = 0; u < 4; u += 2) {
                            const f32x16& av = acc[2 * np + nbl][mb];
                            const f32x2 xr = f32x2{av[4 * g + u], av[4 * g + u + 1]} * rstd;
                            const f32x2 gl = gelu_as2(f32x2{mixf<0>(xr[0], g4[u >> 1], b4[u >> 1]), mixf<1>(xr[1], g4[u >> 1], b4[u >> 1])});
                            o[u] = (f16)gl[0];
                            o[u + 1] = (f16)gl[1];
                        }
                        *(__attribute__((address_space(3))) f16x4*)(stg + r * 128 + (((4 * nbl + g) ^ (r & 7)) << 4) + 8 * hh) = o;
                    }
                f16x8 o8[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rl = 8 * i + cr;
                    o8[i] = *(lds_f16x8*)(stg + rl * 128 + ((cc ^ (rl & 7)) << 4));
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = min(m0 + wm * 64 + 32 * mb + 8 * i + cr, p.m - 1);
                    st_out(p.out[0] + (size_t)row * NT + nw0 + 64 * np + 8 * cc, o8[i]);
                }
            }
        }
        if (more) cur = src_of(t + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LN_SEG(4);
#ifdef LG_LN_STAMPS
    if (lane == 0) {
        unsigned long long* d = g_ln_stamps + ((size_t)blockIdx.x * 8 + wave) * 8;
        for (int k = 0; k < 5; ++k) d[k] = sg_[k];
        d[5] = last_ - t_entry_;
        d[6] = (unsigned long long)ntile_w;
    }
#endif
}


constexpr int kFfnOut = 256;  // the FFN's output channels (d)

// ---- the whole FFN in one launch, whole rows per workgroup (lg_linear_cat_ffn, round 6) ----
// out = x + fp16(W2 · GELU(LN(fp16(W1 · [x | heads] + b1))) + b2) with one workgroup per MT = 32 MB rows.
// At a single image pair (M = 1,024..4,096) the FFN was three launches of ~5 us each, every one near
// the launch floor (profiles/r05/single_pair_timelines.txt: 269 of 557 us of a forward at n = 1,024).
// Here one launch: 8 waves, wave w owns hidden channels [64w, 64w + 64) in phase 1 and output
// channels [32w, 32w + 32) in phase 2, so every weight fragment a wave multiplies is its own — W1 and
// W2 stream from L2 straight into VGPRs in the MFMA A-operand layout (lane (r, hh): row r of the
// wave's 32-channel block, k = 16 s + 8 hh .. + 8 of step s; lg_ffn_pack stores them in that order,
// so every load is one contiguous KiB), D steps ahead, as ONE stream that runs from phase 1 into
// phase 2 (W2's first fragments load under the LayerNorm); no barrier in either GEMM loop. The MT
// activation rows [x | heads] (the A-gather of lg_linear_cat) sit in LDS for the whole launch (rows of
// 1 KiB with 16-B units XOR (row & 15): conflict-free ds_read_b128 of 16 rows at one k), as does GELU's
// output h (the second GEMM's B operand, the same layout); the residual x is read back from the A tile.
// Per workgroup the weights are 768 KiB whatever MT (~12 k cycles at the ~64 B/clk a CU takes in):
// MT = 32 (MB = 1) gives the most workgroups for a few rows (latency: single pairs), MT = 64 (MB = 2)
// halves the weight bytes per row where there are rows enough for several rounds (its MFMA work,
// 12 k cycles per SIMD, then matches the stream).
// Arithmetic: the k16 blocks in the 64 x 64 form's order; h = fp16(acc + b1) in one rounding, the
// LayerNorm statistics as lg_layernorm_gelu forms them (sum and sum of squares, fixed reduction order),
// normalisation and GELU as linear_ln_kernel, the output fp16(fp16(acc + b2) + x) as lin_val / res_add.
// phase 3 (lg_linear_cat_ffn_proj): the next attention's projection of the FFN output x'
enum { E3_NONE = 0, E3_SPLIT2 = 1, E3_QKV = 2, E3_PLAIN = 3 };
struct Proj3 {
    const f16* b3;      // [n3] bias
    const f16* cosv;    // E3_QKV: rotary tables [m, 64]
    const f16* sinv;
    f16* out[6];        // SPLIT2: a0 a1 b0 b1; QKV: q0 k0 v0 q1 k1 v1 (per-image head-major); PLAIN: [m, n_store]
    int n_store;        // E3_PLAIN: channels stored per row (the first n_store of 32 NB3 8)
};
// The A tile in two halves (LG_FFN_AHALF, default 1; 0: one tile wait, round 6's first form): the
// x half's loads first, phase 1's first 256 k on it, the heads half written to LDS halfway through.
#ifndef LG_FFN_AHALF
#define LG_FFN_AHALF 1
#endif
// The weight stream's wave sync (A/B, -DLG_FFN_SYNC=<pieces>): a workgroup barrier every that many
// 1-KiB pieces per wave inside each phase, so that no wave runs ahead of the others' streams. The
// waves of a workgroup finish phase 1 ~3.8 k cycles apart (stamps: the LayerNorm's first barrier
// waits for the slowest); with a barrier every 8 pieces 0.5 k apart, but phase 1 itself takes that
// much longer: the CU's stream is bandwidth-bound either way (P = 1 / 4 / 16 FFN 10.0 / 14.6 / 46.0
// us shipped, 10.1 / 15.1 / 46.4 with 8; forwards equal; profiles/r06/ffn_wave_sync_ab.jsonl). Off.
#ifndef LG_FFN_SYNC
#define LG_FFN_SYNC 0
#endif
#define FFN_SYNC(pieces_done, pieces_total)                                                   \
    do {                                                                                      \
        if constexpr (LG_FFN_SYNC > 0) {                                                      \
            if ((pieces_done) % LG_FFN_SYNC == 0 && (pieces_done) < (pieces_total)) __builtin_amdgcn_s_barrier(); \
        }                                                                                     \
    } while (0)
// Diagnostic build (-DLG_FR_STAMPS, tools/fr_stamps.py; never shipped): per wave of the first 256
// workgroups, s_memtime cycles of chained segments (0 entry -> A in LDS, 1 phase 1, 2 LayerNorm + GELU,
// 3 phase 2, 4 epilogue), read back by lg_diag_fr_stamps.
#ifdef LG_FR_STAMPS
__device__ unsigned long long g_fr_stamps[256 * 8 * 8];
#define FR_SEG(k)                                                                                    \
    do {                                                                                             \
        unsigned long long t_;                                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        fr_[k] = t_ - fr_last_;                                                                      \
        fr_last_ = t_;                                                                               \
    } while (0)
#else
#define FR_SEG(k) \
    do {          \
    } while (0)
#endif
template <int MB, int D, int E3, int NB3>
__global__ __launch_bounds__(512, 1) void ffn_rows_kernel(LinArgs p, const f16* __restrict__ gamma,
                                                          const f16* __restrict__ beta, float eps,
                                                          const f16* __restrict__ wp, const f16* __restrict__ b2,
                                                          Proj3 q3) {
    constexpr int MT = 32 * MB;                    // rows per workgroup
    constexpr int K = 512, NO = kFfnOut;           // FFN width (= hidden), output channels
    constexpr int kA = 0, kH = MT * K * 2;         // A and h tiles, [MT][1 KiB] each
    constexpr int kSP = 80;                        // output staging pitch (64 B of a row + 16)
    constexpr int kStg = MB == 1 ? 2 * kH : kH;    // staging: its own region (MB = 1), else over h
    constexpr int kPar = MB == 1 ? kStg + 8 * MT * kSP : 2 * kH;  // b1, gamma, beta [512], b2 [256] fp16
    constexpr int kRed = kPar + (3 * K + NO) * 2;  // row partials [2][MT][8 waves] fp32
    constexpr int NS1 = K / 16, NS = 2 * NS1;      // k16 steps per GEMM; the stream: phase 1, then 2
    constexpr int NS3 = NO / 16;                   // phase 3: k16 steps over x' (K = 256)
    constexpr int NP = 96 + NB3 * NS3;             // the wave's stream: pieces of 1 KiB
    constexpr int R = 2 * D;                       // pieces in flight (a register ring)
    static_assert(D >= 1 && D <= NS1 && (MB == 1 || MB == 2) && (E3 == E3_NONE) == (NB3 == 0), "shape");
    static_assert(MB == 1 || 8 * MT * kSP <= kH, "staging over h");
    // phase 3's vectors, loaded with A: b3 [32 NB3 8] fp16 and (E3_QKV) this tile's rows of cos / sin
    constexpr int kB3 = kRed + 2 * MT * 8 * 4;
    constexpr int kCS = kB3 + NB3 * 256 * 2;           // [2][MT] rows of 64 fp16, 144-B pitch (36 banks
    constexpr int kCSP = 144;                          // a row apart: a column read by 32 rows 2-way, where
    constexpr int kEnd = kCS + (E3 == E3_QKV ? 2 * MT * kCSP : 0);  // a 128-B pitch was 16-way)
    static_assert(kEnd <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) char smem[kEnd];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int m0 = blockIdx.x * MT;
#ifdef LG_FR_STAMPS
    unsigned long long fr_[6] = {0, 0, 0, 0, 0, 0}, fr_last_, fr_entry_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(fr_entry_)::"memory");
    fr_last_ = fr_entry_;
#endif

    // ---- A tile: row 8 i + wave, 16-B unit `lane` (x: units 0..31, head h of the attention output:
    // units 32 + 8 h .. + 7), loaded whole-row coalesced; rows past m repeat row m - 1 ----
    // LG_FFN_AHALF (32-row tiles; the 64-row form measured 45.6 -> 47.6 us with it at P = 16): the x half
    // first, then the heads half — row 16 i + 2 w + lane / 32, unit lane % 32 of each; phase 1's first
    // half (k < 256) runs on x while the heads land
    constexpr bool AH = LG_FFN_AHALF && MB == 1;
    f16x8 av[AH ? 1 : 4 * MB], ax[2 * MB], ac[2 * MB];
    if constexpr (AH) {
#pragma unroll
        for (int i = 0; i < 2 * MB; ++i) {
            const int grow = min(m0 + 16 * i + 2 * wave + (lane >> 5), p.m - 1);
            ax[i] = *reinterpret_cast<const f16x8*>(p.a + (size_t)grow * (K / 2) + (lane & 31) * 8);
        }
#pragma unroll
        for (int i = 0; i < 2 * MB; ++i) {
            const int grow = min(m0 + 16 * i + 2 * wave + (lane >> 5), p.m - 1);
            const LinRow lr = lin_row(p, grow, (lane & 31) >> 3);
            ac[i] = *reinterpret_cast<const f16x8*>((lr.first ? p.ctx0 : p.ctx1) + lr.off + (lane & 7) * 8);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4 * MB; ++i) {
            const int grow = min(m0 + 8 * i + wave, p.m - 1);
            const f16* src;
            if (lane < 32) {
                src = p.a + (size_t)grow * (K / 2) + lane * 8;
            } else {
                const LinRow lr = lin_row(p, grow, (lane - 32) >> 3);
                src = (lr.first ? p.ctx0 : p.ctx1) + lr.off + ((lane - 32) & 7) * 8;
            }
            av[i] = *reinterpret_cast<const f16x8*>(src);
        }
    }
    // the epilogue vectors: b1 / gamma / beta (64 units each) and b2 (32 units)
    f16x8 pv = {};
    if (tid < 224) {
        const f16* const pvs = tid < 64 ? p.bias : tid < 128 ? gamma : tid < 192 ? beta : b2;
        pv = *reinterpret_cast<const f16x8*>(pvs + (tid & 63) * 8);
    }

    constexpr int NV3 = NB3 * 256 * 2 / 16 + (E3 == E3_QKV ? 2 * MT * kD * 2 / 16 : 0);  // 16-B units
    constexpr int NV3T = (NV3 + 511) / 512;
    f16x8 v3[NV3T > 0 ? NV3T : 1];
#pragma unroll
    for (int i = 0; i < NV3T; ++i) {
        const int u = i * 512 + tid;
        if (u < NB3 * 256 * 2 / 16) {
            v3[i] = *reinterpret_cast<const f16x8*>(q3.b3 + u * 8);
        } else if (u < NV3) {  // cos / sin rows: table t, row rw (clamped), unit cu
            const int cu = u - NB3 * 256 * 2 / 16, t = cu / (MT * 8), rw = min(m0 + (cu % (MT * 8)) / 8, p.m - 1);
            v3[i] = *reinterpret_cast<const f16x8*>((t ? q3.sinv : q3.cosv) + (size_t)rw * kD + (cu % 8) * 8);
        }
    }

    // every wave's A loads are issued before any wave's weight stream: the loads of a CU pass its
    // texture unit in issue order, and A behind seven waves' weight prefetch waited ~2.6 k cycles
    asm volatile("s_barrier" ::: "memory");

    // ---- the weight stream (lg_ffn_pack's layout): wave w's 96 KiB, piece i at w * 96 KiB + i KiB,
    // lane l's 16 B at + 16 l: step j of phase 1, block b = piece 2 j + b; step j of phase 2 = 64 + j.
    // Every load is one contiguous KiB (whole 128-B lines: the row-major W's 32-B row pieces per
    // lane fetched each line four times, 26 vs 12 us per launch at 2,048 rows) ----
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(wp), (short)0, 8 * NP * 1024, 0x00020000);
    const unsigned wo = (unsigned)(wave * NP * 1024 + lane * 16);
    auto piece = [&](int i) { return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, wo, i * 1024, 0)); };
    f16x8 q[R];  // piece i in slot i % R; consuming piece i issues piece i + R
#pragma unroll
    for (int i = 0; i < R; ++i) {  // (in stream order: the loops' counted waits assume it)
        q[i] = piece(i);
        if (i & 1) __builtin_amdgcn_sched_barrier(0);
    }
    auto take = [&](int i) {  // piece i (compile-time after unrolling), and the refill behind it
        const f16x8 w = q[i % R];
        if (i + R < NP) q[i % R] = piece(i + R);
        return w;
    };
    // A and the vectors into LDS (the compiler's wait counts the weight loads issued after them)
    auto put_half = [&](const f16x8 (&hv)[2 * MB], int u0) {
#pragma unroll
        for (int i = 0; i < 2 * MB; ++i) {
            const int row = 16 * i + 2 * wave + (lane >> 5), u = u0 + (lane & 31);
            *(lds_f16x8*)(lds + kA + row * 1024 + ((u ^ (row & 15)) << 4)) = hv[i];
        }
    };
    if constexpr (AH) {
        put_half(ax, 0);
    } else {
#pragma unroll
        for (int i = 0; i < 4 * MB; ++i) {
            const int row = 8 * i + wave;
            *(lds_f16x8*)(lds + kA + row * 1024 + ((lane ^ (row & 15)) << 4)) = av[i];
        }
    }
    if (tid < 224) *(lds_f16x8*)(lds + kPar + tid * 16) = pv;
#pragma unroll
    for (int i = 0; i < NV3T; ++i)
        if (i * 512 + tid < NB3 * 256 * 2 / 16) {
            *(lds_f16x8*)(lds + kB3 + (i * 512 + tid) * 16) = v3[i];
        } else if (i * 512 + tid < NV3) {  // cos / sin unit (table t, row rw, unit cu % 8), padded rows
            const int cu = i * 512 + tid - NB3 * 256 * 2 / 16;
            *(lds_f16x8*)(lds + kCS + (cu / 8) * kCSP + (cu % 8) * 16) = v3[i];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    FR_SEG(0);

    // B-operand fragments of step s from an [MT][1 KiB] tile: rows 32 mb + r, unit 2 s + hh
    struct BF {
        f16x8 v[MB];
    };
    auto bfrag = [&](int base, int s) {
        BF f;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            const int row = 32 * mb + r;
            f.v[mb] = *(lds_f16x8*)(lds + base + row * 1024 + (((2 * s + hh) ^ (row & 15)) << 4));
        }
        return f;
    };
    // ---- phase 1: hᵀ (the wave's 64 channels x MT rows) = W1 · Aᵀ; each step's B fragments are read
    // one step ahead (their LDS latency under the previous MFMAs) ----
    f32x16 acc[2][MB] = {};
    BF af = bfrag(kA, 0);
#pragma unroll
    for (int j = 0; j < NS1; ++j) {
        const f16x8 wa = take(2 * j), wb = take(2 * j + 1);
        if constexpr (AH) {
            if (j + 1 == NS1 / 2) {  // the heads half into LDS before step NS1 / 2's fragments are read
                put_half(ac, 32);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
        }
        const BF an = j + 1 < NS1 ? bfrag(kA, j + 1) : af;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            acc[0][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa, af.v[mb], acc[0][mb], 0, 0, 0);
            acc[1][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wb, af.v[mb], acc[1][mb], 0, 0, 0);
        }
        af = an;
        __builtin_amdgcn_sched_barrier(0);
        FFN_SYNC(2 * (j + 1), 2 * NS1);
    }

    FR_SEG(1);
    // ---- LayerNorm over each row's 512 h values: the wave's 64 are in lanes r and r + 32 ----
    // lane (r, hh): acc[b][mb][4 g + t] = hidden channel 64 w + 32 b + 8 g + 4 hh + t of row 32 mb + r.
    // h = fp16(acc + b1) in one rounding (v_fma_mixlo_f16; the two calls' lin_val rounds through fp32
    // first: the same value but for a rare double rounding), then the row's sum and sum of squares
    // in one pass and mean / variance as lg_layernorm_gelu forms them (E[h^2] - mean^2, fp32): one
    // exchange through LDS (vector issue bounds this phase: ~19 VALU per value, two waves a SIMD)
    float* const red = (float*)(void*)(smem + kRed);  // [pass][row][wave]
    float sm[MB], sq[MB];
    unsigned hp[2][MB][8];  // h as packed fp16 pairs: block b, rows mb, (g, pair u) at 2 g + u
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const u32x2 b4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + (64 * wave + 32 * b + 8 * g + 4 * hh) * 2);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    hp[b][mb][2 * g + u] = mixh2(acc[b][mb][4 * g + 2 * u], acc[b][mb][4 * g + 2 * u + 1], b4[u]);
                    row_sums2(hp[b][mb][2 * g + u], s1, s2);
                }
            }
        sm[mb] = s1 + __shfl_xor(s1, 32, 64);
        sq[mb] = s2 + __shfl_xor(s2, 32, 64);
    }
    if (hh == 0) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            red[(32 * mb + r) * 8 + wave] = sm[mb];
            red[MT * 8 + (32 * mb + r) * 8 + wave] = sq[mb];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    auto row_sum = [&](int off, int row) {  // the 8 waves' partials of a row, in a fixed order
        const f32x4 a = *(__attribute__((address_space(3))) f32x4*)(lds + kRed + (off + row * 8) * 4);
        const f32x4 c = *(__attribute__((address_space(3))) f32x4*)(lds + kRed + (off + row * 8 + 4) * 4);
        return ((a[0] + a[1]) + (a[2] + a[3])) + ((c[0] + c[1]) + (c[2] + c[3]));
    };
    // GELU(LN(h)) -> fp16 into the h tile (unit 8 w + 4 b + g of the row, half hh)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        const int row = 32 * mb + r;
        const float mean = row_sum(0, row) * (1.f / K);
        const float rstd = __builtin_amdgcn_rsqf(fmaxf(row_sum(MT * 8, row) * (1.f / K) - mean * mean, 0.f) + eps);
        const float nmr = -mean * rstd;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = 64 * wave + 32 * b + 8 * g + 4 * hh;
                const u32x2 g4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + K * 2 + n * 2);
                const u32x2 be4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + 2 * K * 2 + n * 2);
                f16x4 o;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const unsigned h2 = hp[b][mb][2 * g + u];
                    const float x0 = mixn<0>(h2, rstd, nmr), x1 = mixn<1>(h2, rstd, nmr);
                    const f32x2 gl = gelu_as2(f32x2{mixf<0>(x0, g4[u], be4[u]), mixf<1>(x1, g4[u], be4[u])});
                    o[2 * u] = (f16)gl[0];
                    o[2 * u + 1] = (f16)gl[1];
                }
                *(__attribute__((address_space(3))) f16x4*)(lds + kH + row * 1024 + (((8 * wave + 4 * b + g) ^ (row & 15)) << 4) + 8 * hh) = o;
            }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // h complete
    FR_SEG(2);

    // ---- phase 2: outᵀ (the wave's 32 channels x MT rows) = W2 · hᵀ ----
    f32x16 o2[MB] = {};
    BF hf = bfrag(kH, 0);
#pragma unroll
    for (int j = NS1; j < NS; ++j) {
        const f16x8 wa = take(NS1 + j);
        const BF hn = j + 1 < NS ? bfrag(kH, j + 1 - NS1) : hf;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) o2[mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa, hf.v[mb], o2[mb], 0, 0, 0);
        hf = hn;
        __builtin_amdgcn_sched_barrier(0);
        FFN_SYNC(j + 1 - NS1, NS1);
    }
    FR_SEG(3);
    if constexpr (MB > 1) {  // (the staging rows lie over h: every wave done reading it)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }

    // ---- out = fp16(fp16(acc + b2) + x): the wave's MT x 32 block staged row-major in its own LDS
    // rows (80-B pitch), then two lanes a row, 32 B each, with x from the A tile ----
    lds_char* const stg = lds + kStg + wave * (MT * kSP);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int c = 32 * wave + 8 * g + 4 * hh;
            const f16x4 b4 = *(__attribute__((address_space(3))) f16x4*)(lds + kPar + 3 * K * 2 + c * 2);
            const f16x4 v = f16x4{lin_val(o2[mb][4 * g], b4[0]), lin_val(o2[mb][4 * g + 1], b4[1]),
                                  lin_val(o2[mb][4 * g + 2], b4[2]), lin_val(o2[mb][4 * g + 3], b4[3])};
            *(__attribute__((address_space(3))) f16x4*)(stg + (32 * mb + r) * kSP + (8 * g + 4 * hh) * 2) = v;
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the wave's own rows: LDS ops of a wave in order)
    f16x8 xo[MB][2];  // x' = this lane's out values (phase 3's input)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        const int rr = 32 * mb + (lane >> 1), half = lane & 1;
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
            f16x8 v = *(lds_f16x8*)(stg + rr * kSP + half * 32 + e2 * 16);
            const f16x8 xr = *(lds_f16x8*)(lds + kA + rr * 1024 + (((4 * wave + 2 * half + e2) ^ (rr & 15)) << 4));
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = res_add(v[e], xr[e]);
            xo[mb][e2] = v;
            if (m0 + rr < p.m) *reinterpret_cast<f16x8*>(p.out[0] + (size_t)(m0 + rr) * NO + 32 * wave + 16 * half + 8 * e2) = v;
        }
    }
#ifdef LG_FR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FR_SEG(4);
#endif
    if constexpr (E3 != E3_NONE) {
        // ---- phase 3: the next projection of x' (K = 256): x' rows into the A region ([MT][512 B],
        // units XOR (row & 15)) once every wave has read its residual there ----
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            const int rr = 32 * mb + (lane >> 1), half = lane & 1;
#pragma unroll
            for (int e2 = 0; e2 < 2; ++e2)
                *(lds_f16x8*)(lds + kA + rr * 512 + (((4 * wave + 2 * half + e2) ^ (rr & 15)) << 4)) = xo[mb][e2];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        auto xfrag = [&](int s) {
            BF f;
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                const int row = 32 * mb + r;
                f.v[mb] = *(lds_f16x8*)(lds + kA + row * 512 + (((2 * s + hh) ^ (row & 15)) << 4));
            }
            return f;
        };
        // the wave's NB3 blocks of 32 output channels, c = 32 (NB3 w + b) + ...
        f32x16 a3[NB3][MB] = {};
        BF xf = xfrag(0);
#pragma unroll
        for (int j = 0; j < NS3; ++j) {
            f16x8 w3[NB3];
#pragma unroll
            for (int b = 0; b < NB3; ++b) w3[b] = take(96 + NB3 * j + b);
            const BF xn = j + 1 < NS3 ? xfrag(j + 1) : xf;
#pragma unroll
            for (int b = 0; b < NB3; ++b)
#pragma unroll
                for (int mb = 0; mb < MB; ++mb) a3[b][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w3[b], xf.v[mb], a3[b][mb], 0, 0, 0);
            xf = xn;
            __builtin_amdgcn_sched_barrier(0);
            FFN_SYNC(NB3 * (j + 1), NB3 * NS3);
        }
        // epilogue: fp16(acc + b3) (+ rotary for q, k) as the standalone projections compute it, the
        // wave's rows x 32 channels of a block staged (its own rows of the staging region), then two
        // lanes a row, 32 B each, to the row's head-major (or row-major) destination
#pragma unroll
        for (int b = 0; b < NB3; ++b) {
            const int cb = 32 * (NB3 * wave + b);  // the block's first channel (one head of one part)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c = cb + 8 * g + 4 * hh;
                    const f16x4 b4 = *(__attribute__((address_space(3))) f16x4*)(lds + kB3 + c * 2);
                    f16x4 v = f16x4{lin_val(a3[b][mb][4 * g], b4[0]), lin_val(a3[b][mb][4 * g + 1], b4[1]),
                                    lin_val(a3[b][mb][4 * g + 2], b4[2]), lin_val(a3[b][mb][4 * g + 3], b4[3])};
#ifndef LG_FR_ABL
                    constexpr int kAbl = 0;
#else
                    constexpr int kAbl = LG_FR_ABL;  // diagnostic builds: 1 no rotary, 2 no phase-3 stores
#endif
                    if constexpr (E3 == E3_QKV && kAbl != 1) {
                        if (cb < 2 * NO) {  // q, k: rotary pairs (d, d + 1) from this row's tables
                            const int rw = 32 * mb + r;  // (tile row; rows past m hold row m - 1's tables)
                            const f16x4 cc = *(__attribute__((address_space(3))) f16x4*)(lds + kCS + rw * kCSP + (c % kD) * 2);
                            const f16x4 ss = *(__attribute__((address_space(3))) f16x4*)(lds + kCS + (MT + rw) * kCSP + (c % kD) * 2);
#pragma unroll
                            for (int t = 0; t < 4; t += 2) rot_pair(v, t, cc[t], ss[t], cc[t + 1], ss[t + 1]);
                        }
                    }
                    *(__attribute__((address_space(3))) f16x4*)(stg + (32 * mb + r) * kSP + (8 * g + 4 * hh) * 2) = v;
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                const int rr = 32 * mb + (lane >> 1), half = lane & 1;
                const f16x8 v0 = *(lds_f16x8*)(stg + rr * kSP + half * 32);
                const f16x8 v1 = *(lds_f16x8*)(stg + rr * kSP + half * 32 + 16);
                const int row = m0 + rr;
                if (row < p.m) {
                    f16* dst;
                    if constexpr (E3 == E3_PLAIN) {
                        dst = cb < q3.n_store ? q3.out[0] + (size_t)row * q3.n_store + cb + 16 * half : nullptr;
                    } else {
                        const int part = cb / NO, h = (cb % NO) / kD;
                        const LinRow lr = lin_row(p, row, h);
                        dst = q3.out[E3 == E3_QKV ? (lr.first ? 0 : 3) + part : (lr.first ? 0 : 1) + 2 * part] + lr.off +
                              cb % kD + 16 * half;
                    }
#ifdef LG_FR_ABL
                    if (LG_FR_ABL == 2) dst = nullptr;
#endif
                    if (dst) {
                        *reinterpret_cast<f16x8*>(dst) = v0;
                        *reinterpret_cast<f16x8*>(dst + 8) = v1;
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the next block rewrites the staging rows)
        }
    }
#ifdef LG_FR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FR_SEG(5);  // (phase 3 and its epilogue; segment 4 then ends at phase 2's stores)
#endif
#ifdef LG_FR_STAMPS
    if (lane == 0 && blockIdx.x < 256) {
        unsigned long long* d = g_fr_stamps + ((size_t)blockIdx.x * 8 + wave) * 8;
        for (int k = 0; k < 5; ++k) d[k] = fr_[k];
        d[5] = fr_last_ - fr_entry_;
        d[6] = fr_entry_;
        d[7] = fr_[5];
    }
#endif
}

// ---- the 16-row form (round 6): the same FFN (+ phase 3) with v_mfma_f32_16x16x32_f16 on 16-row tiles ----
// At a few thousand rows the 32-row kernel above fills a quarter of the chip (2,048 rows: 64
// workgroups) and its time is the per-CU weight stream (each workgroup reads all of W1, W2, W3) plus
// the LayerNorm+GELU vector work of its 32 x 512 values (~8 k cycles, profiles/r06/ffn_rows_stamps*):
// 16-row tiles double the workgroups and halve the vector work per CU at the same stream. Operands
// (cdna_hip_programming.md §3): lane l holds A[i = l & 15][k = 8 (l >> 4) + e] (weights: channel i of a
// 16-channel block), B[k][j = l & 15] (activation row j), D[4 (l >> 4) + t][l & 15] — channels
// 4 q + t (q = l >> 4) of row l & 15. The weight stream is lg_ffn_pack's second layout: wave w's
// pieces are phase 1 W1[64 w + 16 b + i][32 s + 8 q ..] (piece 4 s + b), phase 2 W2[32 w + 16 b + i]
// (64 + 2 s + b), phase 3 W3[16 (2 NB3 w + b) + i][32 s + 8 q ..] (96 + 2 NB3 s + b): the same channel
// sets per wave as the 32-row layout, so the rounding and order of every sum are unchanged but for
// the k order inside an MFMA.
template <int D, int E3, int NB3, int SP = 1>
__global__ __launch_bounds__(512, 1) void ffn_rows16_kernel(LinArgs p, const f16* __restrict__ gamma,
                                                            const f16* __restrict__ beta, float eps,
                                                            const f16* __restrict__ wp, const f16* __restrict__ b2,
                                                            Proj3 q3) {
    constexpr int MT = 16, K = 512, NO = kFfnOut;
    constexpr int NP = 96 + NB3 * 16;              // the wave's stream: pieces of 1 KiB
    constexpr int R = 2 * D;                       // pieces in flight (a register ring)
    constexpr int NB = 2 * NB3;                    // phase 3: 16-channel blocks per wave
    constexpr int NBP = NB / (SP > 1 ? SP : 1);    // ... of them this workgroup's (SP parts of a tile)
    constexpr int NPS = 96 + 8 * NBP;              // the pieces this workgroup's waves consume
    constexpr int U3 = 32 * NB3;                   // phase 3: 16-B units per output row
    constexpr int kA = 0;                          // A tile [16][1 KiB]: x units 0..31, heads 32..63
    constexpr int kH = kA + MT * 1024;             // h tile [16][1 KiB]
    constexpr int kX = kH + MT * 1024;             // out / x' tile [16][512 B]
    constexpr int kS3 = kX + MT * 512;             // phase 3's staging [16][U3 units]
    constexpr int kPar = kS3 + MT * U3 * 16;       // b1, gamma, beta [512], b2 [256] fp16
    constexpr int kRed = kPar + (3 * K + NO) * 2;  // row partials [2][16][8 waves] fp32
    constexpr int kB3 = kRed + 2 * MT * 8 * 4;     // b3 [n3] fp16
    constexpr int kCS = kB3 + NB3 * 256 * 2;       // E3_QKV: cos / sin rows [2][16] fp16, 144-B pitch
    constexpr int kCSP = 144;                      // (36 banks a row apart: a column read by 16 rows is
                                                   // conflict-free, where a 128-B pitch was 8-way)
    constexpr int kEnd = kCS + (E3 == E3_QKV ? 2 * MT * kCSP : 0);
    static_assert(D >= 1 && D <= 16 && (E3 == E3_NONE) == (NB3 == 0) && kEnd <= 160 * 1024, "shape");
    static_assert(SP == 1 || (E3 != E3_NONE && NB % SP == 0), "parts");
    __shared__ __attribute__((aligned(16))) char smem[kEnd];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, q = lane >> 4;
    // SP > 1: SP workgroups per 16-row tile, each running phases 1 and 2 whole and 1/SP of phase 3
    // (at a few hundred tiles the chip has the CUs; the projection's weight stream and epilogue halve)
    const int part = SP > 1 ? (int)blockIdx.x % SP : 0;
    const int m0 = (SP > 1 ? (int)blockIdx.x / SP : (int)blockIdx.x) * MT;
#ifdef LG_FR_STAMPS
    unsigned long long fr_[7] = {0, 0, 0, 0, 0, 0, 0}, fr_last_, fr_entry_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(fr_entry_)::"memory");
    fr_last_ = fr_entry_;
#endif
    auto tile_unit = [](int row, int u) { return row * 1024 + ((u ^ (row & 15)) << 4); };  // A / h tiles
    auto x_unit = [](int row, int u) { return row * 512 + ((u ^ (row & 15)) << 4); };      // x' tile

    // ---- A tile (two 16-B units a thread: row f / 64, unit f % 64), the vectors; rows past m repeat
    // row m - 1 ----
#if LG_FFN_AHALF
    // (row tid / 32: its x unit tid % 32 first, then its heads unit; phase 1's first half runs on x)
    f16x8 ax, ac;
    {
        const int grow = min(m0 + (tid >> 5), p.m - 1);
        ax = *reinterpret_cast<const f16x8*>(p.a + (size_t)grow * (K / 2) + (tid & 31) * 8);
        const LinRow lr = lin_row(p, grow, (tid & 31) >> 3);
        ac = *reinterpret_cast<const f16x8*>((lr.first ? p.ctx0 : p.ctx1) + lr.off + (tid & 7) * 8);
    }
#else
    f16x8 av[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int f = 512 * i + tid, row = f >> 6, u = f & 63;
        const int grow = min(m0 + row, p.m - 1);
        const f16* src;
        if (u < 32) {
            src = p.a + (size_t)grow * (K / 2) + u * 8;
        } else {
            const LinRow lr = lin_row(p, grow, (u - 32) >> 3);
            src = (lr.first ? p.ctx0 : p.ctx1) + lr.off + ((u - 32) & 7) * 8;
        }
        av[i] = *reinterpret_cast<const f16x8*>(src);
    }
#endif
    f16x8 pv = {};
    if (tid < 224) {
        const f16* const pvs = tid < 64 ? p.bias : tid < 128 ? gamma : tid < 192 ? beta : b2;
        pv = *reinterpret_cast<const f16x8*>(pvs + (tid & 63) * 8);
    }
    constexpr int NVB = NB3 * 256 * 2 / 16;                         // b3 units
    constexpr int NV3 = NVB + (E3 == E3_QKV ? 2 * MT * 8 : 0);      // + cos / sin units
    static_assert(NV3 <= 512, "phase 3 vectors");
    f16x8 v3 = {};
    if (tid < NV3) {
        if (tid < NVB) {
            v3 = *reinterpret_cast<const f16x8*>(q3.b3 + tid * 8);
        } else {  // table t, row rw (clamped), unit cu % 8
            const int cu = tid - NVB, t = cu / (MT * 8), rw = min(m0 + (cu % (MT * 8)) / 8, p.m - 1);
            v3 = *reinterpret_cast<const f16x8*>((t ? q3.sinv : q3.cosv) + (size_t)rw * kD + (cu % 8) * 8);
        }
    }
    asm volatile("s_barrier" ::: "memory");  // (every wave's A loads ahead of the weight stream)

    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(wp), (short)0, 8 * NP * 1024, 0x00020000);
    const unsigned wo = (unsigned)(wave * NP * 1024 + lane * 16);
    // stream position i -> packed piece (phase 3: this part's NBP blocks of each k32 step)
    const int p3off = __builtin_amdgcn_readfirstlane(part * NBP * 1024);
    auto piece = [&](int i) {
        const int so = i < 96 ? i * 1024 : (96 + NB * ((i - 96) / NBP) + (i - 96) % NBP) * 1024 + p3off;
        return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, wo, so, 0));
    };
    f16x8 w_[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        w_[i] = piece(i);
        if (i & 1) __builtin_amdgcn_sched_barrier(0);
    }
    auto take = [&](int i) {
        const f16x8 w = w_[i % R];
        if (i + R < NPS) w_[i % R] = piece(i + R);
        return w;
    };
#if LG_FFN_AHALF
    *(lds_f16x8*)(lds + kA + tile_unit(tid >> 5, tid & 31)) = ax;
#else
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int f = 512 * i + tid;
        *(lds_f16x8*)(lds + kA + tile_unit(f >> 6, f & 63)) = av[i];
    }
#endif
    if (tid < 224) *(lds_f16x8*)(lds + kPar + tid * 16) = pv;
    if (tid < NVB) {
        *(lds_f16x8*)(lds + kB3 + tid * 16) = v3;
    } else if (tid < NV3) {  // cos / sin unit (table t, row rw, unit cu % 8) into its padded row
        const int cu = tid - NVB;
        *(lds_f16x8*)(lds + kCS + (cu / 8) * kCSP + (cu % 8) * 16) = v3;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    FR_SEG(0);

    // ---- phase 1: hᵀ (the wave's 64 channels x 16 rows) = W1 · Aᵀ, k32 steps, B read a step ahead ----
    f32x4 acc[4] = {};
    f16x8 bf = *(lds_f16x8*)(lds + kA + tile_unit(r, q));
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        f16x8 w4[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) w4[b] = take(4 * s + b);
#if LG_FFN_AHALF
        if (s + 1 == 8) {  // the heads half into LDS before step 8's fragments are read
            *(lds_f16x8*)(lds + kA + tile_unit(tid >> 5, 32 + (tid & 31))) = ac;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
#endif
        const f16x8 bn = s + 1 < 16 ? *(lds_f16x8*)(lds + kA + tile_unit(r, 4 * (s + 1) + q)) : bf;
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w4[b], bf, acc[b], 0, 0, 0);
        bf = bn;
        __builtin_amdgcn_sched_barrier(0);
        FFN_SYNC(4 * (s + 1), 64);
    }
    FR_SEG(1);

    // ---- LayerNorm: lane (r, q) holds channels 64 w + 16 b + 4 q + t of row r; h = fp16(acc + b1) in
    // one rounding, the row's sum and sum of squares over the 4 q lanes, then the 8 waves via LDS ----
    float* const red = (float*)(void*)(smem + kRed);
    float s1 = 0.f, s2 = 0.f;
    unsigned hp[4][2];  // h as packed fp16 pairs: block b, channels 4 q + 2 u, + 1
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const u32x2 b4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + (64 * wave + 16 * b + 4 * q) * 2);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            hp[b][u] = mixh2(acc[b][2 * u], acc[b][2 * u + 1], b4[u]);
            row_sums2(hp[b][u], s1, s2);
        }
    }
    // over the row's 4 lanes (l, l ^ 16, l ^ 32, l ^ 48) by lane-group swaps (VALU, no LDS trip)
    auto xsum = [](float x) {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        const float y = __uint_as_float(a[0]) + __uint_as_float(a[1]);
        const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
        return __uint_as_float(c[0]) + __uint_as_float(c[1]);
    };
    s1 = xsum(s1);
    s2 = xsum(s2);
    if (q == 0) {
        red[r * 8 + wave] = s1;
        red[MT * 8 + r * 8 + wave] = s2;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    auto row_sum = [&](int off, int row) {  // the 8 waves' partials of a row, in a fixed order
        const f32x4 a = *(__attribute__((address_space(3))) f32x4*)(lds + kRed + (off + row * 8) * 4);
        const f32x4 c = *(__attribute__((address_space(3))) f32x4*)(lds + kRed + (off + row * 8 + 4) * 4);
        return ((a[0] + a[1]) + (a[2] + a[3])) + ((c[0] + c[1]) + (c[2] + c[3]));
    };
    {
        const float mean = row_sum(0, r) * (1.f / K);
        const float rstd = __builtin_amdgcn_rsqf(fmaxf(row_sum(MT * 8, r) * (1.f / K) - mean * mean, 0.f) + eps);
        const float nmr = -mean * rstd;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int n = 64 * wave + 16 * b + 4 * q;
            const u32x2 g4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + K * 2 + n * 2);
            const u32x2 be4 = *(__attribute__((address_space(3))) u32x2*)(lds + kPar + 2 * K * 2 + n * 2);
            f16x4 o;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float x0 = mixn<0>(hp[b][u], rstd, nmr), x1 = mixn<1>(hp[b][u], rstd, nmr);
                const f32x2 gl = gelu_as2(f32x2{mixf<0>(x0, g4[u], be4[u]), mixf<1>(x1, g4[u], be4[u])});
                o[2 * u] = (f16)gl[0];
                o[2 * u + 1] = (f16)gl[1];
            }
            *(__attribute__((address_space(3))) f16x4*)(lds + kH + tile_unit(r, n >> 3) + 8 * (q & 1)) = o;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // h complete
    FR_SEG(2);

    // ---- phase 2: outᵀ (the wave's 32 channels x 16 rows) = W2 · hᵀ ----
    f32x4 o2[2] = {};
    f16x8 hf = *(lds_f16x8*)(lds + kH + tile_unit(r, q));
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const f16x8 wa = take(64 + 2 * s), wb = take(64 + 2 * s + 1);
        const f16x8 hn = s + 1 < 16 ? *(lds_f16x8*)(lds + kH + tile_unit(r, 4 * (s + 1) + q)) : hf;
        o2[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, hf, o2[0], 0, 0, 0);
        o2[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wb, hf, o2[1], 0, 0, 0);
        hf = hn;
        __builtin_amdgcn_sched_barrier(0);
        FFN_SYNC(2 * (s + 1), 32);
    }
    FR_SEG(3);
    // ---- out = fp16(fp16(acc + b2) + x): fp16(acc + b2) into the x' tile, then one 16-B unit a thread
    // (row tid / 32, unit tid % 32) with x from the A tile, to memory and back into the x' tile ----
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int c = 32 * wave + 16 * b + 4 * q;
        const f16x4 b4 = *(__attribute__((address_space(3))) f16x4*)(lds + kPar + 3 * K * 2 + c * 2);
        const f16x4 v = f16x4{lin_val(o2[b][0], b4[0]), lin_val(o2[b][1], b4[1]), lin_val(o2[b][2], b4[2]),
                              lin_val(o2[b][3], b4[3])};
        *(__attribute__((address_space(3))) f16x4*)(lds + kX + x_unit(r, c >> 3) + 8 * (q & 1)) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
        const int row = tid >> 5, u = tid & 31;
        f16x8 v = *(lds_f16x8*)(lds + kX + x_unit(row, u));
        const f16x8 xr = *(lds_f16x8*)(lds + kA + tile_unit(row, u));
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = res_add(v[e], xr[e]);
        if (part == 0 && m0 + row < p.m) *reinterpret_cast<f16x8*>(p.out[0] + (size_t)(m0 + row) * NO + 8 * u) = v;
        if constexpr (E3 != E3_NONE) *(lds_f16x8*)(lds + kX + x_unit(row, u)) = v;
    }
#ifdef LG_FR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FR_SEG(4);
#endif
    if constexpr (E3 != E3_NONE) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // x' complete
        // ---- phase 3: the wave's NB blocks of 16 output channels, c = 16 (NB w + b) + 4 q + t ----
        // (E3_QKV: this lane's rotary factors read here, their LDS latency under the MFMAs; the v
        // blocks read a harmless column too)
        f16x4 rc[E3 == E3_QKV ? NBP : 1], rs[E3 == E3_QKV ? NBP : 1];
        if constexpr (E3 == E3_QKV) {
#pragma unroll
            for (int b = 0; b < NBP; ++b) {
                const int d = (16 * (NB * wave + part * NBP + b) + 4 * q) % kD;
                rc[b] = *(__attribute__((address_space(3))) f16x4*)(lds + kCS + r * kCSP + d * 2);
                rs[b] = *(__attribute__((address_space(3))) f16x4*)(lds + kCS + (MT + r) * kCSP + d * 2);
            }
        }
        f32x4 a3[NBP] = {};
        f16x8 xf = *(lds_f16x8*)(lds + kX + x_unit(r, q));
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            f16x8 w3[NBP];
#pragma unroll
            for (int b = 0; b < NBP; ++b) w3[b] = take(96 + NBP * s + b);
            const f16x8 xn = s + 1 < 8 ? *(lds_f16x8*)(lds + kX + x_unit(r, 4 * (s + 1) + q)) : xf;
#pragma unroll
            for (int b = 0; b < NBP; ++b) a3[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w3[b], xf, a3[b], 0, 0, 0);
            xf = xn;
            __builtin_amdgcn_sched_barrier(0);
            FFN_SYNC(NBP * (s + 1), 8 * NBP);
        }
        FR_SEG(5);  // (the projection's MFMA loop; its epilogue: segment 6)
        // epilogue: fp16(acc + b3) (+ rotary for q, k) into the staging rows, then one 16-B unit a thread
        // (row, unit u: channels 8 u .. + 7, one head of one part) to its destination
#pragma unroll
        for (int b = 0; b < NBP; ++b) {
            const int c = 16 * (NB * wave + part * NBP + b) + 4 * q;
            const f16x4 b4 = *(__attribute__((address_space(3))) f16x4*)(lds + kB3 + c * 2);
            f16x4 v = f16x4{lin_val(a3[b][0], b4[0]), lin_val(a3[b][1], b4[1]), lin_val(a3[b][2], b4[2]),
                            lin_val(a3[b][3], b4[3])};
#ifndef LG_FR_ABL
            constexpr int kAbl = 0;
#else
            constexpr int kAbl = LG_FR_ABL;  // diagnostic builds: 1 no rotary, 2 no phase-3 stores
#endif
            if constexpr (E3 == E3_QKV && kAbl != 1) {
                if (c < 2 * NO) {  // q, k: rotary pairs (d, d + 1) from this row's tables
#pragma unroll
                    for (int t = 0; t < 4; t += 2) rot_pair(v, t, rc[b][t], rs[b][t], rc[b][t + 1], rs[b][t + 1]);
                }
            }
            *(__attribute__((address_space(3))) f16x4*)(lds + kS3 + r * (U3 * 16) + (((c >> 3) ^ r) << 4) + 8 * (q & 1)) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        {  // thread -> row tid / 32, units t + 32 j (t = tid % 32): part j, head t / 8 — one row
           // lookup per thread, and 32 consecutive threads write a row's 512 B of one part
            const int row = tid >> 5, t = tid & 31, grow = m0 + row;
            if (grow < p.m) {
                if constexpr (E3 == E3_PLAIN) {
#pragma unroll
                    for (int j = 0; j < U3 / 32; ++j) {
                        const int u = t + 32 * j;
#ifdef LG_FR_ABL
                        if (LG_FR_ABL == 2) continue;
#endif
                        if (SP > 1 && ((8 * u) % (16 * NB)) / (16 * NBP) != part) continue;  // (another part's)
                        if (8 * u < q3.n_store)
                            *reinterpret_cast<f16x8*>(q3.out[0] + (size_t)grow * q3.n_store + 8 * u) =
                                *(lds_f16x8*)(lds + kS3 + row * (U3 * 16) + ((u ^ row) << 4));
                    }
                } else {
                    const LinRow lr = lin_row(p, grow, t >> 3);
                    const size_t off = lr.off + (8 * t) % kD;
#pragma unroll
                    for (int j = 0; j < U3 / 32; ++j) {
                        const int u = t + 32 * j;
                        if (SP > 1 && ((8 * u) % (16 * NB)) / (16 * NBP) != part) continue;  // (another part's)
                        const f16x8 v = *(lds_f16x8*)(lds + kS3 + row * (U3 * 16) + ((u ^ row) << 4));
                        f16* const dst = q3.out[E3 == E3_QKV ? (lr.first ? 0 : 3) + j : (lr.first ? 0 : 1) + 2 * j] + off;
#ifdef LG_FR_ABL
                        if (LG_FR_ABL == 2) continue;
#endif
                        *reinterpret_cast<f16x8*>(dst) = v;
                    }
                }
            }
        }
    }
#ifdef LG_FR_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FR_SEG(6);
    if (lane == 0 && blockIdx.x < 256) {  // (slot 6: the phase-3 epilogue, not the entry time)
        unsigned long long* d = g_fr_stamps + ((size_t)blockIdx.x * 8 + wave) * 8;
        for (int i = 0; i < 5; ++i) d[i] = fr_[i];
        d[5] = fr_last_ - fr_entry_;
        d[6] = fr_[6];
        d[7] = fr_[5];
    }
#endif
}

// lg_ffn_pack: one thread per 16-B fragment of the packed stream (layout: include/lightglue_glue.h);
// wave w's stream: 64 W1 pieces, 32 W2 pieces, then NB3 x 16 W3 pieces (NB3 = n3 / 256). form 0: the
// 32-row kernel's fragments (32 channels x k16 a piece), form 1: the 16-row kernel's (16 x k32)
__global__ __launch_bounds__(256) void ffn_pack_kernel(const f16* __restrict__ w1, const f16* __restrict__ w2,
                                                       const f16* __restrict__ w3, int nb3, int form, f16* packed) {
    const int np = 96 + 16 * nb3;                  // pieces per wave
    const int f = blockIdx.x * 256 + threadIdx.x;  // fragment: wave w, piece i, lane l
    if (f >= 8 * np * 64) return;
    const int w = f / (np * 64), i = (f % (np * 64)) / 64, l = f % 64;
    const f16* src;
    if (form == 0) {
        const int r = l % 32, hh = l / 32;
        if (i < 64) src = w1 + (size_t)(64 * w + 32 * (i & 1) + r) * 512 + 16 * (i >> 1) + 8 * hh;
        else if (i < 96) src = w2 + (size_t)(32 * w + r) * 512 + 16 * (i - 64) + 8 * hh;
        else {
            const int j = (i - 96) / nb3, b = (i - 96) % nb3;
            src = w3 + (size_t)(32 * (nb3 * w + b) + r) * 256 + 16 * j + 8 * hh;
        }
    } else {
        const int r = l % 16, q = l / 16;
        if (i < 64) src = w1 + (size_t)(64 * w + 16 * (i & 3) + r) * 512 + 32 * (i >> 2) + 8 * q;
        else if (i < 96) src = w2 + (size_t)(32 * w + 16 * ((i - 64) & 1) + r) * 512 + 32 * ((i - 64) >> 1) + 8 * q;
        else {
            const int j = (i - 96) / (2 * nb3), b = (i - 96) % (2 * nb3);
            src = w3 + (size_t)(16 * (2 * nb3 * w + b) + r) * 256 + 32 * j + 8 * q;
        }
    }
    *reinterpret_cast<f16x8*>(packed + (size_t)f * 8) = *reinterpret_cast<const f16x8*>(src);
}

// ---- the assignment head: similarity + dual log-softmax in two launches (lg_assign_scores, round 6) ----
// MatchAssignment (lightglue.py:208-233) on the fp16 model: sim = m0 · m1ᵀ (fp16 out, the reference's
// bmm), scores = log_softmax(sim, 2) + log_softmax(sim, 1) + logsig(z0) + logsig(z1)ᵀ. Round 5 ran the
// similarity as a framework GEMM and three glue launches (row pass, column pass, combine: ~31 us per
// single-pair forward at n = 1,024, profiles/r05/single_pair_timelines.txt). Here:
//  * assign_lse_kernel: a workgroup owns 32 rows of ONE image and computes their similarity against
//    1/S of the OTHER image's rows by MFMA (own rows in LDS, the other image streamed per wave through
//    a 2-slot LDS-DMA ring of 128-deep K halves, whole 256-B row pieces), then the (max, sum of
//    exponentials) of each own row over that share, reduced over the 8 waves through LDS. Image-0
//    workgroups give the row partials (and write sim in fp16 for the combine), image-1 workgroups the
//    column partials: no cross-workgroup exchange. (An image-1 workgroup recomputes its columns of sim
//    with the operands swapped: the same products in the same k-step order.) S splits of the other
//    image fill the chip at a single pair (each workgroup then streams 1/S of it).
//  * assign_combine_kernel closes the S partials of its rows and columns (fixed order) into the terms
//    logsig(z) - logsumexp and writes scores = 2 sim + row term + column term.
struct AsArgs {
    const f16* v;     // [batch][m + n][ld]: image 0's rows then image 1's; channels 0..255 the scaled
                      // final projection, channel zc the matchability logit
    long ps;          // pair stride of v (elements)
    int ld, zc, m, n, rb0, S;
    f16* sim;         // workspace [batch][m][n]
    float2* rpart;    // workspace [batch][S][m]: (max, sum of exp) of row i over split s
    float2* cpart;    // workspace [batch][S][n]: the same for column j
    float* rterm;     // workspace [batch][m] (round 6's separate close; kept in the workspace layout)
    float* cterm;     // workspace [batch][n]
    float* scores;    // [batch][m][n]
};
__device__ __forceinline__ float log_sigmoid_f(float z) { return fminf(z, 0.f) - log1pf(__expf(-fabsf(z))); }

template <int BPW>  // 32-row blocks of the other image per wave
__global__ __launch_bounds__(512, 1) void assign_lse_kernel(AsArgs a) {
    constexpr int kOwn = 0;                       // own rows [32][512 B], units XOR (row & 15)
    constexpr int kRing = 32 * 512;               // per wave 2 slots of [32][256 B]
    constexpr int kRed = kRing + 8 * 2 * 8192;    // [32 rows][8 waves] fp32
    __shared__ __attribute__((aligned(16))) char smem[kRed + 32 * 8 * 4];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int p = blockIdx.y, sp = blockIdx.z;
    const bool side = (int)blockIdx.x >= a.rb0;
    const int o0 = (side ? (int)blockIdx.x - a.rb0 : (int)blockIdx.x) * 32;
    const int nown = side ? a.n : a.m, noth = side ? a.m : a.n;
    const f16* const vp = a.v + (size_t)p * a.ps;
    const f16* const own = vp + (size_t)(side ? a.m : 0) * a.ld;
    const f16* const oth = vp + (size_t)(side ? 0 : a.m) * a.ld;

    // own rows: 32 rows x 32 units, two per thread
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int u = i * 512 + tid, row = u >> 5, un = u & 31;
        const f16x8 x = *reinterpret_cast<const f16x8*>(own + (size_t)min(o0 + row, nown - 1) * a.ld + un * 8);
        *(lds_f16x8*)(lds + kOwn + row * 512 + ((un ^ (row & 15)) << 4)) = x;
    }
    // the other image's rows, streamed per wave: block t of this wave = other rows 32 ((t S + sp) 8 + w);
    // chunk c = (block t, K half hk) -> slot c & 1
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(oth), (short)0,
                                                                         (int)((size_t)noth * a.ld * 2), 0x00020000);
    auto blk_row0 = [&](int t) { return ((t * a.S + sp) * 8 + wave) * 32; };
    auto issue = [&](int c) {  // 8 pieces of 4 rows x 256 B; lane -> (row 4 i + lane / 16, unit lane % 16)
        const int t = c >> 1, hk = c & 1;
        const unsigned m0 = mha_hd64::lds_addr(smem + kRing + wave * 16384 + (c & 1) * 8192);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = 4 * i + (lane >> 4), pu = lane & 15;
            const int grow = min(blk_row0(t) + row, noth - 1);
            const unsigned voff = (unsigned)(grow * a.ld * 2 + hk * 256 + ((pu ^ (row & 15)) << 4));
            mha_hd64::lds_dma16(m0 + i * 1024, voff, ors, 0);
        }
    };
    constexpr int nch = 2 * BPW;
    auto live = [&](int t) { return blk_row0(t) < noth; };  // (wave-uniform)
    if (live(0)) issue(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // own rows in LDS

    f16 sv[BPW][16];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < BPW; ++t) {
        f32x16 acc = {};
        if (live(t)) {
#pragma unroll
            for (int hk = 0; hk < 2; ++hk) {
                const int c = 2 * t + hk;
                // the next chunk in flight, then this one landed (this wave's own pieces: no barrier)
                if (c + 1 < nch && live((c + 1) >> 1)) {
                    issue(c + 1);
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                const unsigned sb = kRing + wave * 16384 + (c & 1) * 8192;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const int u = 2 * s + hh;
                    const f16x8 af = *(lds_f16x8*)(lds + sb + r * 256 + ((u ^ (r & 15)) << 4));
                    const int uo = 16 * hk + u;
                    const f16x8 bf = *(lds_f16x8*)(lds + kOwn + r * 512 + ((uo ^ (r & 15)) << 4));
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc, 0, 0, 0);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the slot is refilled next chunk)
            }
        }
        // lane (r, hh): acc[4 g + e] = sim of own row o0 + r with other row blk_row0(t) + 8 g + 4 hh + e
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int j0 = blk_row0(t) + 8 * g + 4 * hh;
            f16x4 h4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const f16 h = (f16)acc[4 * g + e];
                h4[e] = h;
                sv[t][4 * g + e] = (j0 + e < noth) ? h : (f16)-INFINITY;
                mx = fmaxf(mx, (float)sv[t][4 * g + e]);
            }
            if (!side && o0 + r < a.m && j0 < a.n)
                *reinterpret_cast<f16x4*>(a.sim + ((size_t)p * a.m + o0 + r) * a.n + j0) = h4;
        }
    }
    // (max, sum of exp) of each own row over this split: the max over the 8 waves, then the sum
    float* const red = (float*)(void*)(smem + kRed);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (hh == 0) red[r * 8 + wave] = mx;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    float M = red[r * 8];
#pragma unroll
    for (int w = 1; w < 8; ++w) M = fmaxf(M, red[r * 8 + w]);
    float s = 0.f;
    if (M != -INFINITY) {
#pragma unroll
        for (int t = 0; t < BPW; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) s += __expf((float)sv[t][e] - M);
    }
    s += __shfl_xor(s, 32, 64);
    __builtin_amdgcn_s_barrier();  // (every wave has read the maxima)
    if (hh == 0) red[r * 8 + wave] = s;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wave == 0 && hh == 0 && o0 + r < nown) {
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) tot += red[r * 8 + w];
        (side ? a.cpart + ((size_t)p * a.S + sp) * a.n : a.rpart + ((size_t)p * a.S + sp) * a.m)[o0 + r] = make_float2(M, tot);
    }
}

// the logsumexp of S (max, sum) partials, merged in split order; every partial's load issued before
// the merge (round 6's first combine-side close walked them one dependent load at a time: 18-38 us)
__device__ __forceinline__ float lse_close(const float2* part, size_t stride, int S) {
    float2 q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = k < S ? part[k * stride] : make_float2(-INFINITY, 0.f);
    float mx = -INFINITY, s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (q[k].x == -INFINITY) continue;
        if (q[k].x > mx) {
            s = s * __expf(mx - q[k].x) + q[k].y;
            mx = q[k].x;
        } else {
            s += q[k].y * __expf(q[k].x - mx);
        }
    }
    return mx + __logf(s);
}

// scores = 2 sim + rterm[i] + cterm[j] (fp32), the terms logsig(z) - logsumexp closed here from the S
// partials (round 6: a separate close launch cost ~4.7 us at a single pair): the block's 8 W rows'
// and 512 columns' terms into LDS (256 threads; every partial and z load in flight at once), then each
// of the W combine waves writes 8 rows, a lane 8 columns (16-B loads, 2 x 16-B stores)
template <int W>
__global__ __launch_bounds__(256) void assign_combine_kernel(AsArgs a) {
    __shared__ float rts[8 * W], cts[512];
    const int p = blockIdx.z, tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int ib = blockIdx.x * 8 * W, jb = blockIdx.y * 512;
    const f16* const vp = a.v + (size_t)p * a.ps;
    if (tid < 8 * W && ib + tid < a.m) {
        const float z = (float)vp[(size_t)(ib + tid) * a.ld + a.zc];
        rts[tid] = log_sigmoid_f(z) - lse_close(a.rpart + (size_t)p * a.S * a.m + ib + tid, a.m, a.S);
    }
#pragma unroll
    for (int c = tid; c < 512; c += 256) {
        if (jb + c < a.n) {
            const float z = (float)vp[(size_t)(a.m + jb + c) * a.ld + a.zc];
            cts[c] = log_sigmoid_f(z) - lse_close(a.cpart + (size_t)p * a.S * a.n + jb + c, a.n, a.S);
        }
    }
    __syncthreads();
    const int i0 = ib + wave * 8, j = jb + lane * 8;
    if (wave >= W || i0 >= a.m || j >= a.n) return;
    const int i1 = min(i0 + 8, a.m);
    const f16* sim = a.sim + (size_t)p * a.m * a.n;
    float* out = a.scores + (size_t)p * a.m * a.n;
    f16x8 x[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) x[b] = *reinterpret_cast<const f16x8*>(sim + (size_t)min(i0 + b, i1 - 1) * a.n + j);
    float cl[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cl[e] = cts[lane * 8 + e];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        if (i0 + b >= i1) break;
        const float rt = rts[wave * 8 + b];
        f32x4 o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            o0[e] = 2.f * (float)x[b][e] + rt + cl[e];
            o1[e] = 2.f * (float)x[b][e + 4] + rt + cl[e + 4];
        }
        *reinterpret_cast<f32x4*>(out + (size_t)(i0 + b) * a.n + j) = o0;
        *reinterpret_cast<f32x4*>(out + (size_t)(i0 + b) * a.n + j + 4) = o1;
    }
}

constexpr int kTileGrid = 256;  // the 256-row forms: one workgroup per CU
// lg_linear_cat_ln_gelu's one-launch form (linear_ln_kernel), by size: its 128-row tiles from one
// full round of them on (256: M >= 32,768 rows, P >= 16 pairs of 1024 keypoints), its 64-row tiles
// from a full round of those (256: M >= 16,384), two launches below. Measured against the two launches
// (profiles/r05/ln_fused_by_size.jsonl, ln64_by_size.jsonl; op alone, us, two launches / 128-row /
// 64-row): P = 1 9.2 / 28.3 / 16.8, P = 4 19.7 / 29.4 / 18.3, P = 8 27.1-27.7 / 32.2 / 21.9, P = 16
// 42.2 / 36.3-39.4 / 38.4, P = 32 74.4-77.7 / 72.7 / 77.0 (few workgroups: each one's GELU vector work
// runs after its GEMM with no other wave's MFMAs beside it; more rows per tile: fewer W bytes per
// row); whole forwards P = 8 1.53-1.54 -> 1.45-1.47 ms (64-row), P = 16 2.541 -> 2.487 (128-row), P =
// 32 4.701 -> 4.642, but P = 4 (half a round of 64-row tiles) 1.03-1.04 -> 1.05-1.06 (profiles/r05/
// ln64_forms_forwards.txt). lg_linear_set_ln_fused: 1 by size (default), 0 always two launches, 2 always one.
std::atomic<int> g_ln_fused{1};
// lg_linear_cat_ffn's form (lg_linear_set_ffn_fused): 1 (default) the one-launch ffn_rows_kernel when
// the caller passes the packed weight stream, 0 always its two calls (lg_linear_cat_ln_gelu, then
// lg_linear with the residual). Measured against the
// two calls (profiles/r06/ffn_rows_*_ab.jsonl, op alone, us): P = 1 (2,048 rows) 15.5 -> 12.1, P = 4
// 31.0 -> 14.4, P = 8 32.4 -> 23.4, P = 16 53.6 -> 46.5, P = 32 94.0 -> 87.3; forwards P = 1 / 8 / 16 / 32
// 0.546 / 1.471 / 2.336 / 4.295 -> 0.501 / 1.204 / 2.145 / 4.029 ms. (Round 5's 128-row one-launch form,
// ffn_kernel, GELU output in LDS and W2 fragments per 128-row tile from L2: 56 vs 52.7 us at P = 16, not
// adopted, and removed in round 6: profiles/r05/ffn_one_launch_ab.jsonl.)
std::atomic<int> g_ffn_fused{1};
// ffn_rows_kernel's weight-stream depth: k16 steps of fragments in flight per wave (measured flat over
// 6..20 at 2,048 and 8,192 rows: the stream is throughput-bound, profiles/r06/ffn_rows_rowmajor_w_ab.jsonl)
constexpr int kFrDepth = 12;
// The tile form (tile_form below): lg_linear_set_wide(0..3) or LG_LINEAR_WIDE forces one (where n
// allows), for tests and A/B timing; -1 (the default) chooses by size.
std::atomic<int> g_wide{-2};
int wide_mode() {
    int v = g_wide.load();
    if (v == -2) {
        const char* e = std::getenv("LG_LINEAR_WIDE");
        long m = -1;  // unset or unparsable: chosen by size
        if (e && *e) {
            char* end = nullptr;
            const long x = std::strtol(e, &end, 10);
            if (end != e) m = x < -1 ? -1 : (x > 5 ? 5 : x);
        }
        int expect = -2;
        g_wide.compare_exchange_strong(expect, (int)m);
        v = g_wide.load();
    }
    return v;
}
bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }
bool aligned8(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 7) == 0; }

// The 256-row tile forms (linear_tile_kernel): 1 = 256 x 128, 2 = 256 x 256 (32-deep K steps, 4
// stages; plain EPI_BIAS only: the residual / rotary tables and the scatter addressing do not fit
// beside its accumulators), 4 = 128 x 128 on 4 waves, two workgroups per CU (64-deep K steps through
// 2 stages). (Round 5's A/B forms 3 = 128 x 256 and 5 = form 4 with 32-deep K steps through 4 stages,
// both slower, were removed in round 6; 3 and 5 now select 1 and 4.) Form 4 against form 1 (profiles/r05/
// tile_form4_ab.jsonl, us): qkv 18.5 / 26.6 / 48.8 -> 15.9 / 25.1 / 46.5 at P = 8 / 16 / 32, split2
// 17.5 -> 17.0 and linear+res 12.2 / 16.9 / 30.7 -> 9.8 / 16.6 / 28.5 (form 1 leaves half the CUs idle
// at P = 8), cat 14.5 / 24.6 / 45.1 -> 14.8 / 24.3 / 46.0; at P = 4 qkv 10.9 = 10.9, split2 8.6 -> 7.4,
// linear+res 10.5 (64 x 64) -> 8.1, cat 11.5 -> 9.3; whole forwards P = 4 / 8 / 16 +2.3 / +2.9 / +0.8 %,
// P = 32 -1.0 % (form_fwd_ab.jsonl): the default below; forms 1 and 2 (the round's earlier default was
// form 1 from half a round of its tiles) stay for lg_linear_set_wide / LG_LINEAR_WIDE, which force a
// form where n and the operand alignment allow.
#ifndef LG_LINEAR_AB_FORMS
#define LG_LINEAR_AB_FORMS 0  // 1: forms 1 and 2 built (A/B builds: tools/build_linear_variant.sh); the
#endif                        // shipped library maps them to form 4 (no kernel that its default never runs)
int tile_form(const LinArgs& p, int epi, bool gather) {
    bool al = aligned16(p.bias);
    const int nout = epi == EPI_BIAS ? 1 : epi == EPI_QKV_ROTARY ? 6 : 4;
    for (int i = 0; i < nout; ++i) al = al && aligned16(p.out[i]);
    if (p.res) al = al && aligned16(p.res);
    if (epi == EPI_QKV_ROTARY) al = al && aligned16(p.cosv) && aligned16(p.sinv);
    if (!al) return 0;
    // (the head-major epilogue's element offsets are 32-bit: every per-image output below 2^32 elements;
    // (and it steps through the rows of a tile with one wrap at most: pairs of more than 56 rows)
    if (epi != EPI_BIAS && ((long long)p.m * p.heads * kD >= (1LL << 32) || p.n0 + p.n1 <= 56)) return 0;
    const int w = wide_mode();
    // by size: the 4-wave 128 x 128 form (two workgroups per CU) from 128 of its tiles and 8,192 rows
    // on, else the 64 x 64 form (profiles/r05/tile_form4_ab.jsonl: at 128 tiles form 4 wins
    // linear+res at P = 4 and lg_linear_cat at P = 2, loses split2 at P = 2 by 1 us; from 192 tiles on
    // it wins or ties every op but lg_linear_cat at P = 32, 2 % behind 256 x 128, which the matcher
    // does not call there. Whole forwards (form_fwd_ab_final.jsonl): P = 2 (4,096 rows) 2 % faster
    // with the 64 x 64 form everywhere, P = 4 / 8 / 16 7 / 3 / 1 % faster than form 1 with this rule)
    (void)gather;
    int f = w >= 0 ? w : (p.m >= 8192 && (long)((p.m + 127) / 128) * (p.n / 128) >= 128 ? 4 : 0);
    if (!LG_LINEAR_AB_FORMS && (f == 1 || f == 2 || f == 3)) f = 4;
    if (f == 2 && p.n % 256 == 0) return (p.res || epi != EPI_BIAS) ? 1 : 2;
    if (f >= 4 && p.n % 128 == 0) return 4;  // (5: round 5's 32-deep A/B variant of form 4, removed in round 6)
    return f >= 1 && p.n % 128 == 0 ? 1 : 0;  // (3: round 5's 128 x 256 A/B form, removed in round 6)
}

template <int EPI, bool GATHER, bool RES, int MT, int NT, int BK, int NST, int NWV>
void launch_tile_r(LinArgs& p, hipStream_t stream) {
    p.mtiles = (p.m + MT - 1) / MT;
    p.total = p.mtiles * (p.n / NT);
    constexpr int cap = kTileGrid * 8 / NWV;  // persistent: one round (4 waves: two workgroups per CU)
    const int grid = p.total < cap ? p.total : cap;
    if (p.k == 256)
        hipLaunchKernelGGL((linear_tile_kernel<EPI, GATHER, RES, 256 / BK, MT, NT, BK, NST, NWV>), dim3(grid), dim3(64 * NWV), 0, stream, p);
    else
        hipLaunchKernelGGL((linear_tile_kernel<EPI, GATHER, RES, 512 / BK, MT, NT, BK, NST, NWV>), dim3(grid), dim3(64 * NWV), 0, stream, p);
}
template <int EPI, bool GATHER, int MT, int NT, int BK, int NST, int NWV = 8>
void launch_tile(LinArgs& p, hipStream_t stream) {
    constexpr bool WIDE_WAVE = NT * MT / 64 / NWV / 32 > 2;  // 64 x 128 wave tiles
    if constexpr (EPI == EPI_BIAS && !GATHER && !WIDE_WAVE) {
        if (p.res) return launch_tile_r<EPI, GATHER, true, MT, NT, BK, NST, NWV>(p, stream);
    }
    if constexpr (!(WIDE_WAVE && EPI == EPI_QKV_ROTARY)) launch_tile_r<EPI, GATHER, false, MT, NT, BK, NST, NWV>(p, stream);
}

template <int EPI, bool GATHER>
int32_t launch(LinArgs& p, hipStream_t stream, const char* what) {
    int form = tile_form(p, EPI, GATHER);
    if (GATHER && form == 2) form = 1;  // (the gather's per-piece sources do not fit beside 64 x 128 wave tiles)
    switch (form) {
#if LG_LINEAR_AB_FORMS
        case 1: launch_tile<EPI, GATHER, 256, 128, 64, 3>(p, stream); break;
        case 2:
            if constexpr (!GATHER && EPI == EPI_BIAS) launch_tile<EPI, GATHER, 256, 256, 32, 4>(p, stream);
            break;
#endif
        case 4: launch_tile<EPI, GATHER, 128, 128, 64, 2, 4>(p, stream); break;
        default:
            p.mtiles = (p.m + kBM - 1) / kBM;
            p.total = p.mtiles * (p.n / kBN);
            if (p.k == 256)
                hipLaunchKernelGGL((linear_kernel<EPI, GATHER, 2>), dim3(p.total), dim3(256), 0, stream, p);
            else
                hipLaunchKernelGGL((linear_kernel<EPI, GATHER, 4>), dim3(p.total), dim3(256), 0, stream, p);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, what, hipGetErrorString(e));
}

// The one-launch FFN by size (lg_linear_set_ffn_fused 1): 16-row workgroups up to one round of them
// (ffn_rows16_kernel: the most workgroups and the least vector work per CU, for latency), 32-row up
// to one round, 64-row beyond (half the weight bytes per row); 2 / 3: the 32/64-row / 16-row kernel at
// every size (A/B). wp: lg_ffn_pack's two layouts, the 32-row kernel's first. (Tried and dropped: the
// 32-row kernel two workgroups per CU (128 VGPRs, an 8-piece ring, staging over h), for one workgroup's
// A-tile latency under the other's stream — 46.0 -> 47.1 us at 32,768 rows, 23.0 -> 24.1 at 16,384,
// equal bits; profiles/r06/ffn_rows_occ2_ab.jsonl.)
// The 16-row kernel's projection split over two workgroups per tile (ffn_rows16_kernel<…, SP = 2>):
// up to 64 tiles (LG_FFN_SPLIT=0: never, =2: while 2 x tiles fill at most one round). Measured
// (profiles/r06/ffn_phase3_split_ab.jsonl, single-pair forwards, ms): n = 512 (64 tiles) 0.368 -> 0.353;
// n = 1024 (128 tiles) 0.427-0.431 -> 0.434 split, kept whole. Three / four parts (one or two blocks
// per wave, an A/B build) : n = 512 0.351-0.354 -> 0.355-0.359, n = 256 0.334 -> 0.325.
int ffn_split_parts(int tiles) {
    static const int env = [] {
        const char* e = std::getenv("LG_FFN_SPLIT");
        return e ? std::atoi(e) : -1;
    }();
    if (env == 0) return 1;
    return (env == 2 ? 2 * tiles <= kTileGrid : tiles <= 64) ? 2 : 1;
}
template <int E3, int NB3>
void launch_ffn_rows(const LinArgs& p, const f16* gamma, const f16* beta, float eps, const f16* wp, const f16* b2,
                     const Proj3& q3, hipStream_t stream) {
    const int mode = g_ffn_fused.load();
    if (mode == 3 || (mode != 2 && p.m <= 16 * kTileGrid)) {
        const f16* wp16 = wp + (size_t)8 * (96 + 16 * NB3) * 1024 / 2;
        const int tiles = (p.m + 15) / 16;
        if constexpr (E3 != E3_NONE) {
            const int sp = ffn_split_parts(tiles);
            if (sp == 2) {
                hipLaunchKernelGGL((ffn_rows16_kernel<kFrDepth, E3, NB3, 2>), dim3(2 * tiles), dim3(512), 0, stream, p,
                                   gamma, beta, eps, wp16, b2, q3);
                return;
            }
        }
        hipLaunchKernelGGL((ffn_rows16_kernel<kFrDepth, E3, NB3>), dim3(tiles), dim3(512), 0, stream, p, gamma, beta, eps,
                           wp16, b2, q3);
    } else if (p.m <= 32 * kTileGrid)
        hipLaunchKernelGGL((ffn_rows_kernel<1, kFrDepth, E3, NB3>), dim3((p.m + 31) / 32), dim3(512), 0, stream, p, gamma, beta,
                           eps, wp, b2, q3);
    else
        hipLaunchKernelGGL((ffn_rows_kernel<2, kFrDepth, E3, NB3>), dim3((p.m + 63) / 64), dim3(512), 0, stream, p, gamma, beta,
                           eps, wp, b2, q3);
}

bool shape_ok(int m, int n, int k) { return m >= 0 && n > 0 && n % kBN == 0 && (k == 256 || k == 512); }

int32_t bad(const char* what) { return mha_hd64::report_error(MHA_HD64_STATUS_BAD_PARAM, what, "bad arguments"); }

}  // namespace

extern "C" {

int32_t lg_linear(const void* a, const void* w, const void* bias, const void* res, int32_t m, int32_t n, int32_t k,
                  void* out, hipStream_t stream) {
    if (!shape_ok(m, n, k) || !a || !w || !bias || !out || !aligned16(a) || !aligned16(w) || !aligned8(bias) ||
        !aligned8(out) || (res && !aligned8(res)))
        return bad("lg_linear");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    LinArgs p{};
    p.a = (const f16*)a, p.w = (const f16*)w, p.bias = (const f16*)bias, p.res = (const f16*)res;
    p.out[0] = (f16*)out;
    p.m = m, p.n = n, p.k = k, p.n0 = m, p.n1 = 0;
    return launch<EPI_BIAS, false>(p, stream, "lg_linear");
}

int32_t lg_linear_cat(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                      int32_t pairs, const void* w, const void* bias, int32_t n, void* out, hipStream_t stream) {
    const int k = 2 * heads * kD, m = pairs * (n0 + n1);
    if (heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !shape_ok(m, n, k) || !x || !w || !bias || !out || !aligned16(x) ||
        (n0 && !aligned16(ctx0)) || (n1 && !aligned16(ctx1)) || !aligned16(w) || !aligned8(bias) || !aligned8(out))
        return bad("lg_linear_cat");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    LinArgs p{};
    p.a = (const f16*)x, p.ctx0 = (const f16*)ctx0, p.ctx1 = (const f16*)ctx1, p.w = (const f16*)w;
    p.bias = (const f16*)bias, p.out[0] = (f16*)out;
    p.m = m, p.n = n, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    return launch<EPI_BIAS, true>(p, stream, "lg_linear_cat");
}

int32_t lg_linear_cat_ln_gelu(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                              int32_t pairs, const void* w, const void* bias, const void* gamma, const void* beta,
                              float eps, void* out, hipStream_t stream) {
    const int k = 2 * heads * kD, m = pairs * (n0 + n1), n = k;
    if (heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !shape_ok(m, n, k) || !x || !w || !bias || !gamma || !beta ||
        !out || !aligned16(x) || (n0 && !aligned16(ctx0)) || (n1 && !aligned16(ctx1)) || !aligned16(w) ||
        !aligned8(bias) || !aligned8(out) || !(eps >= 0.f))
        return bad("lg_linear_cat_ln_gelu");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    const int lnf = g_ln_fused.load();  // 1: by size; 2: at every size (A/B)
    const bool big = m >= 128 * kTileGrid;  // a full round of 128-row tiles (32,768 rows)
    const bool fused = lnf && n == kLnN && (lnf == 2 || big || m >= 64 * kTileGrid) && aligned16(bias) && aligned16(gamma) &&
                       aligned16(beta) && aligned16(out) && wide_mode() != 0;
    if (!fused) {  // the projection, then LayerNorm+GELU in place (lightglue_glue.hip)
        const int32_t st = lg_linear_cat(x, ctx0, ctx1, heads, n0, n1, pairs, w, bias, n, out, stream);
        if (st != MHA_HD64_STATUS_SUCCESS) return st;
        return lg_layernorm_gelu(MHA_HD64_DT_HALF, out, gamma, beta, m, n, eps, out, stream);
    }
    LinArgs p{};
    p.a = (const f16*)x, p.ctx0 = (const f16*)ctx0, p.ctx1 = (const f16*)ctx1, p.w = (const f16*)w;
    p.bias = (const f16*)bias, p.out[0] = (f16*)out;
    p.m = m, p.n = n, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    p.mtiles = big ? (m + 127) / 128 : (m + 63) / 64;
    p.total = p.mtiles;
    const int grid = p.total < kTileGrid ? p.total : kTileGrid;
    if (big)
        hipLaunchKernelGGL((linear_ln_kernel<512 / 32, 128, 32, 3>), dim3(grid), dim3(512), 0, stream, p,
                           (const f16*)gamma, (const f16*)beta, eps);
    else
        hipLaunchKernelGGL((linear_ln_kernel<512 / 64, 64, 64, 2>), dim3(grid), dim3(512), 0, stream, p,
                           (const f16*)gamma, (const f16*)beta, eps);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, "lg_linear_cat_ln_gelu",
                                                    hipGetErrorString(e));
}

int32_t lg_linear_cat_ffn(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                          int32_t pairs, const void* w1, const void* b1, const void* gamma, const void* beta, float eps,
                          const void* w2, const void* b2, const void* w_packed, void* h, void* out, hipStream_t stream) {
    const int d = heads * kD, k = 2 * d, m = pairs * (n0 + n1);
    if (heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !shape_ok(m, k, k) || !x || !w1 || !b1 || !gamma || !beta || !w2 ||
        !b2 || !h || !out || out == x || !aligned16(x) || (n0 && !aligned16(ctx0)) || (n1 && !aligned16(ctx1)) ||
        !aligned16(w1) || !aligned16(w2) || !aligned8(b1) || !aligned8(b2) || !aligned16(h) || !aligned8(out) || !(eps >= 0.f) ||
        (w_packed && !aligned16(w_packed)))
        return bad("lg_linear_cat_ffn");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    const bool one = g_ffn_fused.load() != 0 && w_packed && k == kLnN && d == kFfnOut && aligned16(b1) && aligned16(gamma) &&
                     aligned16(beta) && aligned16(b2) && aligned16(out);
    if (!one) {  // h in the caller's buffer, then the output projection with the residual
        const int32_t st = lg_linear_cat_ln_gelu(x, ctx0, ctx1, heads, n0, n1, pairs, w1, b1, gamma, beta, eps, h, stream);
        if (st != MHA_HD64_STATUS_SUCCESS) return st;
        return lg_linear(h, w2, b2, x, m, d, k, out, stream);
    }
    LinArgs p{};
    p.a = (const f16*)x, p.ctx0 = (const f16*)ctx0, p.ctx1 = (const f16*)ctx1, p.w = (const f16*)w1;
    p.bias = (const f16*)b1, p.out[0] = (f16*)out;
    p.m = m, p.n = k, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    launch_ffn_rows<E3_NONE, 0>(p, (const f16*)gamma, (const f16*)beta, eps, (const f16*)w_packed, (const f16*)b2, Proj3{}, stream);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, "lg_linear_cat_ffn", hipGetErrorString(e));
}

size_t lg_ffn_packed_bytes(int32_t heads, int32_t n3) {  // both layouts, the 32-row kernel's first
    return heads == 4 && (n3 == 0 || n3 == 512 || n3 == 768) ? (size_t)2 * 8 * (96 + n3 / 16) * 1024 : 0;
}

int32_t lg_ffn_pack(const void* w1, const void* w2, const void* w3, int32_t n3, int32_t heads, void* packed, hipStream_t stream) {
    if (!lg_ffn_packed_bytes(heads, n3) || !w1 || !w2 || !packed || !aligned16(w1) || !aligned16(w2) || !aligned16(packed) ||
        (n3 && (!w3 || !aligned16(w3))))
        return bad("lg_ffn_pack");
    const int nb3 = n3 / 256, frags = 8 * (96 + 16 * nb3) * 64;
    for (int form = 0; form < 2; ++form)
        hipLaunchKernelGGL(ffn_pack_kernel, dim3((frags + 255) / 256), dim3(256), 0, stream, (const f16*)w1, (const f16*)w2,
                           (const f16*)w3, nb3, form, (f16*)packed + (size_t)form * frags * 8);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, "lg_ffn_pack", hipGetErrorString(e));
}

int32_t lg_linear_cat_ffn_proj(const void* x, const void* ctx0, const void* ctx1, int32_t heads, int32_t n0, int32_t n1,
                               int32_t pairs, const void* b1, const void* gamma, const void* beta, float eps, const void* b2,
                               const void* w_packed, int32_t kind, const void* b3, const void* cosv, const void* sinv,
                               int32_t n_store, void* const* outs3, void* out, hipStream_t stream) {
    const int d = heads * kD, k = 2 * d, m = pairs * (n0 + n1);
    const int nouts = kind == LG_PROJ_SPLIT2 ? 4 : kind == LG_PROJ_QKV ? 6 : kind == LG_PROJ_PLAIN ? 1 : 0;
    bool ok = heads == 4 && n0 >= 0 && n1 >= 0 && pairs >= 0 && nouts && x && b1 && gamma && beta && b2 && w_packed && b3 && outs3 &&
              out && out != x && aligned16(x) && (!n0 || aligned16(ctx0)) && (!n1 || aligned16(ctx1)) && aligned16(b1) &&
              aligned16(gamma) && aligned16(beta) && aligned16(b2) && aligned16(w_packed) && aligned8(b3) && aligned16(out) &&
              eps >= 0.f && (kind != LG_PROJ_QKV || (cosv && sinv && aligned8(cosv) && aligned8(sinv))) &&
              (kind != LG_PROJ_PLAIN || (n_store > 0 && n_store <= 512 && n_store % 8 == 0)) &&
              (kind == LG_PROJ_PLAIN || (long long)m * heads * kD < (1LL << 31));
    for (int i = 0; ok && i < nouts; ++i) ok = outs3[i] && aligned16(outs3[i]);
    if (!ok) return bad("lg_linear_cat_ffn_proj");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    LinArgs p{};
    p.a = (const f16*)x, p.ctx0 = (const f16*)ctx0, p.ctx1 = (const f16*)ctx1, p.w = nullptr;
    p.bias = (const f16*)b1, p.out[0] = (f16*)out;
    p.m = m, p.n = k, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    Proj3 q3{};
    q3.b3 = (const f16*)b3, q3.cosv = (const f16*)cosv, q3.sinv = (const f16*)sinv, q3.n_store = n_store;
    for (int i = 0; i < nouts; ++i) q3.out[i] = (f16*)outs3[i];
    const f16 *g = (const f16*)gamma, *be = (const f16*)beta, *wp = (const f16*)w_packed, *bb2 = (const f16*)b2;
    if (kind == LG_PROJ_SPLIT2) launch_ffn_rows<E3_SPLIT2, 2>(p, g, be, eps, wp, bb2, q3, stream);
    else if (kind == LG_PROJ_QKV) launch_ffn_rows<E3_QKV, 3>(p, g, be, eps, wp, bb2, q3, stream);
    else launch_ffn_rows<E3_PLAIN, 2>(p, g, be, eps, wp, bb2, q3, stream);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, "lg_linear_cat_ffn_proj", hipGetErrorString(e));
}

namespace {
// lg_assign_scores' split of the other image: enough workgroups for one round of the chip (256)
int assign_splits(int32_t m, int32_t n, int32_t batch) {
    const long base = (long)((m + 31) / 32 + (n + 31) / 32) * batch;
    int S = 1;
    while (S < 8 && base * S * 2 <= 256) S *= 2;
    return S;
}
}  // namespace

size_t lg_assign_scores_workspace(int32_t m, int32_t n, int32_t batch) {
    if (m <= 0 || n <= 0 || batch <= 0) return 0;
    const size_t b = (size_t)batch, S = (size_t)assign_splits(m, n, batch);
    return (b * m * n * 2 + 255) / 256 * 256 + (b * S * m * 8 + 255) / 256 * 256 + (b * S * n * 8 + 255) / 256 * 256 +
           (b * m * 4 + 255) / 256 * 256 + (b * n * 4 + 255) / 256 * 256;
}

int32_t lg_assign_scores(const void* v, int64_t pair_stride, int32_t ld, int32_t zc, int32_t m, int32_t n, int32_t batch,
                         float* scores, void* workspace, hipStream_t stream) {
    if (m < 0 || n < 0 || batch < 0 || m > 2048 || n > 2048 || n % 8 != 0 || ld < 256 || ld % 8 != 0 || zc < 256 ||
        zc >= ld || pair_stride < (int64_t)(m + n) * ld ||
        ((m > 0 && n > 0 && batch > 0) && (!v || !scores || !workspace || !aligned16(v) || !aligned16(scores) ||
                                          !aligned16(workspace))))
        return bad("lg_assign_scores");
    if (m == 0 || n == 0 || batch == 0) return MHA_HD64_STATUS_SUCCESS;
    AsArgs a{};
    a.v = (const f16*)v, a.ps = (long)pair_stride, a.ld = ld, a.zc = zc, a.m = m, a.n = n, a.rb0 = (m + 31) / 32;
    a.S = assign_splits(m, n, batch);
    char* ws = (char*)workspace;
    const size_t b = (size_t)batch, S = (size_t)a.S;
    a.sim = (f16*)ws;
    a.rpart = (float2*)(ws + (b * m * n * 2 + 255) / 256 * 256);
    a.cpart = (float2*)((char*)a.rpart + (b * S * m * 8 + 255) / 256 * 256);
    a.rterm = (float*)((char*)a.cpart + (b * S * n * 8 + 255) / 256 * 256);
    a.cterm = (float*)((char*)a.rterm + (b * m * 4 + 255) / 256 * 256);
    a.scores = scores;
    const dim3 g1(a.rb0 + (n + 31) / 32, batch, a.S);
    const int oth = m > n ? m : n;  // other-image blocks per wave: ceil(blocks / (8 S))
    const int bpw = ((oth + 31) / 32 + 8 * a.S - 1) / (8 * a.S);
    if (bpw <= 1) hipLaunchKernelGGL(assign_lse_kernel<1>, g1, dim3(512), 0, stream, a);
    else if (bpw <= 2) hipLaunchKernelGGL(assign_lse_kernel<2>, g1, dim3(512), 0, stream, a);
    else if (bpw <= 4) hipLaunchKernelGGL(assign_lse_kernel<4>, g1, dim3(512), 0, stream, a);
    else hipLaunchKernelGGL(assign_lse_kernel<8>, g1, dim3(512), 0, stream, a);
    // combine (with the row / column closes): blocks of 8 W rows x 512 columns (W = 4: 32 rows; 1 where
    // that leaves the chip idle)
    const int cb = (n + 511) / 512;
    if ((long)((m + 31) / 32) * cb * batch >= 128)
        hipLaunchKernelGGL(assign_combine_kernel<4>, dim3((m + 31) / 32, cb, batch), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(assign_combine_kernel<1>, dim3((m + 7) / 8, cb, batch), dim3(256), 0, stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, "lg_assign_scores", hipGetErrorString(e));
}

int32_t lg_linear_qkv_rotary(const void* x, const void* w_perm, const void* b_perm, const void* cosv,
                             const void* sinv, int32_t heads, int32_t n0, int32_t n1, int32_t pairs, int32_t k,
                             void* q0, void* k0, void* v0, void* q1, void* k1, void* v1, hipStream_t stream) {
    const int m = pairs * (n0 + n1), n = 3 * heads * kD;
    if (heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !shape_ok(m, n, k) || !x || !w_perm || !b_perm || !cosv || !sinv ||
        !aligned16(x) || !aligned16(w_perm) || !aligned8(b_perm) || !aligned8(cosv) || !aligned8(sinv))
        return bad("lg_linear_qkv_rotary");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    LinArgs p{};
    p.a = (const f16*)x, p.w = (const f16*)w_perm, p.bias = (const f16*)b_perm;
    p.cosv = (const f16*)cosv, p.sinv = (const f16*)sinv;
    f16* outs[6] = {(f16*)q0, (f16*)k0, (f16*)v0, (f16*)q1, (f16*)k1, (f16*)v1};
    for (int i = 0; i < 6; ++i) p.out[i] = outs[i];
    p.m = m, p.n = n, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    return launch<EPI_QKV_ROTARY, false>(p, stream, "lg_linear_qkv_rotary");
}

int32_t lg_linear_split2(const void* x, const void* w, const void* bias, int32_t heads, int32_t n0, int32_t n1,
                         int32_t pairs, int32_t k, void* a0, void* a1, void* b0, void* b1, hipStream_t stream) {
    const int m = pairs * (n0 + n1), n = 2 * heads * kD;
    if (heads <= 0 || n0 < 0 || n1 < 0 || pairs < 0 || !shape_ok(m, n, k) || !x || !w || !bias || !aligned16(x) ||
        !aligned16(w) || !aligned8(bias))
        return bad("lg_linear_split2");
    if (m == 0) return MHA_HD64_STATUS_SUCCESS;
    LinArgs p{};
    p.a = (const f16*)x, p.w = (const f16*)w, p.bias = (const f16*)bias;
    f16* outs[4] = {(f16*)a0, (f16*)a1, (f16*)b0, (f16*)b1};
    for (int i = 0; i < 4; ++i) p.out[i] = outs[i];
    p.m = m, p.n = n, p.k = k, p.heads = heads, p.n0 = n0, p.n1 = n1;
    return launch<EPI_SPLIT2, false>(p, stream, "lg_linear_split2");
}

int32_t lg_linear_set_wide(int32_t mode) {
    wide_mode();
    return g_wide.exchange(mode < 0 ? -1 : (mode > 5 ? 5 : mode));
}

int32_t lg_glue_abi_version(void) { return LG_GLUE_ABI_VERSION; }

#ifdef LG_LN_STAMPS
int32_t lg_diag_ln_stamps(void* host_dst) {  // (diagnostic build only: not in the header)
    return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_ln_stamps), sizeof(g_ln_stamps)) == hipSuccess ? 0 : 1;
}
#endif
#ifdef LG_FR_STAMPS
int32_t lg_diag_fr_stamps(void* host_dst) {  // (diagnostic build only: not in the header)
    return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_fr_stamps), sizeof(g_fr_stamps)) == hipSuccess ? 0 : 1;
}
#endif
int32_t lg_linear_set_ln_fused(int32_t on) { return g_ln_fused.exchange(on == 2 ? 2 : on ? 1 : 0); }
int32_t lg_linear_set_ffn_fused(int32_t mode) { return g_ffn_fused.exchange(mode >= 0 && mode <= 3 ? mode : 1); }

}  // extern "C"
