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

#include "lightglue_glue.h"
#include "mha_hd64.h"
#include "mha_hd64_internal.h"

namespace {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) f16x8 lds_f16x8;

constexpr int kBM = 64, kBN = 64, kKC = 128;  // tile rows, tile channels, K columns per LDS chunk
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
    int st16;          // 256-row forms, EPI_BIAS: 16-B row-segment stores (default; LG_LINEAR_ST16=0: off)
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
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = acc[4 * g + t] + (float)bias4[g][t];
        if constexpr (EPI == EPI_BIAS) {
            if (p.res) {
#pragma unroll
                for (int t = 0; t < 4; ++t) v[t] += (float)aux0[g][t];
            }
            *reinterpret_cast<f16x4*>(p.out[0] + (size_t)m * p.n + n) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
        } else {
            const int hd = p.heads * kD;
            const int part = n / hd, h = (n % hd) / kD, d = n % kD;
            const LinRow lr = lin_row(p, m, h);
            const bool first = lr.first;
            if constexpr (EPI == EPI_QKV_ROTARY) {
                if (part < 2) {  // q, k: (x0, x1) -> (x0 c - x1 s, x1 c + x0 s), pairs (d, d+1)
                    const f16x4 cc = aux0[g], ss = aux1[g];
#pragma unroll
                    for (int t = 0; t < 4; t += 2) {
                        const float x0 = v[t], x1 = v[t + 1];
                        v[t] = x0 * (float)cc[t] - x1 * (float)ss[t];
                        v[t + 1] = x1 * (float)cc[t + 1] + x0 * (float)ss[t + 1];
                    }
                }
            }
            f16* dst = p.out[(first ? 0 : (EPI == EPI_QKV_ROTARY ? 3 : 1)) + (EPI == EPI_QKV_ROTARY ? part : 2 * part)];
            *reinterpret_cast<f16x4*>(dst + lr.off + d) =
                f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
        }
    }
}

// One lane's 4 consecutive output channels n..n+3 of activation row `row` (acc elements 4g..4g+3):
// bias, then residual (EPI_BIAS) / rotary + per-image head-major scatter / head split.
template <int EPI>
__device__ __forceinline__ void epi_store(const LinArgs& p, int row, int n, const f32x16& acc, int g) {
    const f16x4 b4 = *reinterpret_cast<const f16x4*>(p.bias + n);
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = acc[4 * g + u] + (float)b4[u];
    if constexpr (EPI == EPI_BIAS) {
        if (p.res) {
            const f16x4 rr = *reinterpret_cast<const f16x4*>(p.res + (size_t)row * p.n + n);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += (float)rr[u];
        }
        *reinterpret_cast<f16x4*>(p.out[0] + (size_t)row * p.n + n) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
    } else {
        const int hd = p.heads * kD;
        const int part = n / hd, h = (n % hd) / kD, d = n % kD;
        const LinRow lr = lin_row(p, row, h);
        if constexpr (EPI == EPI_QKV_ROTARY) {
            if (part < 2) {
                const f16x4 cc = *reinterpret_cast<const f16x4*>(p.cosv + (size_t)row * kD + d);
                const f16x4 ss = *reinterpret_cast<const f16x4*>(p.sinv + (size_t)row * kD + d);
#pragma unroll
                for (int u = 0; u < 4; u += 2) {
                    const float x0 = v[u], x1 = v[u + 1];
                    v[u] = x0 * (float)cc[u] - x1 * (float)ss[u];
                    v[u + 1] = x1 * (float)cc[u + 1] + x0 * (float)ss[u + 1];
                }
            }
        }
        f16* dst = p.out[(lr.first ? 0 : (EPI == EPI_QKV_ROTARY ? 3 : 1)) + (EPI == EPI_QKV_ROTARY ? part : 2 * part)];
        *reinterpret_cast<f16x4*>(dst + lr.off + d) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
    }
}

// One 32 x 32 block of a 256-row form (lane = activation row `row`, channels nb0 + 8g + 4hh + t in
// acc[4g + t]): with p.st16 and EPI_BIAS, v_permlane32_swap pairs (g, g + 1) between the two
// half-waves so each lane stores 8 consecutive channels (16 B) per pair (lg_linear_cat 35.0 -> 32.3
// us, lg_linear 23.7 -> 21.9 at P = 16; linear_ab_st16.jsonl); else epi_store per group.
template <int EPI>
__device__ __forceinline__ void epi_block(const LinArgs& p, int row, int nb0, const f32x16& acc, int hh) {
    if constexpr (EPI == EPI_BIAS) {
        if (p.st16) {
            typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
            typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
            u32x2_ rk[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = nb0 + 8 * g + 4 * hh;
                const f16x4 b4 = *reinterpret_cast<const f16x4*>(p.bias + n);
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = acc[4 * g + u] + (float)b4[u];
                if (p.res) {
                    const f16x4 rr = *reinterpret_cast<const f16x4*>(p.res + (size_t)row * p.n + n);
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] += (float)rr[u];
                }
                rk[g] = __builtin_bit_cast(u32x2_, f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]});
            }
#pragma unroll
            for (int k = 0; k < 4; k += 2) {
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const auto sw = __builtin_amdgcn_permlane32_swap(rk[k][w], rk[k + 1][w], false, false);
                    rk[k][w] = sw[0];
                    rk[k + 1][w] = sw[1];
                }
                *reinterpret_cast<u32x4_*>(p.out[0] + (size_t)row * p.n + nb0 + 8 * (k + hh)) =
                    u32x4_{rk[k][0], rk[k][1], rk[k + 1][0], rk[k + 1][1]};
            }
            return;
        }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) epi_store<EPI>(p, row, nb0 + 8 * g + 4 * hh, acc, g);
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
template <bool GATHER, int BK, int NWP, int NAP>
__device__ __forceinline__ TileSrc<NWP, NAP> tile_src(const LinArgs& p, int m0, int n0, int wave, int lane) {
    constexpr int U = BK / 8, RP = 1024 / (2 * BK);
    TileSrc<NWP, NAP> t;
#pragma unroll
    for (int h = 0; h < NWP; ++h) {
        const int row = RP * (wave + 8 * h) + lane / U;
        const int wr = min(n0 + row, p.n - 1);
        t.w[h] = p.w + (size_t)wr * p.k + src_unit<BK>(row, lane % U) * 8;
    }
#pragma unroll
    for (int h = 0; h < NAP; ++h) {
        const int row = RP * (wave + 8 * h) + lane / U;
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
// wave + 8h at sb, A pieces at sb + BN BK 2
template <bool GATHER, int BK, int KS, int BN, int NWP, int NAP>
__device__ __forceinline__ void tile_issue(const TileSrc<NWP, NAP>& t, int ks, char* sb, int wave) {
#pragma unroll
    for (int h = 0; h < NWP; ++h)
        __builtin_amdgcn_global_load_lds((const void*)(t.w[h] + ks * BK),
                                         (__attribute__((address_space(3))) void*)(sb + (wave + 8 * h) * 1024), 16, 0, 0);
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
                                         (__attribute__((address_space(3))) void*)(sb + BN * BK * 2 + (wave + 8 * h) * 1024),
                                         16, 0, 0);
    }
}

// ---- the wide form, for launches with many rows (several image pairs per forward) ----
// Workgroup: 256 rows (m) x 128 output channels (n) a tile, persistent over tiles (the DMA ring
// runs on across tile seams: the next tile's first two K steps load during the current tile's
// last two), 8 waves as 4 (m) x 2 (n) tiles of 64 x 64
// (2 x 2 MFMA blocks of 32 x 32 each); K in 64-deep steps through a 3-stage LDS-DMA ring (48 KiB a
// stage: W [128 rows][128 B] + A [256 rows][128 B], 16-B units XOR-swizzled by (row >> 1) & 7 on
// the source address: conflict-free ds_read_b128 in every lane group), two steps in flight. Per
// step and wave: 16 MFMA beside 16 fragment reads. The k16 blocks enter each accumulator in the
// same order as in linear_kernel, so both forms give the same bits. Against the 64 x 64 form it
// moves a quarter of the operand bytes per MAC out of L2 (128 KiB per 64 x 64 x 512 tile there).
constexpr int kWM = 256, kWN = 128, kWK = 64;
constexpr int kWStage = (kWM + kWN) * kWK * 2;  // 48 KiB
constexpr int kWStages = 3;
constexpr int kWGrid = 256;  // one workgroup per CU

template <int EPI, bool GATHER, int KS>
__global__ __launch_bounds__(512, 1) void linear_wide_kernel(LinArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[kWStages * kWStage];  // 144 KiB
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 3, wn = wave >> 2;  // this wave's 64 x 64 tile of the 256 x 128
    const int r = lane & 31, hh = lane >> 5;
    // Persistent and XCD-aware: the workgroups of XCD x walk the contiguous tile range [jb, je)
    // (tile j = m tile j / ntiles, n tile j % ntiles: the n tiles of one m tile run side by side
    // on one XCD, so their A tile is read through one L2), every G-th tile from their local index.
    const int T = p.total, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8), je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    const int ntiles = p.n / kWN;
    const int j0 = jb + loc;
    if (j0 >= je) return;
    const int ntile_w = (je - j0 + G - 1) / G;  // tiles of this workgroup
    const int nsteps = ntile_w * KS;            // K steps over all of them

    // DMA sources of this workgroup's tile t (computed once per tile)
    auto src_of = [&](int t) {
        const int jt = j0 + G * t, mt = jt / ntiles;
        return tile_src<GATHER, kWK, 2, 4>(p, mt * kWM, (jt - mt * ntiles) * kWN, wave, lane);
    };
    TileSrc<2, 4> cur = src_of(0), nxt = cur;
    tile_issue<GATHER, kWK, KS, kWN>(cur, 0, smem, wave);
    tile_issue<GATHER, kWK, KS, kWN>(cur, 1, smem + kWStage, wave);

    unsigned wro[2], aro[2];  // per block: row offset and swizzle key of this lane's fragment row
    int wsw[2], asw[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int wrow = wn * 64 + 32 * b + r, arow = wm * 64 + 32 * b + r;
        wro[b] = (unsigned)(wrow * 128), wsw[b] = (wrow >> 1) & 7;
        aro[b] = (unsigned)(kWN * 128 + arow * 128), asw[b] = (arow >> 1) & 7;
    }
    int st = 0;  // stage of global step gs
    for (int t = 0; t < ntile_w; ++t) {
        const int jt = j0 + G * t;
        const int mt = jt / ntiles, m0 = mt * kWM, n0 = (jt - mt * ntiles) * kWN;
        const bool more = t + 1 < ntile_w;
        if (more) nxt = src_of(t + 1);
        f32x16 acc[2][2] = {};  // [n block][m block]
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int gs = t * KS + ks;
            // step gs landed for this wave's 6 DMAs (step gs + 1's stay in flight), then for
            // everyone's; after this barrier every wave is past step gs − 1, so its stage takes
            // step gs + 2 (lgkmcnt(0): this wave's fragment reads of step gs − 1 are done)
            if (gs + 1 < nsteps) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            {
                char* const fb = smem + (st == 0 ? 2 : st - 1) * kWStage;
                if (ks + 2 < KS) tile_issue<GATHER, kWK, KS, kWN>(cur, ks + 2, fb, wave);
                else if (more) tile_issue<GATHER, kWK, KS, kWN>(nxt, ks + 2 - KS, fb, wave);
            }
            const unsigned sb = (unsigned)(st * kWStage);
            st = st == 2 ? 0 : st + 1;
#pragma unroll
            for (int s = 0; s < kWK / 16; ++s) {
                f16x8 wf[2], af[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int u = 2 * s + hh;
                    wf[b] = *(lds_f16x8*)(lds + sb + wro[b] + ((u ^ wsw[b]) << 4));
                    af[b] = *(lds_f16x8*)(lds + sb + aro[b] + ((u ^ asw[b]) << 4));
                }
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb)
                        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[nb], af[mb], acc[nb][mb], 0, 0, 0);
            }
        }

        // ---- epilogue: per (n block, m block), lane = activation row; acc[.][.][4g + t] =
        // channel n0 + wn*64 + 32 nb + 8g + 4hh + t (the 64 x 64 form's epilogue per 32 x 32
        // block). Its operand loads return after the next tile's first two DMA steps (issued
        // above): the wait for them is the wait the next tile's first step makes anyway. ----
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int row = m0 + wm * 64 + 32 * mb + r;
            if (row >= p.m) continue;
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) epi_block<EPI>(p, row, n0 + wn * 64 + 32 * nb, acc[nb][mb], hh);
        }
        cur = nxt;
    }
}

// ---- the square form: 256 x 256 tiles, K in 32-deep steps through a 4-stage ring (32 KiB a
// stage: W and A [256 rows][64 B], 16-B units XOR-swizzled by (row >> 2) & 3), three steps in
// flight; 8 waves as 4 (m) x 2 (n) tiles of 64 rows x 128 channels (2 x 4 MFMA blocks). A step
// stages 32 KiB for 4.2 MFLOP (the 256 x 128 form: 48 KiB). Same k16 order per accumulator as
// the other forms: same bits. (lg_linear_set_wide(2) / LG_LINEAR_WIDE=2, where n % 256 == 0.)
constexpr int kSM_ = 256, kSN = 256, kSK = 32;
constexpr int kSStage = (kSM_ + kSN) * kSK * 2;  // 32 KiB

// NST stages (4: 128 KiB; 5: the whole 160 KiB), NST − 1 steps in flight
template <int EPI, bool GATHER, int KS, int NST>
__global__ __launch_bounds__(512, 1) void linear_sq_kernel(LinArgs p) {
    __shared__ __attribute__((aligned(16))) char smem[NST * kSStage];
    lds_char* const lds = (lds_char*)smem;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 3, wn = wave >> 2;  // this wave's 64 x 128 tile of the 256 x 256
    const int r = lane & 31, hh = lane >> 5;
    const int T = p.total, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8), je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    const int ntiles = p.n / kSN;
    const int j0 = jb + loc;
    if (j0 >= je) return;
    const int ntile_w = (je - j0 + G - 1) / G;
    const int nsteps = ntile_w * KS;

    // DMA sources of this workgroup's tile t (computed once per tile)
    auto src_of = [&](int t) {
        const int jt = j0 + G * t, mt = jt / ntiles;
        return tile_src<GATHER, kSK, 2, 2>(p, mt * kSM_, (jt - mt * ntiles) * kSN, wave, lane);
    };
    TileSrc<2, 2> cur = src_of(0), nxt = cur;
#pragma unroll
    for (int i = 0; i < NST - 1; ++i) tile_issue<GATHER, kSK, KS, kSN>(cur, i, smem + i * kSStage, wave);

    unsigned wro[4], aro[2];
    int wsw[4], asw[2];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int wrow = wn * 128 + 32 * b + r;
        wro[b] = (unsigned)(wrow * 64), wsw[b] = (wrow >> 2) & 3;
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int arow = wm * 64 + 32 * b + r;
        aro[b] = (unsigned)(kSN * 64 + arow * 64), asw[b] = (arow >> 2) & 3;
    }
    int st = 0;
    for (int t = 0; t < ntile_w; ++t) {
        const int jt = j0 + G * t;
        const int mt = jt / ntiles, m0 = mt * kSM_, n0 = (jt - mt * ntiles) * kSN;
        const bool more = t + 1 < ntile_w;
        if (more) nxt = src_of(t + 1);
        f32x16 acc[4][2] = {};  // [n block][m block]
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int gs = t * KS + ks;
            // step gs landed (up to NST − 2 later steps stay in flight: 4 DMAs each per wave),
            // then everyone's; past this barrier every wave is done with step gs − 1's stage
            const int later = min(NST - 2, nsteps - 1 - gs);
            if (later >= 3) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
            else if (later == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
            else if (later == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            {
                char* const fb = smem + (st == 0 ? NST - 1 : st - 1) * kSStage;
                if (ks + NST - 1 < KS) tile_issue<GATHER, kSK, KS, kSN>(cur, ks + NST - 1, fb, wave);
                else if (more) tile_issue<GATHER, kSK, KS, kSN>(nxt, ks + NST - 1 - KS, fb, wave);
            }
            const unsigned sb = (unsigned)(st * kSStage);
            st = st == NST - 1 ? 0 : st + 1;
#pragma unroll
            for (int s = 0; s < kSK / 16; ++s) {
                const int u = 2 * s + hh;
                f16x8 wf[4], af[2];
#pragma unroll
                for (int b = 0; b < 4; ++b) wf[b] = *(lds_f16x8*)(lds + sb + wro[b] + ((u ^ wsw[b]) << 4));
#pragma unroll
                for (int b = 0; b < 2; ++b) af[b] = *(lds_f16x8*)(lds + sb + aro[b] + ((u ^ asw[b]) << 4));
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb)
                        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[nb], af[mb], acc[nb][mb], 0, 0, 0);
            }
        }
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int row = m0 + wm * 64 + 32 * mb + r;
            if (row >= p.m) continue;
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) epi_block<EPI>(p, row, n0 + wn * 128 + 32 * nb, acc[nb][mb], hh);
        }
        cur = nxt;
    }
}

// The wide form where it fills the chip: at least one round of its 256 x 128 tiles (n a multiple of
// 128). lg_linear_set_wide(0 / 1) or LG_LINEAR_WIDE=0 / 1 forces it off / on (where n allows), for
// tests and A/B timing; -1 (the default) chooses by size.
std::atomic<int> g_wide{-2};
int wide_mode() {
    int v = g_wide.load();
    if (v == -2) {
        const char* e = std::getenv("LG_LINEAR_WIDE");
        int expect = -2;
        g_wide.compare_exchange_strong(expect, e ? (e[0] == '2' ? 2 : e[0] == '1' ? 1 : 0) : -1);
        v = g_wide.load();
    }
    return v;
}
bool use_wide(const LinArgs& p) {
    if (p.n % kWN) return false;
    const int w = wide_mode();
    if (w >= 0) return w >= 1;
    return (long)((p.m + kWM - 1) / kWM) * (p.n / kWN) >= 256;
}
// the square form: forced (mode 2), or by size where its tiles fill whole rounds of the chip
// (N = 512 at P = 16, N = 1024: cat 36.5 -> 33.2 us, cross qk|v 27.5 -> 25.1; N = 256 / 768 take
// half / one and a half rounds of it and stay on the 256 x 128 form; linear_ab_square.jsonl)
bool use_sq(const LinArgs& p) {
    if (p.n % kSN) return false;
    const int w = wide_mode();
    if (w >= 0) return w >= 2;
    const long t = (long)((p.m + kSM_ - 1) / kSM_) * (p.n / kSN);
    return t >= kWGrid && (t % kWGrid == 0 || t >= 4 * kWGrid);
}

int st16_env() {
    static const int v = [] {
        const char* e = std::getenv("LG_LINEAR_ST16");  // (0: the per-group 8-B stores)
        return (e && e[0] == '0') ? 0 : 1;
    }();
    return v;
}

template <int EPI, bool GATHER>
int32_t launch(LinArgs& p, hipStream_t stream, const char* what) {
    p.st16 = st16_env();
    if (use_sq(p)) {
        p.mtiles = (p.m + kSM_ - 1) / kSM_;
        p.total = p.mtiles * (p.n / kSN);
        const int grid = p.total < kWGrid ? p.total : kWGrid;
        if (wide_mode() == 3) {  // (A/B: five stages)
            if (p.k == 256)
                hipLaunchKernelGGL((linear_sq_kernel<EPI, GATHER, 8, 5>), dim3(grid), dim3(512), 0, stream, p);
            else
                hipLaunchKernelGGL((linear_sq_kernel<EPI, GATHER, 16, 5>), dim3(grid), dim3(512), 0, stream, p);
        } else if (p.k == 256) {
            hipLaunchKernelGGL((linear_sq_kernel<EPI, GATHER, 8, 4>), dim3(grid), dim3(512), 0, stream, p);
        } else {
            hipLaunchKernelGGL((linear_sq_kernel<EPI, GATHER, 16, 4>), dim3(grid), dim3(512), 0, stream, p);
        }
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                               : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, what, hipGetErrorString(e));
    }
    if (use_wide(p)) {
        p.mtiles = (p.m + kWM - 1) / kWM;
        p.total = p.mtiles * (p.n / kWN);
        const int grid = p.total < kWGrid ? p.total : kWGrid;  // persistent: one round
        if (p.k == 256)
            hipLaunchKernelGGL((linear_wide_kernel<EPI, GATHER, 4>), dim3(grid), dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((linear_wide_kernel<EPI, GATHER, 8>), dim3(grid), dim3(512), 0, stream, p);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                               : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, what, hipGetErrorString(e));
    }
    p.mtiles = (p.m + kBM - 1) / kBM;
    p.total = p.mtiles * (p.n / kBN);
    if (p.k == 256)
        hipLaunchKernelGGL((linear_kernel<EPI, GATHER, 2>), dim3(p.total), dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((linear_kernel<EPI, GATHER, 4>), dim3(p.total), dim3(256), 0, stream, p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MHA_HD64_STATUS_SUCCESS
                           : mha_hd64::report_error(MHA_HD64_STATUS_LAUNCH_FAILED, what, hipGetErrorString(e));
}

bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }
bool aligned8(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 7) == 0; }
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
    return g_wide.exchange(mode < 0 ? -1 : (mode > 3 ? 3 : mode));
}

}  // extern "C"
