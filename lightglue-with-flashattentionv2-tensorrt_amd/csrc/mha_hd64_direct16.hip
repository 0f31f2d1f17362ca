// mha_hd64_direct16.hip — single-pass FlashAttention forward, head_dim = 64, 16-row query blocks,
// for gfx950 (MI355X).
//
// The operator of mha_hd64_kernels.hip / mha_hd64_direct.hip (O = softmax(Q·Kᵀ·0.125)·V per
// (batch, head); the reference's attention_headdim_64_fp16in_fp16out.cu:253-733 /
// …fp16in_fp32out.cu:253-703) for launches whose 32-row blocks fill at most half the chip: the
// plugin's single 1x4x1024x1024 call is 128 blocks of 32 rows (128 of 256 CUs busy, the other
// half idle) but 256 blocks of 16 rows. Each workgroup streams all of its head's keys as the
// 32-row kernel does (the per-CU load volume is the same; twice the L2 reads in total), and
// each wave does half the arithmetic.
//  * 4 waves, wave w owns keys [64·TPW·w, 64·TPW·(w+1)); K and V by LDS-DMA into the wave's own
//    slots (K(t) into slot t, V(t) over it once K(t)'s fragments are in registers), no barrier
//    before the epilogue — the 32-row kernel's load schedule.
//  * Sᵀ = K·Qᵀ on v_mfma_f32_16x16x32_f16: per 64-key tile 4 key blocks x 2 dim steps. A lane
//    holds keys 16kb + 4g + j (j < 4) of query i = lane % 16 (g = lane / 16), so the fp16 P of
//    key blocks 2u and 2u+1 concatenated is directly the B operand of step u of Oᵀ = Vᵀ·Pᵀ (key
//    order k = 8g + j <-> 32u + 4g + j, 8g + 4 + j <-> 32u + 16 + 4g + j), and the matching A
//    operand (Vᵀ) is two ds_read_b64_tr_b16 of 4 rows each (rows 4g..4g+3 and 16 + 4g..).
//  * Softmax as the 32-row kernel: the first tile sets the running max, the later tiles' scores
//    wait for ONE lazy-rescale decision (threshold 8, log2 units), row sums on the matrix pipe
//    (an all-ones A operand), masking of keys past nkv on the vector pipe (partial tiles only).
//  * Epilogue: each wave stages Oᵀ (fp32) and (m, l) in its region; one barrier; 256 threads
//    merge (row, 4 dims) over the 4 waves and store O.
// LDS images (bank rule of cdna_hip_programming.md §2): K rows XOR chunk (row>>1)&7 (k_off: the
// 16 rows of every ds_read_b128 lane group on distinct 16-B slots); V rows XOR chunk
// 2·((row>>1)&3) (the 8 rows x 2 chunks of every tr_b16 half-wave on distinct slots).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

// Diagnostic timestamps (-DMHA_STAMPS builds, tools/dstamps.py ... 22): wave 0's s_memtime at the
// phase boundaries of mha_hd64_direct.hip's slots (0 entry, 1 Q + K(0) landed, 3 V(0) landed,
// 2 later tiles' exponentials done, 4 PV done, 5 after the epilogue barrier, 6 stores acked).
#ifdef MHA_STAMPS
#define DSTAMP(slot)                                                                              \
    do {                                                                                          \
        unsigned long long t_;                                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
        if (threadIdx.x == 0) a.stamps[blockIdx.x * 8 + (slot)] = t_;                             \
    } while (0)
#else
#define DSTAMP(slot) \
    do {             \
    } while (0)
#endif

#ifndef MHA_D16_WAVES
#define MHA_D16_WAVES 4  // waves per workgroup for nkv in (512, 1024]; 8 (8 x 2 tiles, two waves per
                         // SIMD) measured 5.23 against 4.89 us at 1x4x1024^2: an A/B hook only
#endif

namespace mha_hd64 {
namespace {

template <int N>
__device__ __forceinline__ void wait_vmc() {
    static_assert(N % 8 == 0 && N <= 40, "vmcnt");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
}
// s_waitcnt vmcnt(8 * groups) for a value known after unrolling
__device__ __forceinline__ void wait_groups(int groups) {
    switch (groups) {
        case 0: wait_vmc<0>(); break;
        case 1: wait_vmc<8>(); break;
        case 2: wait_vmc<16>(); break;
        case 3: wait_vmc<24>(); break;
        case 4: wait_vmc<32>(); break;
        default: wait_vmc<40>(); break;
    }
}

// max over the lanes of one query (i, i+16, i+32, i+48): v_permlane32_swap then v_permlane16_swap
__device__ __forceinline__ float xquad_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    const float y = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
    return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

__device__ __forceinline__ float max16(const f32x4 (&c)[4]) {
    float t[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) t[kb] = fmaxf(fmaxf(c[kb][0], c[kb][1]), fmaxf(c[kb][2], c[kb][3]));
    return fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3]));
}

// PASSES = 2 (nkv in (1024, 2048], 4 waves): each wave's 2·TPW tiles go through its TPW slots twice,
// as in mha_hd64_direct.hip's two-pass form (pass 1's K(TPW + t) refills slot t once pass 0's PV
// has V(t)'s fragments in registers).
template <typename TOut, int KW, int TPW, bool MULTI, int PASSES = 1, bool F32IN = false>
// The single call's own arguments come first as plain scalars (q0 .. qtiles0: 12 dwords), so the
// command processor can preload them into SGPRs (-amdgpu-kernarg-preload-count, Makefile) and the
// first loads need no dependent kernarg fetch; grouped launches (MULTI) read the table `a`.
__global__ __launch_bounds__(64 * KW, 1) void mha_hd64_direct16_kernel(const void* q0, const void* k0, const void* v0,
                                                                        void* o0, int total_blocks, int nq0, int nkv0,
                                                                        int qtiles0, FwdArgs a) {
    static_assert(TPW >= 2 && TPW <= 4 && (KW == 4 || KW == 8), "waves x tiles per wave");
    static_assert(PASSES == 1 || (PASSES == 2 && TPW == 4 && KW == 4), "two passes: 4 waves x 2 x 4 tiles");
    static_assert(!F32IN || KW == 4, "fp32 inputs: the 4-wave forms");
#ifndef MHA_D16_STAGE16
#define MHA_D16_STAGE16 0  // A/B hook: fp16 K/V through VGPRs + ds_write (the F32IN pipeline) instead of LDS-DMA
#endif
    // the VGPR-staged pipeline: fp32 inputs always; fp16 inputs under the A/B hook (4-wave forms)
    constexpr bool STAGED = F32IN || (MHA_D16_STAGE16 && KW == 4);
    using TIn = std::conditional_t<F32IN, float, f16>;
    constexpr unsigned ISZ = sizeof(TIn);
    constexpr int BLOCK_M = 16;                     // query rows per workgroup
    constexpr int WAVE_KEYS = kTileKV * TPW * PASSES;
    constexpr int OROW = 68;                        // epilogue fp32 row pitch
    constexpr int EPI_WAVE = BLOCK_M * OROW * 4;
    constexpr int RS = TPW * kTileBytes > EPI_WAVE ? TPW * kTileBytes : EPI_WAVE;
    constexpr int LDS_BYTES = KW * RS + KW * BLOCK_M * 2 * 4;
    static_assert(RS % 128 == 0 && LDS_BYTES <= 160 * 1024, "LDS layout");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    lds_char* const lds = (lds_char*)smem;

    DSTAMP(0);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int i16 = lane & 15;  // query column of the MFMA tiles
    const int g = lane >> 4;    // operand k-group / result row group
    // XCD-aware order (as the other kernels): consecutive j share an XCD and its L2
    int qtile, bh, j;
    {
        const int T = total_blocks, L = blockIdx.x;
        const int q8 = T >> 3, r8 = T & 7, xcd = L & 7;
        j = xcd * q8 + min(xcd, r8) + (L >> 3);
    }
    int ci = 0;
    if constexpr (MULTI) {
#pragma unroll
        for (int i = 1; i < kMaxCalls; ++i) ci += (int)((i < a.n_calls) & (j >= a.c[i].block_begin));
    }
    CallArgs ca;
    if constexpr (MULTI) {
        ca = pick_call(a, ci);
    } else {
        ca.q = q0;
        ca.k = k0;
        ca.v = v0;
        ca.o = o0;
        ca.nq = nq0;
        ca.nkv = nkv0;
        ca.qtiles = qtiles0;
        ca.block_begin = 0;
    }
    {
        const int jl = j - ca.block_begin;
        qtile = jl % ca.qtiles;
        bh = jl / ca.qtiles;
    }
    const int nq = ca.nq, nkv = ca.nkv;
    const f16* Qb = reinterpret_cast<const f16*>(ca.q) + (size_t)bh * nq * kHeadDim;
    const f16* Kb = reinterpret_cast<const f16*>(ca.k) + (size_t)bh * nkv * kHeadDim;
    const f16* Vb = reinterpret_cast<const f16*>(ca.v) + (size_t)bh * nkv * kHeadDim;
    const __amdgpu_buffer_rsrc_t q_rs = make_rsrc(Qb, (unsigned)nq * kHeadDim * 2);
    const __amdgpu_buffer_rsrc_t k_rs = make_rsrc(Kb, (unsigned)nkv * kHeadDim * 2);
    const __amdgpu_buffer_rsrc_t v_rs = make_rsrc(Vb, (unsigned)nkv * kHeadDim * 2);
    const int q_row = qtile * BLOCK_M + i16;
    const int key0 = wave * WAVE_KEYS;
    const int n_t = max(0, min(TPW * PASSES, (nkv - key0 + kTileKV - 1) / kTileKV));
    const unsigned region = (unsigned)wave * RS;

    f32x4 o[4];  // Oᵀ: dims 16db + 4g + j of query i16
    f32x4 l_acc;
    float m_run = 0.f;

    if (n_t == 0) {  // a wave wholly past nkv contributes nothing (m = -inf in the merge)
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
        l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
    } else if constexpr (STAGED) {
        // ---- the Float boundary inside the kernel: fp32 Q/K/V through VGPRs ----
        // fp32 rows are 256 B. Lane L of piece i (rows 8i..8i+7 of a tile) loads the 8 floats of
        // chunk c = L & 7 of row 8i + L/8, rounds them to fp16 (RNE, as the reference's convert
        // kernel …fp16in_fp32out.cu:706-768) and writes the 16-B chunk where the K / V image puts
        // it (the same images as the DMA path). Tiles in the order K(0..TPW-1), V(0..TPW-1), two
        // in flight; tile j goes into slot j % TPW once that slot's K fragments are in registers.
        // Loads are plain (compiler-tracked) buffer loads: no hand-counted waits in this form.
        const TIn* Qf = reinterpret_cast<const TIn*>(ca.q) + (size_t)bh * nq * kHeadDim;
        const TIn* Kf = reinterpret_cast<const TIn*>(ca.k) + (size_t)bh * nkv * kHeadDim;
        const TIn* Vf = reinterpret_cast<const TIn*>(ca.v) + (size_t)bh * nkv * kHeadDim;
        const __amdgpu_buffer_rsrc_t q32 = make_rsrc(Qf, (unsigned)nq * kHeadDim * ISZ);
        const __amdgpu_buffer_rsrc_t k32 = make_rsrc(Kf, (unsigned)nkv * kHeadDim * ISZ);
        const __amdgpu_buffer_rsrc_t v32 = make_rsrc(Vf, (unsigned)nkv * kHeadDim * ISZ);
        struct Tile {
            Raw8<TIn> p[8];
        };
        const int prow = lane >> 3, pc = lane & 7;
        // item j of the order K(0..TPW-1), V(0..TPW-1) of pass 0, then the same for pass 1:
        // tile TPW·pass + (j % TPW) of K (first half of the pass) or V, into slot j % TPW
        constexpr int NI = 2 * TPW * PASSES;
        auto ld_tile = [&](int j, Tile& x) {
            const int r = j % (2 * TPW), t = (j / (2 * TPW)) * TPW + r % TPW;
            const unsigned base = ((unsigned)(key0 + kTileKV * t + prow) * kHeadDim + 8 * pc) * ISZ;
#pragma unroll
            for (int i = 0; i < 8; ++i) bload8(x.p[i], r < TPW ? k32 : v32, base + i * 8 * kHeadDim * ISZ, 0);
        };
        auto st_tile = [&](int j, const Tile& x) {
            const int r = j % (2 * TPW);
            const unsigned slot = region + (unsigned)(r % TPW) * kTileBytes;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = 8 * i + prow;
                const int pos = r < TPW ? (pc ^ ((row >> 1) & 7)) : (pc ^ (((row >> 1) & 3) << 1));
                lds_write16(lds, slot + row * 128 + (pos << 4), to_f16(x.p[i]));
            }
        };
        // Q: Q[q_row][32s+8g..+7] rounded to fp16, then scaled as the fp16 path does
        f16x8 qf[2];
        {
            Raw8<TIn> qr[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) bload8(qr[s], q32, (unsigned)(q_row * kHeadDim + 32 * s + 8 * g) * ISZ, 0);
            const float sc = kScaleLog2;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const u32x4 in = __builtin_bit_cast(u32x4, to_f16(qr[s]));
                u32x4 outv;
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[1,0,0]\n\t"
                        "v_fma_mixhi_f16 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                        : "=&v"(outv[w])
                        : "v"(in[w]), "v"(sc));
                qf[s] = __builtin_bit_cast(f16x8, outv);
            }
        }
        auto read_k = [&](int t, f16x8(&kf)[4][2]) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    kf[kb][s] = lds_read16(lds, region + k_off(kTileKV * t + 16 * kb + i16, 4 * s + g));
        };
        const f16x8 ones = f16x8{1, 1, 1, 1, 1, 1, 1, 1};
        const int qq = (lane & 15) >> 2, pp = lane & 3;
        const int sw = ((4 * g + qq) >> 1) & 3;
        unsigned vbase[4];
#pragma unroll
        for (int db = 0; db < 4; ++db)
            vbase[db] = region + (unsigned)(4 * g + qq) * 128 + ((2 * (db ^ sw) + (pp >> 1)) << 4) + 8 * (pp & 1);
        f16x8 p[TPW][2];
        f32x4 sc[TPW][4];
        auto pv = [&](int t, bool first) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    const unsigned off = (unsigned)(t * kTileBytes + 128 * 32 * u);
                    const f16x8 va = cat8(tr_read(lds, vbase[db] + off), tr_read(lds, vbase[db] + off + 16 * 128));
                    o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, p[t][u], (first && u == 0) ? f32x4{} : o[db], 0,
                                                                   0, 0);
                }
                l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, p[t][u], (first && u == 0) ? f32x4{} : l_acc, 0,
                                                               0, 0);
            }
        };
        auto exp_pack = [&](f32x4(&c)[4], f16x8(&pt)[2], float m) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int e = 0; e < 4; ++e) c[kb][e] = __builtin_amdgcn_exp2f(c[kb][e] - m);
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pt[u] = f16x8{(f16)c[2 * u][0],     (f16)c[2 * u][1],     (f16)c[2 * u][2],     (f16)c[2 * u][3],
                              (f16)c[2 * u + 1][0], (f16)c[2 * u + 1][1], (f16)c[2 * u + 1][2], (f16)c[2 * u + 1][3]};
        };
        auto scores = [&](int tile) {  // tile TPW·pass + t, in slot t
            const int t = tile % TPW;
            f16x8 kf[4][2];
            read_k(t, kf);
            f32x4 c[4];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][0], qf[0], f32x4{}, 0, 0, 0);
                c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][1], qf[1], c[kb], 0, 0, 0);
            }
            if (key0 + kTileKV * (tile + 1) > nkv) {  // wave-uniform: mask keys past nkv
#pragma unroll
                for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (key0 + kTileKV * tile + 16 * kb + 4 * g + e >= nkv) c[kb][e] = -INFINITY;
            }
            if (tile == 0) {
                const float mx = xquad_max(max16(c));
                m_run = (mx < kEmptyMax) ? 0.f : mx;
                exp_pack(c, p[0], m_run);
            } else {
#pragma unroll
                for (int kb = 0; kb < 4; ++kb) sc[t][kb] = c[kb];
            }
        };
        // the pipeline: store item j, issue item j + NB, then the scores its store made possible;
        // V(t) for t >= 2 is stored just before its PV (its slot's K was read by then); pass 1's
        // K(t) goes into slot t once pass 0's PV(t) has read V(t)
#ifndef MHA_F32_NB
#define MHA_F32_NB 0  // fp32 tiles in flight per wave (A/B hook; 0 = per form)
#endif
        // 3 for the 2-tile form (1x4x512^2 5.00 vs 5.10 us), 2 for the 4-tile form (the third
        // buffer lands in AGPRs: 1024^2 7.45-7.51 vs 7.11; tools/f32_probe.py over MHA_F32_NB builds)
#ifndef MHA_D16_NB16
#define MHA_D16_NB16 3  // fp16 tiles in flight per wave in the staged A/B form
#endif
        constexpr int NB = !F32IN ? MHA_D16_NB16 : MHA_F32_NB > 0 ? MHA_F32_NB : (TPW == 2 ? 3 : 2);
        Tile buf[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) ld_tile(j, buf[j]);
        auto store = [&](int j) {  // item j into its slot, then the load NB items ahead
            st_tile(j, buf[j % NB]);
            if (j + NB < NI) ld_tile(j + NB, buf[j % NB]);
        };
#pragma unroll
        for (int ps = 0; ps < PASSES; ++ps) {
            const int b = 2 * TPW * ps, t0 = TPW * ps;
#pragma unroll
            for (int j = 0; j < TPW + 2; ++j) {  // K(0..TPW-1), V(0), V(1) of the pass
                store(b + j);
                if (j >= 1 && j - 1 < TPW) scores(t0 + j - 1);
            }
            // ONE rescale decision per pass (wave-uniform, rare): pass 0 against the first
            // tile's max (its P rescaled), later passes against the running max (O and l rescaled)
            {
                float mx = -INFINITY;
#pragma unroll
                for (int t = (ps == 0 ? 1 : 0); t < TPW; ++t) mx = fmaxf(mx, max16(sc[t]));
                const float ex = xquad_max(mx) - m_run;
                if (__builtin_amdgcn_ballot_w64(ex > kRescaleThr) != 0) {
                    const float d = fmaxf(ex, 0.f);
                    if (ps == 0) {
                        const f16 alpha = (f16)__builtin_amdgcn_exp2f(-d);
#pragma unroll
                        for (int u = 0; u < 2; ++u) p[0][u] *= alpha;
                    } else {
                        const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
                        for (int db = 0; db < 4; ++db) o[db] *= alpha;
                        l_acc *= alpha;
                    }
                    m_run += d;
                }
            }
            if (ps == 0) pv(0, true);
#pragma unroll
            for (int t = (ps == 0 ? 1 : 0); t < TPW; ++t) exp_pack(sc[t], p[t], m_run);
#pragma unroll
            for (int t = (ps == 0 ? 1 : 0); t < TPW; ++t) {
                if (t >= 2) store(b + TPW + t);
                pv(t, false);
            }
        }
    } else {
        // ---- loads, all up front (rows past nkv / nq read as zero through the descriptors) ----
        // DMA piece i = rows 8i..8i+7 of the wave's slice; lane L writes LDS chunk L&7 of row
        // 8i + L/8 and reads the source chunk that the image puts there.
        const unsigned lrow = (unsigned)(key0 + (lane >> 3)) * kHeadDim * 2;
        const unsigned k_lane[2] = {lrow + (((lane & 7) ^ ((lane >> 4) & 7)) << 4),
                                    lrow + (((lane & 7) ^ ((4 + (lane >> 4)) & 7)) << 4)};
        const unsigned v_lane_off = lrow + (((lane & 7) ^ (((lane >> 4) & 3) << 1)) << 4);
        // source piece i of the wave's key slice into region piece li (li = i except in pass 1)
        auto dma_piece = [&](__amdgpu_buffer_rsrc_t rs, unsigned voff, int i, int li) {
            // asm DMA in the multi-pass forms (no compiler drain before the transposing reads:
            // 1x4x1024x2048 7.28 vs 7.64 us); the one-pass forms measured neutral (1024^2 5.02 vs
            // 5.00, 768^2 4.48 vs 4.28) and keep the builtin
            if (MHA_DMA_ASM && PASSES > 1) {
                lds_dma16(lds_addr(smem + region + 1024 * li), voff, rs, 1024u * i);
            } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(smem + region + 1024 * li),
                                                         16, voff, 1024 * i, 0, 0);
            }
        };
        auto dma_k = [&](int t0, int t1) {
#pragma unroll
            for (int i = 8 * t0; i < 8 * t1; ++i) dma_piece(k_rs, k_lane[i & 1], i, i);
        };
        auto dma_k2 = [&](int t) {  // K of tile TPW + t into slot t (the swizzle repeats every 2 pieces)
#pragma unroll
            for (int i = 0; i < 8; ++i) dma_piece(k_rs, k_lane[i & 1], 8 * (TPW + t) + i, 8 * t + i);
        };
        auto dma_v = [&](int t, int slot) {  // V of tile t into `slot`
#pragma unroll
            for (int i = 0; i < 8; ++i) dma_piece(v_rs, v_lane_off, 8 * t + i, 8 * slot + i);
        };
        // K fragments of tile t (A operand of Sᵀ = K·Qᵀ): kf[kb][s] = K[64t+16kb+i16][32s+8g..+7]
        auto read_k = [&](int t, f16x8(&kf)[4][2]) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    kf[kb][s] = lds_read16(lds, region + k_off(kTileKV * t + 16 * kb + i16, 4 * s + g));
        };
        // Q (B operand of Sᵀ = K·Qᵀ): Q[q_row][32s+8g..+7], by inline-asm loads (outside the
        // compiler's wait bookkeeping, which would drain every DMA at their use)
        f16x8 qraw[2], qf[2];
#ifndef MHA_D16_K0_FIRST
#define MHA_D16_K0_FIRST 0  // 1: K(0)'s DMA ahead of the Q loads for every form (A/B hook)
#endif
        // K(0)'s DMA ahead of the Q loads (same wait counts) for the 2-tile form: 1x4x512^2 3.36-3.40
        // vs 3.42-3.52 us; the 4-tile form (the metric call) keeps Q first (4.97-5.04 vs 4.89-4.99)
        constexpr bool K0F = MHA_D16_K0_FIRST || (TPW == 2 && PASSES == 1);
#ifndef MHA_D16_PREFETCH
#define MHA_D16_PREFETCH 1  // 0: no L2 prefetch (A/B hook)
#endif
        // L2 prefetch of the rows requested late (mha_hd64_device.h). Measured at 1x4x1024^2
        // (tools/cold_probe.py, profiles/r02/prefetch_ab.txt): inputs from HBM 6.72 -> 5.7 us,
        // L2-resident inputs +0.02 us (4.65); at 768^2 / 1024x2048 -15 / -22 % cold, +2 % warm.
        L2Prefetch pf;
        if constexpr (MHA_D16_PREFETCH != 0)
            l2_prefetch<WAVE_KEYS, 2 * kTileKV>(pf, k_rs, v_rs, nkv, qtile,  // K(0), K(1) at entry
                                                prefetch_group(total_blocks, ca.qtiles), lane, wave == 0);
        if constexpr (K0F) dma_k(0, 1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"
                         : "=v"(qraw[s])
                         : "v"((unsigned)(q_row * kHeadDim + 32 * s + 8 * g) * 2), "s"(q_rs));
        dma_k(K0F ? 1 : 0, 2);
        wait_vmc<8>();  // Q and K(0) landed (younger: K(1)); the prefetch too
        asm volatile("" : "+v"(qraw[0]), "+v"(qraw[1])::"memory");
        l2_prefetch_done(pf);
        DSTAMP(1);
        dma_k(2, TPW);
        {
            const float sc = kScaleLog2;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const u32x4 in = __builtin_bit_cast(u32x4, qraw[s]);
                u32x4 outv;
#pragma unroll
                for (int w = 0; w < 4; ++w)
                    asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[1,0,0]\n\t"
                        "v_fma_mixhi_f16 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                        : "=&v"(outv[w])
                        : "v"(in[w]), "v"(sc));
                qf[s] = __builtin_bit_cast(f16x8, outv);
            }
        }
        const f16x8 ones = f16x8{1, 1, 1, 1, 1, 1, 1, 1};
        // V tr-read bases: lane 4qq+pp of group g reads row 4g+qq (+ tile/step/half constants),
        // dims 16db + 4pp..+3: chunk 2db + pp/2 at image position 2(db ^ sw) + pp/2
        const int qq = (lane & 15) >> 2, pp = lane & 3;
        const int sw = ((4 * g + qq) >> 1) & 3;
        unsigned vbase[4];
#pragma unroll
        for (int db = 0; db < 4; ++db)
            vbase[db] = region + (unsigned)(4 * g + qq) * 128 + ((2 * (db ^ sw) + (pp >> 1)) << 4) + 8 * (pp & 1);

        f16x8 p[TPW][2];   // P (fp16), B operand of step u of tile t
        f32x4 sc[TPW][4];  // raw scores of tiles 1..
        // Oᵀ += Vᵀ·Pᵀ for the tile in slot t; first: accumulators from an inline 0; refill: V's
        // fragments all in registers, then K of tile TPW + t into slot t, then the MFMAs
        auto pv = [&](int t, bool first, bool refill) {
            f16x8 va[2][4];
            auto read_v = [&](int u, int db) {
                const unsigned off = (unsigned)(t * kTileBytes + 128 * 32 * u);
                va[u][db] = cat8(tr_read(lds, vbase[db] + off), tr_read(lds, vbase[db] + off + 16 * 128));
            };
            if (refill) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int db = 0; db < 4; ++db) read_v(u, db);
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(va[0][0]), "+v"(va[0][1]), "+v"(va[0][2]), "+v"(va[0][3]), "+v"(va[1][0]),
                               "+v"(va[1][1]), "+v"(va[1][2]), "+v"(va[1][3])::"memory");
                dma_k2(t);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
#pragma unroll
                for (int db = 0; db < 4; ++db) {
                    if (!refill) read_v(u, db);
                    const bool z = first && u == 0;
                    o[db] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[u][db], p[t][u], z ? f32x4{} : o[db], 0, 0, 0);
                }
                l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ones, p[t][u], (first && u == 0) ? f32x4{} : l_acc, 0,
                                                               0, 0);
            }
        };
        auto exp_pack = [&](f32x4(&c)[4], f16x8(&pt)[2], float m) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int e = 0; e < 4; ++e) c[kb][e] = __builtin_amdgcn_exp2f(c[kb][e] - m);
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pt[u] = f16x8{(f16)c[2 * u][0],     (f16)c[2 * u][1],     (f16)c[2 * u][2],     (f16)c[2 * u][3],
                              (f16)c[2 * u + 1][0], (f16)c[2 * u + 1][1], (f16)c[2 * u + 1][2], (f16)c[2 * u + 1][3]};
        };

        // Phase 1, while V streams in: every tile's scores; the first tile's probabilities.
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            f16x8 kf[4][2];
            if (t > 0) wait_vmc<8 * (TPW - 1)>();  // K(t) landed: younger are K(t+1..), V(0..t-1)
            read_k(t, kf);
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[1][0]), "+v"(kf[1][1]), "+v"(kf[2][0]),
                           "+v"(kf[2][1]), "+v"(kf[3][0]), "+v"(kf[3][1])::"memory");
            dma_v(t, t);  // over slot t, whose K is in registers
            f32x4 c[4];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][0], qf[0], f32x4{}, 0, 0, 0);
                c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][1], qf[1], c[kb], 0, 0, 0);
            }
            if (key0 + kTileKV * (t + 1) > nkv) {  // wave-uniform: mask keys past nkv
#pragma unroll
                for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (key0 + kTileKV * t + 16 * kb + 4 * g + e >= nkv) c[kb][e] = -INFINITY;
            }
            if (t == 0) {
                const float mx = xquad_max(max16(c));
                m_run = (mx < kEmptyMax) ? 0.f : mx;  // a fully masked tile: m = 0
                exp_pack(c, p[0], m_run);
            } else {
#pragma unroll
                for (int kb = 0; kb < 4; ++kb) sc[t][kb] = c[kb];
            }
        }
        // ONE rescale decision for the later tiles (wave-uniform, rare): move the max by the
        // largest excess over kRescaleThr, rescaling the first tile's probabilities.
        {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 1; t < TPW; ++t) mx = fmaxf(mx, max16(sc[t]));
            const float ex = xquad_max(mx) - m_run;
            if (__builtin_amdgcn_ballot_w64(ex > kRescaleThr) != 0) {
                const float d = fmaxf(ex, 0.f);
                const f16 alpha = (f16)__builtin_amdgcn_exp2f(-d);
#pragma unroll
                for (int u = 0; u < 2; ++u) p[0][u] *= alpha;
                m_run += d;
            }
        }
        wait_vmc<8 * (TPW - 1)>();  // V(0) landed
        DSTAMP(3);
        pv(0, true, PASSES > 1);    // beside the later tiles' exponentials
#pragma unroll
        for (int t = 1; t < TPW; ++t) exp_pack(sc[t], p[t], m_run);
        DSTAMP(2);
        if constexpr (PASSES == 1) {
            wait_vmc<0>();
#pragma unroll
            for (int t = 1; t < TPW; ++t) pv(t, false, false);
        } else {
            // pass 1: tiles TPW + u through slot u, raw scores; ONE rescale decision for the pass
            // (O and the row sums rescaled), then exponentials against the running max and PV.
            // score2(u): K(TPW+u) landed (`younger` DMA groups after it), its fragments in registers,
            // V(TPW+u) into the slot, the MFMAs.
            auto score2 = [&](int u, int younger) {
                f16x8 kf[4][2];
                wait_groups(younger);
                read_k(u, kf);
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[1][0]), "+v"(kf[1][1]), "+v"(kf[2][0]),
                               "+v"(kf[2][1]), "+v"(kf[3][0]), "+v"(kf[3][1])::"memory");
                dma_v(TPW + u, u);
                f32x4 c[4];
#pragma unroll
                for (int kb = 0; kb < 4; ++kb) {
                    c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][0], qf[0], f32x4{}, 0, 0, 0);
                    c[kb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kb][1], qf[1], c[kb], 0, 0, 0);
                }
                if (key0 + kTileKV * (TPW + u + 1) > nkv) {  // wave-uniform: mask keys past nkv
#pragma unroll
                    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (key0 + kTileKV * (TPW + u) + 16 * kb + 4 * g + e >= nkv) c[kb][e] = -INFINITY;
                }
#pragma unroll
                for (int kb = 0; kb < 4; ++kb) sc[u][kb] = c[kb];
            };
            // pass 0's remaining PVs (each refilling its slot with a pass-1 K) interleaved with
            // pass 1's scores (mha_hd64_direct.hip's order): DMA issue order after pass 0's V is
            // K(TPW) at pv(0), then K(TPW+t) at pv(t) and V(TPW+t-1) at score2(t-1), V(2TPW-1) last
#pragma unroll
            for (int t = 1; t < TPW; ++t) {
                wait_groups(TPW - 2 + t);  // V(t): V(t+1..), K(TPW..TPW+t-1), V(TPW..TPW+t-2)
                pv(t, false, true);
                score2(t - 1, t == 1 ? 1 : 2);
            }
            score2(TPW - 1, 1);
            {
                float mx = -INFINITY;
#pragma unroll
                for (int t = 0; t < TPW; ++t) mx = fmaxf(mx, max16(sc[t]));
                const float ex = xquad_max(mx) - m_run;
                if (__builtin_amdgcn_ballot_w64(ex > kRescaleThr) != 0) {
                    const float d = fmaxf(ex, 0.f);
                    const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
                    for (int db = 0; db < 4; ++db) o[db] *= alpha;
                    l_acc *= alpha;
                    m_run += d;
                }
            }
#pragma unroll
            for (int t = 0; t < TPW; ++t) exp_pack(sc[t], p[t], m_run);
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                wait_groups(t == TPW - 1 ? 0 : 2 * TPW - 3 - 2 * t);  // V(TPW+t): the groups issued after it
                pv(t, false, false);
            }
        }
    }
    DSTAMP(4);

    // ---- epilogue: merge the 4 key slices through LDS ----
    float* ol = reinterpret_cast<float*>(smem + region);     // [16][OROW]
    float* mlb = reinterpret_cast<float*>(smem + KW * RS);  // [KW][16][2]
    {
        const float L_w = l_acc[0];
        const float m_w = (L_w > 0.f) ? m_run : -INFINITY;
        float* dst = ol + i16 * OROW + 4 * g;
#pragma unroll
        for (int db = 0; db < 4; ++db) *reinterpret_cast<f32x4*>(dst + 16 * db) = o[db];
        if (g == 0) *reinterpret_cast<float2*>(mlb + (wave * BLOCK_M + i16) * 2) = make_float2(m_w, L_w);
    }
    __syncthreads();
    DSTAMP(5);
#ifndef MHA_D16_EPI8
#define MHA_D16_EPI8 0  // 1: 128 threads merge (row, 8 dims) with 16-B stores (A/B hook)
#endif
    constexpr int EDPT = MHA_D16_EPI8 ? 8 : 4;            // dims per merging thread
    constexpr int EMERGE = BLOCK_M * kHeadDim / EDPT;     // merging threads
    if (EMERGE < 64 * KW && tid >= EMERGE) return;
    const int row = tid / (kHeadDim / EDPT), c = (tid % (kHeadDim / EDPT)) * EDPT;
    const int q = qtile * BLOCK_M + row;
    float2 ml[KW];
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        ml[k] = *reinterpret_cast<const float2*>(mlb + (k * BLOCK_M + row) * 2);
        M = fmaxf(M, ml[k].x);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const float w = (ml[k].x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml[k].x - M);
        L += w * ml[k].y;
        const float* src = reinterpret_cast<const float*>(smem + k * RS) + row * OROW + c;
        acc += w * *reinterpret_cast<const f32x4*>(src);
        if constexpr (EDPT == 8) acc1 += w * *reinterpret_cast<const f32x4*>(src + 4);
    }
    if (q < nq) {
        const __amdgpu_buffer_rsrc_t o_rs = make_rsrc(reinterpret_cast<TOut*>(ca.o) + (size_t)bh * nq * kHeadDim,
                                                      (unsigned)(nq * kHeadDim * sizeof(TOut)));
        const float inv = 1.f / L;
        store_dims<TOut, EDPT, MHA_ST_AUX>(o_rs, (unsigned)((q * kHeadDim + c) * sizeof(TOut)), acc * inv,
                                           acc1 * inv);
    }
#ifdef MHA_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DSTAMP(6);
#endif
}

template <typename TOut, int KW, int TPW, int PASSES = 1, bool F32IN = false>
hipError_t launch16_t(const FwdArgs& a, int grid, hipStream_t stream) {
    if (a.n_calls > 1)
        hipLaunchKernelGGL((mha_hd64_direct16_kernel<TOut, KW, TPW, true, PASSES, F32IN>), dim3(grid), dim3(64 * KW), 0,
                           stream, nullptr, nullptr, nullptr, nullptr, a.total_blocks, 0, 0, 0, a);
    else
        hipLaunchKernelGGL((mha_hd64_direct16_kernel<TOut, KW, TPW, false, PASSES, F32IN>), dim3(grid), dim3(64 * KW), 0,
                           stream, a.c[0].q, a.c[0].k, a.c[0].v, a.c[0].o, a.total_blocks, a.c[0].nq, a.c[0].nkv,
                           a.c[0].qtiles, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_direct16(const FwdArgs& a, int grid, int tiles_per_wave, bool out_f32, hipStream_t stream,
                           bool in_f32) {
    // tiles_per_wave counts 64-key tiles per wave of the 8-wave form (1: nkv <= 512, 2: <= 1024);
    // 4 waves take twice as many
    if (in_f32) {  // fp32 Q/K/V rounded in the kernel: the one-pass forms (the planner's choice)
        if (tiles_per_wave > 2)  // two-pass forms: diagnostic only (MHA_HD64_F32_INKERNEL=2)
            return out_f32 ? launch16_t<float, 4, 4, 2, true>(a, grid, stream)
                           : launch16_t<f16, 4, 4, 2, true>(a, grid, stream);
        switch (tiles_per_wave * 2 + (out_f32 ? 1 : 0)) {
            case 2: return launch16_t<f16, 4, 2, 1, true>(a, grid, stream);
            case 3: return launch16_t<float, 4, 2, 1, true>(a, grid, stream);
            case 4: return launch16_t<f16, 4, 4, 1, true>(a, grid, stream);
            case 5: return launch16_t<float, 4, 4, 1, true>(a, grid, stream);
            default: return hipErrorInvalidValue;
        }
    }
    if (tiles_per_wave > 2)  // nkv in (1024, 2048]: 4 waves x two passes of 4 tiles
        return out_f32 ? launch16_t<float, 4, 4, 2>(a, grid, stream) : launch16_t<f16, 4, 4, 2>(a, grid, stream);
    switch (tiles_per_wave * 2 + (out_f32 ? 1 : 0)) {
        case 2: return launch16_t<f16, 4, 2>(a, grid, stream);
        case 3: return launch16_t<float, 4, 2>(a, grid, stream);
#if MHA_D16_WAVES == 8
        case 4: return launch16_t<f16, 8, 2>(a, grid, stream);
        case 5: return launch16_t<float, 8, 2>(a, grid, stream);
#else
        case 4: return launch16_t<f16, 4, 4>(a, grid, stream);
        case 5: return launch16_t<float, 4, 4>(a, grid, stream);
#endif
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mha_hd64
