// mha_hd64_direct.hip — single-pass FlashAttention forward, head_dim = 64, for gfx950 (MI355X).
//
// The same operator as mha_hd64_kernels.hip (O = softmax(Q·Kᵀ·0.125)·V per (batch, head); the
// reference's attention_headdim_64_fp16in_fp16out.cu:253-733 / …fp16in_fp32out.cu:253-703), laid
// out for launches that cannot fill the chip with query blocks alone — the plugin's single
// 1x4x1024x1024 call is 128 blocks of 32 rows.
//
// The LDS-ring kernel fills 256 CUs there by splitting each query block's keys over two
// workgroups and merging the two partials through L2 (publish, ticket, read back: ≈ 1.7 µs of
// dependent round trips per call). This kernel gives ONE workgroup all the keys of its 32-row
// query block instead: 8 waves, wave w owns keys [64·TPW·w, 64·TPW·(w+1)), so no other workgroup
// ever needs its partial and the merge is an LDS exchange between the 8 waves.
//  * Nothing is shared between waves until the epilogue, so nothing is staged for sharing: every
//    wave loads its own K straight into MFMA A-operand registers (K rows on lanes), and its own V
//    through a wave-private LDS image (the transposing ds_read_b64_tr_b16 needs V in LDS), with no
//    barrier before the epilogue. All loads are issued up front (Q, K tile by tile, then V), so
//    QKᵀ of the first tile starts as soon as its K lands while the rest streams in.
//  * Per tile (64 keys): Sᵀ = K·Qᵀ on v_mfma_f32_32x32x16_f16 with the running max and the tail
//    mask folded into a bias k-step, one v_exp_f32 per probability, P packed to fp16 as the B
//    operand of Oᵀ = Vᵀ·Pᵀ, row sums on a 16x16x32 MFMA, lazy rescale (threshold 8 in log2
//    units) — the arithmetic of the ring kernel's step, so both kernels agree to rounding.
//  * Epilogue: each wave stages Oᵀ (fp32, at its own max) and (m, l) in its own LDS region; one
//    barrier; 512 threads merge (row, 4 dims) over the 8 waves and store O.
// The planner (plan_group) picks this kernel for fp16 inputs when nkv <= 1024 and the launch has
// at most 256 such workgroups (one residency round); everything else runs the ring kernel.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

// Diagnostic timestamps (-DMHA_STAMPS builds, tools/dstamps.py): wave 0's s_memtime at phase
// boundaries, without draining memory (the waits of the phase boundaries themselves are kept).
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


namespace mha_hd64 {
namespace {

// s_waitcnt vmcnt(N) for a compile-time N (multiples of 8 up to 24)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N % 8 == 0 && N <= 40, "vmcnt");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
}
// s_waitcnt vmcnt(8 * groups) for a value known after unrolling
__device__ __forceinline__ void wait_vm_groups(int groups) {
    switch (groups) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<8>(); break;
        case 2: wait_vm<16>(); break;
        case 3: wait_vm<24>(); break;
        case 4: wait_vm<32>(); break;
        default: wait_vm<40>(); break;
    }
}

#ifndef MHA_D2P_EARLY
#define MHA_D2P_EARLY 1  // two-pass form: second-pass scores between the first pass's PVs (0: after them)
#endif

// KW waves (key slices) per workgroup x TPW 64-key tiles per wave. (16 waves x 1 tile, four per
// SIMD, measured 7.7 us against 6.3 us for 8 x 2 at 1x4x1024x1024.)
// PASSES = 2 (nkv in (1024, 2048], 4 waves): each wave's 2·TPW tiles go through its TPW slots twice;
// pass 1's K(TPW + t) is issued into slot t as soon as pass 0's PV has V(t)'s fragments in
// registers, so the second pass's loads queue behind the first pass's without a gap.
template <typename TOut, int KW, int TPW, bool MULTI, int PASSES = 1>
__global__ __launch_bounds__(64 * KW, 1) void mha_hd64_direct_kernel(FwdArgs a) {
    static_assert(PASSES == 1 || (PASSES == 2 && (TPW * KW == 16 || (TPW == 2 && KW == 4))) ||
                      (PASSES == 4 && TPW == 2 && KW == 4),
                  "passes x tiles: 4 waves x 2 x 4, 8 x 2 x 2, or 4 x {2, 4} x 2 (65 KiB LDS: two workgroups per CU)");
    constexpr int NT = 64 * KW;
    constexpr int BLOCK_M = 32;                         // query rows per workgroup
    constexpr int WAVE_KEYS = kTileKV * TPW * PASSES;   // keys per wave
    constexpr int OROW = 68;                            // epilogue fp32 row pitch (64 dims + 4 pad)
    constexpr int EPI_WAVE = BLOCK_M * OROW * 4;        // one wave's staged Oᵀ
    // Wave-private region: the wave's V tiles, later its staged Oᵀ (8704 = 68 x 128 B keeps the
    // bank phase of every region the same as a region at 0).
    constexpr int RS = TPW * kTileBytes > EPI_WAVE ? TPW * kTileBytes : EPI_WAVE;
    constexpr int LDS_BYTES = KW * RS + KW * BLOCK_M * 2 * 4 + 16;  // + wave 0's non-finite-query mask
    static_assert(RS % 128 == 0 && LDS_BYTES <= 160 * 1024, "LDS layout");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    lds_char* const lds = (lds_char*)smem;

    DSTAMP(0);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave
    // XCD-aware order (as the ring kernel): consecutive j share an XCD, so the query blocks of
    // one (batch, head) read its K/V through one L2.
    int qtile, bh, j;
    {
        const int T = a.total_blocks, L = blockIdx.x;
        const int q8 = T >> 3, r8 = T & 7, xcd = L & 7;
        j = xcd * q8 + min(xcd, r8) + (L >> 3);
    }
    int ci = 0;
    if constexpr (MULTI) {
#pragma unroll
        for (int i = 1; i < kMaxCalls; ++i) ci += (int)((i < a.n_calls) & (j >= a.c[i].block_begin));
    }
    const CallArgs ca = MULTI ? pick_call(a, ci) : a.c[0];
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
    const int q_row = qtile * BLOCK_M + r;
    const int key0 = wave * WAVE_KEYS;
    // tiles of this wave holding at least one key (wave-uniform)
    const int n_t = max(0, min(TPW * PASSES, (nkv - key0 + kTileKV - 1) / kTileKV));
    const unsigned region = (unsigned)wave * RS;

    f32x16 o0, o1;  // Oᵀ: dims 0..31 / 32..63, query on the lane
    f32x4 l_acc;
    float m_run = 0.f;
    unsigned qbad = 0;  // queries of the block with a non-finite Q (q_nonfinite_fix)

    if (n_t == 0) {  // a wave wholly past nkv contributes nothing (m = -inf in the merge)
        o0 = o1 = f32x16{};
        l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
        // ---- loads, all up front (unconditional: rows past nkv read as zero) ----
        // K reaches LDS by LDS-DMA in whole 128-B rows (1 KiB per instruction: rows 8i..8i+7),
        // swizzled on the source side (the DMA writes lane-linear): LDS position p of row `row`
        // receives the 16-B chunk p ^ swz(row) (the k_off / v_off images).
        // Per-lane byte offsets: row 8i + lane/8 of the wave's slice, chunk swizzled; piece i adds
        // i KiB (a scalar offset), and the swizzles repeat every two pieces (K) or never vary (V).
        const unsigned lrow = (unsigned)(key0 + (lane >> 3)) * kHeadDim * 2;
        const unsigned k_lane[2] = {lrow + (((lane & 7) ^ ((lane >> 4) & 7)) << 4),
                                    lrow + (((lane & 7) ^ ((4 + (lane >> 4)) & 7)) << 4)};
        const unsigned v_lane_off = lrow + (((lane & 7) ^ (((lane >> 4) & 1) << 2)) << 4);
        // piece i of the wave's key slice (source) into piece li of its region (li = i except in
        // the second pass, whose tile TPW + t goes into slot t)
        auto dma_piece = [&](__amdgpu_buffer_rsrc_t rs, unsigned voff, int i, int li) {
            if (MHA_ABL & ABL_NO_GLOAD) return;
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
        auto dma_k = [&](int t0, int t1) {  // K of tiles [t0, t1) into their slots
#pragma unroll
            for (int i = 8 * t0; i < 8 * t1; ++i) dma_piece(k_rs, k_lane[i & 1], i, i);
        };
        // K of tile TPW + t (second pass) into slot t; the swizzle repeats every 2 pieces
        auto dma_kt = [&](int tile, int slot) {
#pragma unroll
            for (int i = 0; i < 8; ++i) dma_piece(k_rs, k_lane[i & 1], 8 * tile + i, 8 * slot + i);
        };
        auto dma_tile = [&](__amdgpu_buffer_rsrc_t rs, int t, int slot) {  // V of tile t into `slot`
#pragma unroll
            for (int i = 0; i < 8; ++i) dma_piece(rs, v_lane_off, 8 * t + i, 8 * slot + i);
        };
        // K fragments of tile t (A operand of Sᵀ = K·Qᵀ): kf[2s] = K[64t+r][16s+8hh..+7], kf[2s+1] = rows +32
        auto read_k = [&](int t, f16x8(&kf)[8]) {  // t: the slot
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2)
                    kf[2 * s + h2] = lds_read16(lds, region + k_off(kTileKV * t + 32 * h2 + r, 2 * s + hh));
        };
        f16x8 qf[4];  // Q fragments (B operand of Sᵀ = K·Qᵀ), scaled by 0.125·log2(e) in fp16
        // Q by plain loads in inline asm (unseen by the compiler's wait bookkeeping: a plain load's
        // use behind an LDS-DMA would make it drain every DMA), K then V by DMA, tile by tile
        // through the wave's two 8 KiB slots: tile t's V is issued into slot t as soon as K(t)'s
        // fragments are in registers, so K(1) lands under QKᵀ(0) and V under all of the scores.
        f16x8 qraw[4];
        // K(0) and K(1) first: the first tile's K is not queued behind the whole wave's K
        constexpr int KFIRST = TPW < 2 ? TPW : 2;
#ifndef MHA_D_PREFETCH
#define MHA_D_PREFETCH 1  // 0: no L2 prefetch (A/B hook)
#endif
        // L2 prefetch of the rows requested late (mha_hd64_device.h; profiles/r02/prefetch_ab.txt)
        L2Prefetch pf;
        if constexpr (MHA_D_PREFETCH != 0 && !(MHA_ABL & ABL_NO_GLOAD))
            l2_prefetch<WAVE_KEYS, kTileKV * KFIRST>(pf, k_rs, v_rs, nkv, qtile,
                                                     prefetch_group(a.total_blocks, ca.qtiles), lane, wave == 0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (MHA_ABL & ABL_NO_GLOAD) qraw[s] = f16x8{} + (f16)(lane * 0.01f);
            else asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"
                              : "=v"(qraw[s])
                              : "v"((unsigned)(q_row * kHeadDim + 16 * s + 8 * hh) * 2), "s"(q_rs));
        }
        dma_k(0, KFIRST);
        // Q and K(0) have landed (issue order: Q, K(0), K(1), 8 pieces per tile)
        wait_vm<8 * (KFIRST - 1)>();
        asm volatile("" : "+v"(qraw[0]), "+v"(qraw[1]), "+v"(qraw[2]), "+v"(qraw[3])::"memory");
        l2_prefetch_done(pf);  // older than Q
        DSTAMP(1);
        // the rest of K; every later K(t) wait sees K(t+1..) and V(0..t-1) younger: vmcnt(8*(TPW-1))
        dma_k(KFIRST, TPW);
        // q * 0.125·log2(e) in fp32, rounded to fp16: one v_fma_mix{lo,hi}_f16 per value (the compiler
        // emits convert + multiply + pack, twice the vector instructions)
        {
            const float sc = kScaleLog2;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
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
        qbad = q_nonfinite_fix(qf);  // non-finite query rows: zeroed here, NaN rows at the store

        // Row sums on the matrix pipe and the bias k-step: as the ring kernel (mha_hd64_kernels.hip).
        const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
        const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};
        const f16 one_h = hh == 0 ? (f16)1.f : (f16)0.f;
        f16x8 b_bias = f16x8{0, 0, one_h, 0, 0, 0, 0, 0};  // m_run = 0
        auto set_bias = [&]() {
            const f16 hi = (f16)(-m_run);
            const f16 lo = (f16)(-m_run - (float)hi);
            b_bias = hh == 0 ? f16x8{hi, lo, (f16)1.f, 0, 0, 0, 0, 0} : f16x8{0, 0, 0, 0, 0, 0, 0, 0};
        };
        auto a_bias_of = [&](int t, int half) -> f16x8 {
            const int key = key0 + kTileKV * t + 32 * half + r;
            const f16 mk = (hh == 0 && key >= nkv) ? (f16)kMaskBias : (f16)0.f;
            return f16x8{one_h, one_h, mk, 0, 0, 0, 0, 0};
        };
        // V tr-read lane addressing (see the ring kernel): rows 4hh+qq (+const), swizzled halves.
        const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
        const int vb = (qq >> 1) & 1;
        const unsigned v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);

        // Phase 1, while V is still in flight: the probabilities of every tile of the wave. Every
        // tile runs, even one wholly past nkv (its keys are masked: P = 0 and the max does not
        // move), so no branch separates the up-front loads from their uses.
        f16x8 p[TPW][2][2];  // P (fp16) as the B operand: p[t][half][k-step]
        f32x16 sc[TPW][2];   // scores of tiles 1.. (log2 units, against the first tile's max)
        // Oᵀ += Vᵀ·Pᵀ for tile t and the row sums, once V(t) has landed (V(t+1..) may be in flight)
        // Oᵀ += Vᵀ·Pᵀ for the tile in slot t (probabilities pt) and the row sums, once its V has
        // landed: `younger` = DMA groups of 8 issued after it (-1: already waited). first: the
        // accumulators start from an inline 0. refill: K of tile TPW + t is issued into slot t as
        // soon as V's fragments are in registers (the two-pass form's first pass).
        auto pv = [&](int t, const f16x8(&pt)[2][2], int younger, bool first, int refill_tile) {
            const bool refill = refill_tile >= 0;
            if (younger >= 0) wait_vm_groups(younger);
            if (first) DSTAMP(3);
            const unsigned va0 = region + t * kTileBytes + v_lane + 64 * vb;
            const unsigned va1 = region + t * kTileBytes + v_lane + 64 * (1 - vb);
            f16x8 vfa[2][2], vfb[2][2];
            auto read_v = [&](int jj, int ss) {
                const unsigned rowc = 128 * (32 * jj + 16 * ss);
                vfa[jj][ss] = cat8(tr_read(lds, va0 + rowc), tr_read(lds, va0 + rowc + 8 * 128));
                vfb[jj][ss] = cat8(tr_read(lds, va1 + rowc), tr_read(lds, va1 + rowc + 8 * 128));
            };
            if (refill) {  // every fragment in registers before the slot is refilled
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss) read_v(jj, ss);
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(vfa[0][0]), "+v"(vfa[0][1]), "+v"(vfa[1][0]), "+v"(vfa[1][1]), "+v"(vfb[0][0]),
                               "+v"(vfb[0][1]), "+v"(vfb[1][0]), "+v"(vfb[1][1])::"memory");
                dma_kt(refill_tile, t);
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (!refill) read_v(jj, ss);
                    if (MHA_ABL & ABL_NO_PV) {
                        keep_live(vfa[jj][ss]);
                        keep_live(vfb[jj][ss]);
                        keep_live(pt[jj][ss]);
                        if (first && jj == 0 && ss == 0) {
                            o0 = o1 = f32x16{};
                            l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
                        }
                        continue;
                    }
                    const bool z = first && jj == 0 && ss == 0;  // accumulators start at inline 0
                    o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], pt[jj][ss], z ? f32x16{} : o0, 0, 0, 0);
                    o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], pt[jj][ss], z ? f32x16{} : o1, 0, 0, 0);
                    l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, pt[jj][ss], z ? f32x4{} : l_acc, 0, 0, 0);
                }
        };
        auto exp_pack = [&](f32x16 c0, f32x16 c1, f16x8(&pt)[2][2]) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                if (MHA_ABL & ABL_NO_EXP) continue;
                c0[e] = __builtin_amdgcn_exp2f(c0[e]);
                c1[e] = __builtin_amdgcn_exp2f(c1[e]);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                pt[0][0][e] = (f16)c0[e];
                pt[0][1][e] = (f16)c0[8 + e];
                pt[1][0][e] = (f16)c1[e];
                pt[1][1][e] = (f16)c1[8 + e];
            }
        };
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            f16x8 kf[8];
            // K(t) landed: younger are K(t+1..) and V(0..t-1), 8 pieces each
            if (t > 0) wait_vm<8 * (TPW - 1)>();
            read_k(t, kf);
            // K(t)'s fragments are in registers before V(t)'s DMA overwrites slot t
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]), "+v"(kf[4]),
                         "+v"(kf[5]), "+v"(kf[6]), "+v"(kf[7])::"memory");
            dma_tile(v_rs, t, t);
            // Sᵀ = K·Qᵀ - m, two 32-key halves. The bias k-step (-m and the tail mask) runs first,
            // except on a full first tile: there it runs last, once the tile's max is known, so the
            // scores need no subtraction (an MFMA instead of 32 VALU ops).
            const bool partial = key0 + kTileKV * (t + 1) > nkv;
            const bool bias_last = t == 0 && !partial;  // wave-uniform
            const f16x8 a_plain = f16x8{one_h, one_h, 0, 0, 0, 0, 0, 0};
            const f16x8 ab0 = partial ? a_bias_of(t, 0) : a_plain;
            const f16x8 ab1 = partial ? a_bias_of(t, 1) : a_plain;
            const f32x16 zero = {};
            f32x16 c0, c1;
            // (two straight-line chains: each starts its accumulators from an inline 0)
            auto chain = [&](auto bias_first_c) {
                constexpr bool BF = decltype(bias_first_c)::value;
                if constexpr (BF) {
                    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab0, b_bias, zero, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab1, b_bias, zero, 0, 0, 0);
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if (MHA_ABL & ABL_NO_QK) {
                        keep_live(kf[2 * s]);
                        keep_live(kf[2 * s + 1]);
                        if (!BF && s == 0) c0 = c1 = zero;
                        continue;
                    }
                    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s], qf[s], (!BF && s == 0) ? zero : c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + 1], qf[s], (!BF && s == 0) ? zero : c1, 0, 0,
                                                                0);
                }
            };
            if (bias_last) chain(std::false_type{});
            else chain(std::true_type{});
            if (t == 0) {
                // the first tile sets the running max (a fully masked tile: m = 0)
                const float mx = xhalf_max(tree_max(c0, c1));
                const float d = (mx < kEmptyMax) ? 0.f : mx;
                m_run += d;
                set_bias();
                if (bias_last) {
                    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_plain, b_bias, c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_plain, b_bias, c1, 0, 0, 0);
                } else {
                    c0 -= d;
                    c1 -= d;
                }
                exp_pack(c0, c1, p[0]);
            } else {
                sc[t][0] = c0;
                sc[t][1] = c1;
            }
        }
        // Later tiles' scores were taken against the first tile's max: ONE decision for all of them
        // (wave-uniform, rare) moves the max by the largest excess over kRescaleThr, rescaling the
        // first tile's probabilities and the later scores; then their exponentials. No branch sits
        // between the tiles, so their MFMAs interleave with the first tile's exponentials.
        if constexpr (TPW > 1) {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 1; t < TPW; ++t) mx = fmaxf(mx, tree_max(sc[t][0], sc[t][1]));
            mx = xhalf_max(mx);
            if (__builtin_amdgcn_ballot_w64(mx > kRescaleThr) != 0) {
                const float d = fmaxf(mx, 0.f);
                const f16 alpha = (f16)__builtin_amdgcn_exp2f(-d);
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss) p[0][h2][ss] *= alpha;
#pragma unroll
                for (int t = 1; t < TPW; ++t) {
                    sc[t][0] -= d;
                    sc[t][1] -= d;
                }
                m_run += d;
            }
            // tile 0's PV on the matrix pipe beside the later tiles' exponentials (one block)
            pv(0, p[0], TPW - 1, true, PASSES > 1 ? TPW : -1);
#pragma unroll
            for (int t = 1; t < TPW; ++t) exp_pack(sc[t][0], sc[t][1], p[t]);
        }
        DSTAMP(2);
        if constexpr (PASSES == 1) {
            // Phase 2: the remaining tiles' Oᵀ += Vᵀ·Pᵀ (tile 0's ran beside the exponentials). Every
            // V has long landed by now: one wait, so the compiler may hoist later fragment reads.
            if constexpr (TPW > 1) wait_vm<0>();
#pragma unroll
            for (int t = (TPW > 1 ? 1 : 0); t < TPW; ++t) pv(t, p[t], TPW > 1 ? -1 : 0, TPW == 1, -1);
        } else {
            // Later passes: tiles ps·TPW + u through slot u, scored against the running max (bias
            // k-step first), ONE rescale decision per pass (rescaling O and the row sums),
            // exponentials, then PV as each V lands, each PV refilling its slot with the next pass's K.
            constexpr bool EARLY2 = PASSES == 2 && MHA_D2P_EARLY;
            set_bias();
            // scores of tile `tile` in slot u: its K landed (`younger` DMA groups after it), fragments
            // in registers, its V into the slot, then the MFMAs
            auto score2 = [&](int tile, int u, int younger) {
                f16x8 kf[8];
                wait_vm_groups(younger);
                read_k(u, kf);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]), "+v"(kf[4]),
                             "+v"(kf[5]), "+v"(kf[6]), "+v"(kf[7])::"memory");
                dma_tile(v_rs, tile, u);
                const bool partial = key0 + kTileKV * (tile + 1) > nkv;  // wave-uniform
                const f16x8 a_plain = f16x8{one_h, one_h, 0, 0, 0, 0, 0, 0};
                const f16x8 ab0 = partial ? a_bias_of(tile, 0) : a_plain;
                const f16x8 ab1 = partial ? a_bias_of(tile, 1) : a_plain;
                f32x16 c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab0, b_bias, f32x16{}, 0, 0, 0);
                f32x16 c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab1, b_bias, f32x16{}, 0, 0, 0);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s], qf[s], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + 1], qf[s], c1, 0, 0, 0);
                }
                sc[u][0] = c0;
                sc[u][1] = c1;
            };
            if constexpr (EARLY2) {
                // DMA issue order after the first pass's V: K(TPW) at pv(0); then for t = 1..TPW-1
                // K(TPW+t) at pv(t) and V(TPW+t-1) at score2(t-1); V(2TPW-1) last. The first pass's
                // PVs interleave with the second pass's scores, so each second-pass V is issued one
                // PV after its K.
#pragma unroll
                for (int t = 1; t < TPW; ++t) {
                    pv(t, p[t], TPW - 2 + t, false, TPW + t);  // V(t): V(t+1..), K(TPW..TPW+t-1), V(TPW..TPW+t-2)
                    score2(TPW + t - 1, t - 1, t == 1 ? 1 : 2);  // K(TPW+t-1): K(TPW+t) (+ V(TPW+t-2), t > 1)
                }
                DSTAMP(7);
                score2(2 * TPW - 1, TPW - 1, 1);  // K(2TPW-1): V(2TPW-2)
            } else {
                // sequential order: every wait has TPW - 1 groups younger than its target (the
                // pass's later V and the next pass's earlier K, or its later K and earlier V)
#pragma unroll
                for (int t = 1; t < TPW; ++t) pv(t, p[t], TPW - 1, false, TPW + t);
                DSTAMP(7);
#pragma unroll
                for (int u = 0; u < TPW; ++u) score2(TPW + u, u, TPW - 1);
            }
#pragma unroll
            for (int ps = 1; ps < PASSES; ++ps) {
                if (ps > 1) {
                    set_bias();
#pragma unroll
                    for (int u = 0; u < TPW; ++u) score2(ps * TPW + u, u, TPW - 1);
                }
                {
                    float mx = -INFINITY;
#pragma unroll
                    for (int t = 0; t < TPW; ++t) mx = fmaxf(mx, tree_max(sc[t][0], sc[t][1]));
                    mx = xhalf_max(mx);
                    if (__builtin_amdgcn_ballot_w64(mx > kRescaleThr) != 0) {
                        const float d = fmaxf(mx, 0.f);
                        const float alpha = __builtin_amdgcn_exp2f(-d);
                        o0 *= alpha;
                        o1 *= alpha;
                        l_acc *= alpha;
#pragma unroll
                        for (int t = 0; t < TPW; ++t) {
                            sc[t][0] -= d;
                            sc[t][1] -= d;
                        }
                        m_run += d;
                    }
                }
#pragma unroll
                for (int t = 0; t < TPW; ++t) exp_pack(sc[t][0], sc[t][1], p[t]);
                const bool last = ps == PASSES - 1;
                // the last pass's V(u) has 2TPW-3-2u younger groups in the interleaved order (none
                // for the last tile), TPW-1-u in the sequential one; earlier passes refill
#pragma unroll
                for (int t = 0; t < TPW; ++t)
                    pv(t, p[t],
                       !last ? TPW - 1 : (EARLY2 ? (t == TPW - 1 ? 0 : 2 * TPW - 3 - 2 * t) : TPW - 1 - t), false,
                       last ? -1 : (ps + 1) * TPW + t);
            }
        }
    }

    DSTAMP(4);
    // ---- epilogue: merge the 8 key slices through LDS ----
    // The wave's V region is its own, so its staged Oᵀ overwrites only what it has read itself.
    float* ol = reinterpret_cast<float*>(smem + region);      // [32][OROW]
    float* mlb = reinterpret_cast<float*>(smem + KW * RS);   // [KW][32][2]
    {
        const float L_w = l_acc[0];
        const float m_w = (L_w > 0.f) ? m_run : -INFINITY;
        float* dst = ol + r * OROW;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d = 8 * g4 + 4 * hh;
            *reinterpret_cast<f32x4*>(dst + d) = f32x4{o0[4 * g4], o0[4 * g4 + 1], o0[4 * g4 + 2], o0[4 * g4 + 3]};
            *reinterpret_cast<f32x4*>(dst + 32 + d) =
                f32x4{o1[4 * g4], o1[4 * g4 + 1], o1[4 * g4 + 2], o1[4 * g4 + 3]};
        }
        if (hh == 0) *reinterpret_cast<float2*>(mlb + (wave * BLOCK_M + r) * 2) = make_float2(m_w, L_w);
        // wave 0 always holds keys, so its mask is the block's (a keyless wave loads no Q)
        if (wave == 0 && lane == 0) *reinterpret_cast<unsigned*>(mlb + KW * BLOCK_M * 2) = qbad;
    }
    __syncthreads();
    DSTAMP(5);
    // thread -> (row, DPT dims): 32 rows x 64/DPT chunks, one item per thread (DPT = 8 at 4 waves:
    // one 16-B fp16 store; DPT = 4 at 8 waves)
    constexpr int DPT = 32 * kHeadDim / NT;
    static_assert(DPT == 4 || DPT == 8, "epilogue items");
    const int row = tid / (kHeadDim / DPT), c = (tid % (kHeadDim / DPT)) * DPT;
    const int q = qtile * BLOCK_M + row;
    float2 ml[KW];
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        ml[k] = *reinterpret_cast<const float2*>(mlb + (k * BLOCK_M + row) * 2);
        M = fmaxf(M, ml[k].x);
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const float w = (ml[k].x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml[k].x - M);
        L += w * ml[k].y;
        const float* src = reinterpret_cast<const float*>(smem + k * RS) + row * OROW + c;
        acc0 += w * *reinterpret_cast<const f32x4*>(src);
        if constexpr (DPT == 8) acc1 += w * *reinterpret_cast<const f32x4*>(src + 4);
    }
    if (q < nq && !(MHA_ABL & ABL_NO_STORE)) {
        const __amdgpu_buffer_rsrc_t o_rs = make_rsrc(reinterpret_cast<TOut*>(ca.o) + (size_t)bh * nq * kHeadDim,
                                                      (unsigned)(nq * kHeadDim * sizeof(TOut)));
        const float inv = inv_or_nan(L, *reinterpret_cast<const unsigned*>(mlb + KW * BLOCK_M * 2), row);
        store_dims<TOut, DPT, MHA_ST_AUX>(o_rs, (unsigned)((q * kHeadDim + c) * sizeof(TOut)), acc0 * inv, acc1 * inv);
    }
#ifdef MHA_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    DSTAMP(6);
#endif
}

template <typename TOut, int KW, int TPW, int PASSES = 1>
hipError_t launch_direct_t(const FwdArgs& a, int grid, hipStream_t stream) {
    if (a.n_calls > 1)
        hipLaunchKernelGGL((mha_hd64_direct_kernel<TOut, KW, TPW, true, PASSES>), dim3(grid), dim3(64 * KW), 0, stream, a);
    else
        hipLaunchKernelGGL((mha_hd64_direct_kernel<TOut, KW, TPW, false, PASSES>), dim3(grid), dim3(64 * KW), 0, stream,
                           a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_direct(const FwdArgs& a, int grid, int tiles_per_wave, bool out_f32, hipStream_t stream) {
    // 4 waves x twice the tiles (one wave per SIMD): 6.02 vs 6.16 us at 1x4x1024^2, 4.33 vs 4.95 at
    // 512^2 against 8 waves; MHA_HD64_DIRECT_WAVES=8 selects the 8-wave form (comparison hook)
    static const bool four = [] {
        const char* e = std::getenv("MHA_HD64_DIRECT_WAVES");
        return !(e && e[0] == '8');
    }();
    // nkv in (1024, 2048] (tiles_per_wave 3, 4): two passes, 4 waves x 2 x 4 tiles (or 8 x 2 x 2)
    // nkv in (512, 1024] on more than one round of 256 workgroups: 4 waves x two passes of 2 tiles
    // through 2 slots per wave (65 KiB LDS), so two workgroups share a CU and one's load latency
    // hides behind the other's work (MHA_HD64_DIRECT_SHARED=0: the one-pass form, one per CU)
    static const bool shared = [] {
        const char* e = std::getenv("MHA_HD64_DIRECT_SHARED");
        return !(e && e[0] == '0');
    }();
    // (a concurrency hint >= 3 takes the two-per-CU form at any grid: each call then leaves room for
    // other streams' calls on the same CUs)
    const bool many = grid > 256 || concurrency_hint() >= 3;
    if (tiles_per_wave == 2 && many && four && shared)
        return out_f32 ? launch_direct_t<float, 4, 2, 2>(a, grid, stream) : launch_direct_t<f16, 4, 2, 2>(a, grid, stream);
    if (tiles_per_wave > 2 && many && four && shared)  // nkv in (1024, 2048], the same: 4 passes of 2
        return out_f32 ? launch_direct_t<float, 4, 2, 4>(a, grid, stream) : launch_direct_t<f16, 4, 2, 4>(a, grid, stream);
    if (tiles_per_wave > 2) {
        if (four)
            return out_f32 ? launch_direct_t<float, 4, 4, 2>(a, grid, stream)
                           : launch_direct_t<f16, 4, 4, 2>(a, grid, stream);
        return out_f32 ? launch_direct_t<float, 8, 2, 2>(a, grid, stream) : launch_direct_t<f16, 8, 2, 2>(a, grid, stream);
    }
    switch ((four ? 100 : 0) + tiles_per_wave * 2 + (out_f32 ? 1 : 0)) {
        case 2: return launch_direct_t<f16, 8, 1>(a, grid, stream);
        case 3: return launch_direct_t<float, 8, 1>(a, grid, stream);
        case 4: return launch_direct_t<f16, 8, 2>(a, grid, stream);
        case 5: return launch_direct_t<float, 8, 2>(a, grid, stream);
        case 102: return launch_direct_t<f16, 4, 2>(a, grid, stream);
        case 103: return launch_direct_t<float, 4, 2>(a, grid, stream);
        case 104: return launch_direct_t<f16, 4, 4>(a, grid, stream);
        case 105: return launch_direct_t<float, 4, 4>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mha_hd64
