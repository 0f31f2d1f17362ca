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
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

namespace mha_hd64 {
namespace {


// ----------------------------------------------------------------------------------------
// Main kernel. Grid: x = query blocks of 32*QW rows, y = batch*heads, z = KV splits.
//
// Software pipeline per wave (tile t = this wave's 64 keys of super-tile t):
//   phase A:  QKᵀ MFMAs of tile t+1            ‖ exp / row-sum / f16-pack of tile t (VALU)
//   phase B:  PV MFMAs of tile t               ‖ tail mask + row max of tile t+1 (VALU)
// so the matrix pipe and the vector pipe of a SIMD work on independent data. LDS is a
// 3-stage ring of super-tiles: iteration t reads V(t) and K(t+1) and fills stage t+2
// (loaded into registers at the start of the iteration, written after phase B), one
// barrier per iteration.
// ----------------------------------------------------------------------------------------
// MULTI = false: a launch of one call (plugin enqueue, L0 launchers) reads only c[0], so the
// prologue's kernarg loads issue in one scalar round; MULTI = true: grouped launches.
// RB = 32-row query blocks per wave: RB = 2 shares every K/V fragment read between two
// query blocks (half the LDS read traffic per FLOP), at twice the registers per wave.
template <typename TIn, typename TOut, int QW, int KW, int RB, bool MULTI>
__global__ __launch_bounds__(64 * QW * KW, 1) void mha_hd64_fwd_kernel(FwdArgs a) {
    constexpr int NT = 64 * QW * KW;                // threads
    constexpr int BLOCK_M = 32 * QW * RB;           // query rows per workgroup
    constexpr int SUPER = kTileKV * KW;             // keys per iteration
    constexpr int STAGE_BYTES = KW * 2 * kTileBytes;
    // LDS ring of super-tiles: step t reads K(t+1) and V(t) and refills super-tile t + NSTAGE-1.
    // Ping-pong (8-wave workgroups, two waves per SIMD; cdna_hip_programming.md T16): every step is a
    // load segment (all LDS reads / writes) and a compute segment (all MFMAs + softmax, from
    // registers), separated by a barrier; waves 4-7 run one segment behind waves 0-3, so each
    // SIMD pairs one wave's matrix work with its partner's memory work. 4-wave shapes keep one
    // barrier per step with the LDS work spread over the step.
    constexpr bool PINGPONG = (NT == 512) && (MHA_PINGPONG != 0);
    // Offset halves read one segment apart, so the ping-pong ring needs a fourth stage.
    // KW = 4 workgroups are the single-super-tile shape: every split is one super-tile (the
    // planner guarantees it), so one stage suffices.
    constexpr int NSTAGE = KW >= 4 ? 1 : (PINGPONG ? 4 : 3);
    constexpr int NLOAD = (2 * KW * 512) / NT;      // 16-B chunks staged per thread per iteration
    constexpr unsigned SZ = sizeof(TIn);
    static_assert(NLOAD * NT == 2 * KW * 512, "staging must divide evenly");
    constexpr int OROW = 68;  // epilogue: fp32 row pitch in LDS (64 dims + 4 pad: rows r, r+1 on different banks)
    constexpr int EPI_BYTES = (KW * BLOCK_M * OROW + KW * BLOCK_M * 2) * 4 + 16;  // + the last-arriver word
    constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES > EPI_BYTES ? NSTAGE * STAGE_BYTES : EPI_BYTES;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS exceeds 160 KiB");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    lds_char* const lds = (lds_char*)smem;

    STAMP(0);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave
    const int qw = wave % QW;
    const int kw = wave / QW;
    // XCD-aware order (T1): the dispatcher deals consecutive blocks round-robin over the 8 XCDs;
    // renumber (bijectively, any count) so that the blocks sharing one XCD are consecutive in
    // j = block_begin(call) + split + S*(qtile + qtiles*bh): the KV splits and neighbouring query
    // blocks of one (batch, head) run on one XCD, read its K/V through one L2 and leave their
    // split partials there for the combine kernel (which maps its blocks to the same XCD).
    int qtile, bh, split, j;
    {
        // branch-free (one basic block, so every kernarg load issues in one round):
        // XCD x holds j in [x*q8 + min(x, r8), ...)
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
        split = jl % ca.splits;
        const int g = jl / ca.splits;
        qtile = g % ca.qtiles;
        bh = g / ca.qtiles;
    }
    const int nq = ca.nq, nkv = ca.nkv;
    const TIn* Qb = reinterpret_cast<const TIn*>(ca.q) + (size_t)bh * nq * kHeadDim;
    const TIn* Kb = reinterpret_cast<const TIn*>(ca.k) + (size_t)bh * nkv * kHeadDim;
    const TIn* Vb = reinterpret_cast<const TIn*>(ca.v) + (size_t)bh * nkv * kHeadDim;
    const __amdgpu_buffer_rsrc_t q_rs = make_rsrc(Qb, (unsigned)nq * kHeadDim * SZ);
    const __amdgpu_buffer_rsrc_t k_rs = make_rsrc(Kb, (unsigned)nkv * kHeadDim * SZ);
    const __amdgpu_buffer_rsrc_t v_rs = make_rsrc(Vb, (unsigned)nkv * kHeadDim * SZ);
    const int q_row0 = qtile * BLOCK_M + qw * 32 * RB + r;  // + 32 * rb

    const int super_total = (nkv + SUPER - 1) / SUPER;
    const int st_begin = split * ca.tiles_per_split;
    const int st_end = min(super_total, st_begin + ca.tiles_per_split);
    const int n_iter = max(0, st_end - st_begin);

    // Staging: load i of this thread covers tile-tensor tt = i / PER (tile tt/2, K or V by tt&1),
    // row (i % PER) * (NT/8) + tid/8, 16-B chunk tid%8. tt is compile-time, so the K/V descriptor
    // choice stays scalar (no waterfall loop around the buffer load).
    constexpr int PER = 512 / NT;  // loads per thread per 8 KiB tile-tensor
    static_assert(PER * NT == 512, "workgroup size must divide a tile");
    // Two staging register sets: the loads of super-tile t+NSTAGE are issued at step t while the
    // set holding super-tile t+NSTAGE-1 is written to LDS.
    Raw8<TIn> stgA[NLOAD], stgB[NLOAD];
    auto issue = [&](int it, Raw8<TIn>(&stg)[NLOAD]) {
        if (MHA_ABL & ABL_NO_GLOAD) {
#pragma unroll
            for (int i = 0; i < NLOAD; ++i) stg[i] = Raw8<TIn>{};
            return;
        }
        const unsigned soff = (unsigned)(st_begin + it) * SUPER * kHeadDim * SZ;
#pragma unroll
        for (int i = 0; i < NLOAD; ++i) {
            const int tt = i / PER;
            const int row = (i % PER) * (NT / 8) + (tid >> 3);
            const unsigned voff = (unsigned)(((tt >> 1) * kTileKV + row) * kHeadDim + (tid & 7) * 8) * SZ;
            bload8(stg[i], (tt & 1) ? v_rs : k_rs, voff, soff);
        }
    };
    auto write = [&](int stage, const Raw8<TIn>(&stg)[NLOAD]) {
#pragma unroll
        for (int i = 0; i < NLOAD; ++i) {
            const int tt = i / PER;
            const int row = (i % PER) * (NT / 8) + (tid >> 3);
            const int ch = tid & 7;
            lds_write16(lds, stage * STAGE_BYTES + tt * kTileBytes + ((tt & 1) ? v_off(row, ch) : k_off(row, ch)),
                        to_f16(stg[i]));
        }
    };

    // Q fragments (B operand of Sᵀ = K·Qᵀ): lane holds Q[q_row][16s + 8hh .. +7] * 0.125*log2(e), fp16.
    f16x8 qf[RB][4];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            Raw8<TIn> t;
            if (MHA_ABL & ABL_NO_GLOAD) t = Raw8<TIn>{};
            else bload8(t, q_rs, (unsigned)((q_row0 + 32 * rb) * kHeadDim + 16 * s + 8 * hh) * SZ, 0);
            const f16x8 h = to_f16(t);
#pragma unroll
            for (int e = 0; e < 8; ++e) qf[rb][s][e] = (f16)((float)h[e] * kScaleLog2);
        }
    // queries with a non-finite Q: fragments zeroed here, their O rows poisoned to NaN before the
    // merge (q_nonfinite_fix, mha_hd64_device.h), so every merge and combine downstream carries it
    unsigned qbad[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) qbad[rb] = q_nonfinite_fix(qf[rb]);

    // Prologue: stage 0 is published first so QKᵀ(0) starts while the next stage(s) are in flight
    // (published right after it).
    // (single-stage ring, KW = 4: every split is one super-tile, so the body is straight-line and
    // the second staging set never exists)
    if (n_iter > 0) issue(0, stgA);
    if constexpr (NSTAGE > 1) {
        if (n_iter > 1) issue(1, stgB);
    }
    if (n_iter > 0) write(0, stgA);
    if constexpr (NSTAGE > 1) {
        if (n_iter > 2) issue(2, stgA);
    }
    __syncthreads();
    STAMP(1);

    // Per-lane LDS addressing (compile-time parts are added as immediates).
    unsigned k_addr[4];  // + (kw * 2) * kTileBytes: this wave's K tile inside a stage
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = k_off(r, 2 * s + hh) + (kw * 2) * kTileBytes;
    // V tr-read: lane (group g, idx 4qq+pp) supplies row (4hh + qq) + const, columns
    // 32dt + 16(g&1) + 4pp. Swizzle bit b = (qq>>1)&1 flips the 64-B half (dt).
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const unsigned v_addr0 = v_lane + 64 * vb + (kw * 2 + 1) * kTileBytes;        // dims 0..31
    const unsigned v_addr1 = v_lane + 64 * (1 - vb) + (kw * 2 + 1) * kTileBytes;  // dims 32..63

    float m_run[RB];          // reference max of this lane's query, log2 units (s·c)
    // Row sums on the matrix pipe: l_acc = ones_sel · P over every k-step (16x16x32 MFMA), so the
    // 31 adds per tile leave the vector pipe. P (the 32x32x16 B operand) read as a 16x16x32 B
    // operand puts query n (lanes 0-15, 32-47) and n+16 (lanes 16-31, 48-63) in column n; the
    // selector row m takes k-group g when ((m>>2)&1) == (g&1), so lane l's four D rows all hold
    // the sum of query l&31 over the step's 16 keys (both half-waves) — the lane's own query.
    const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
    const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};
    f32x4 l_acc[RB];
    // Bias k-step of the QKᵀ chains: A (key side) = [1, 1, mask] per key row, B (query side) =
    // [-m_hi, -m_lo, 1] per query, in k-slots 0..2 of the lower half-wave (zeros elsewhere).
    // One extra MFMA per chain adds -m (fp16 hi + lo, error ~|m|·2^-22) and the tail mask, so
    // the chain starts from an inline-zero C (no register copy) and the softmax needs no
    // subtraction and no masking VALU.
    const f16 one_h = hh == 0 ? (f16)1.f : (f16)0.f;
    const f16x8 a_bias = f16x8{one_h, one_h, 0, 0, 0, 0, 0, 0};
    f16x8 b_bias[RB];
    auto set_bias = [&](int rb) {
        const f16 hi = (f16)(-m_run[rb]);
        const f16 lo = (f16)(-m_run[rb] - (float)hi);
        b_bias[rb] = hh == 0 ? f16x8{hi, lo, (f16)1.f, 0, 0, 0, 0, 0} : f16x8{0, 0, 0, 0, 0, 0, 0, 0};
    };
    f32x16 o0[RB], o1[RB];  // Oᵀ tiles: dims 0..31 and 32..63, query on the lane
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        m_run[rb] = 0.f;
        l_acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
        b_bias[rb] = f16x8{0, 0, one_h, 0, 0, 0, 0, 0};  // m_run = 0
        o0[rb] = f32x16{};
        o1[rb] = f32x16{};
    }

    // K fragments of the tile in stage kstage (A operand of Sᵀ = K·Qᵀ, 8 x ds_read_b128).
    auto read_k = [&](unsigned kstage, f16x8(&kf)[8]) {
        if (MHA_ABL & ABL_K_CONST) {
#pragma unroll
            for (int s = 0; s < 8; ++s) kf[s] = qf[0][s & 3];
            return;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const unsigned ka = k_addr[s] + kstage;
            kf[2 * s] = lds_read16(lds, ka);
            kf[2 * s + 1] = lds_read16(lds, ka + 32 * 128);
        }
    };
    // QKᵀ chain step i (0..9) of the tile: i = 0,1 are the bias k-steps of the two 32-key halves,
    // then K·Qᵀ over the 4 dim k-steps alternating halves. Scores s·c - m (log2 units), masked
    // keys at ~-65504. Split per MFMA so the caller can interleave vector work between them.
    auto qk_step = [&](int i, const f16x8(&kf)[8], const f16x8& ab0, const f16x8& ab1, f32x16& s0, f32x16& s1,
                       int rb) {
        const f32x16 zero = {};
        if (MHA_ABL & ABL_NO_QK) {
            if (i == 0) s0 = zero;
            if (i == 1) s1 = zero;
            if (i >= 2) keep_live(kf[i - 2]);
            return;
        }
        if (i == 0) s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab0, b_bias[rb], zero, 0, 0, 0);
        else if (i == 1) s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab1, b_bias[rb], zero, 0, 0, 0);
        else if ((i & 1) == 0)
            s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i - 2], qf[rb][(i - 2) >> 1], s0, 0, 0, 0);
        else s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i - 2], qf[rb][(i - 2) >> 1], s1, 0, 0, 0);
    };
    auto qk = [&](unsigned kstage, const f16x8& ab0, const f16x8& ab1, f32x16(&s0)[RB], f32x16(&s1)[RB]) {
        f16x8 kf[8];
        read_k(kstage, kf);
#pragma unroll
        for (int i = 0; i < 10; ++i)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) qk_step(i, kf, ab0, ab1, s0[rb], s1[rb], rb);
    };
    // Tail mask (reference: last KV tile only, …fp16out.cu:475-494): the bias A operand of the
    // tile carries kMaskBias in k-slot 2 for key rows >= nkv. Only the last super-tile of the
    // call can hold such keys; the steady-state loop below never runs it.
    auto a_bias_tile = [&](int t, int half) -> f16x8 {
        const int key = (st_begin + t) * SUPER + kw * kTileKV + 32 * half + r;
        const f16 mk = (hh == 0 && key >= nkv) ? (f16)kMaskBias : (f16)0.f;
        return f16x8{one_h, one_h, mk, 0, 0, 0, 0, 0};
    };
    const bool tail = (st_begin + n_iter) * SUPER > nkv;  // last super-tile of this split is partial

    // Ring stage of tile `it` (scalar, advanced once per step).
    int st_cur = 0;
    // Step `it` writes super-tile it+3 from set `wr` and issues super-tile it+4 into set `is`.
#ifdef MHA_STEPSTAMPS
    unsigned long long ck[4] = {}, ck_prev[4] = {}, ck_sum[4] = {};
    bool ck_first = true;
#endif
    auto step = [&](int it, f32x16(&c0)[RB], f32x16(&c1)[RB], const float(&mxc)[RB], f32x16(&n0)[RB],
                    f32x16(&n1)[RB], float(&mxn)[RB],
                    auto has_next_c, bool mask_next, Raw8<TIn>(&wr)[NLOAD], Raw8<TIn>(&is)[NLOAD],
                    bool may_issue, bool may_write) {
        constexpr bool HAS_NEXT = decltype(has_next_c)::value;
        const int st_nxt = st_cur == NSTAGE - 1 ? 0 : st_cur + 1;
        const int st_fill = st_cur == 0 ? NSTAGE - 1 : st_cur - 1;  // (st_cur + NSTAGE-1) mod NSTAGE
        // In the steady loop the refill is unconditional (may_issue = true at compile time): a
        // super-tile past this split's last one lands in a stage nobody reads, and past nkv the
        // buffer descriptor returns zeros. A conditional load would make the compiler's vmcnt
        // analysis drain every load at the next LDS write.
        if (!(MHA_ABL & ABL_NO_REFILL) && may_issue) issue(it + NSTAGE, is);
        TCLK(ck[0]);

        // Fragment reads first: K of tile it+1 (phase A) and Vᵀ of tile it (phase B); both stages
        // are complete since the last barrier, and the reads land while the bias MFMAs run.
        f16x8 kf[8];
        // (8-wave workgroups with fp32 staging registers read Vᵀ in phase B instead: the early
        // reads' 32 VGPRs would spill there.)
        constexpr bool kEarlyV = !(NT == 512 && SZ == 4);
        f16x8 vfa[2][2], vfb[2][2];
        auto read_v = [&]() {
            if (MHA_ABL & ABL_V_CONST) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss) {
                        vfa[j][ss] = qf[0][j + 2 * ss];
                        vfb[j][ss] = qf[0][(j + 2 * ss + 1) & 3];
                    }
                return;
            }
            const unsigned va0 = v_addr0 + (unsigned)st_cur * STAGE_BYTES;
            const unsigned va1 = v_addr1 + (unsigned)st_cur * STAGE_BYTES;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const unsigned rowc = 128 * (32 * j + 16 * ss);
                    vfa[j][ss] = cat8(tr_read(lds, va0 + rowc), tr_read(lds, va0 + rowc + 8 * 128));
                    vfb[j][ss] = cat8(tr_read(lds, va1 + rowc), tr_read(lds, va1 + rowc + 8 * 128));
                }
        };
        if constexpr (PINGPONG) {
            // Load segment (ping-pong): every LDS access of the step — K(it+1) and Vᵀ(it) fragments
            // into registers, the refill of super-tile it+3 — while the partner wave on this SIMD
            // runs its compute segment; the barrier's lgkmcnt(0) lands them all.
            if constexpr (HAS_NEXT) read_k((unsigned)st_nxt * STAGE_BYTES, kf);
            read_v();
            if (!(MHA_ABL & ABL_NO_REFILL) && may_write) write(st_fill, wr);
            if (!(MHA_ABL & ABL_NO_BARRIER)) __syncthreads();
        }

        // online-softmax decision for tile `it` (first tile: set the max exactly; later tiles:
        // move it only when some query's tile max exceeds it by > kRescaleThr)
        const bool first = (it == 0);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            if (first || __builtin_amdgcn_ballot_w64(mxc[rb] > kRescaleThr) != 0) {  // wave-uniform, rare
                const float d = first ? ((mxc[rb] < kEmptyMax) ? 0.f : mxc[rb])  // fully masked tile: m = 0
                                      : fmaxf(mxc[rb], 0.f);
                const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-d);
                o0[rb] *= alpha;
                o1[rb] *= alpha;
                l_acc[rb] *= alpha;
                m_run[rb] += d;
                c0[rb] -= d;
                c1[rb] -= d;
                set_bias(rb);
            }
        }

        if constexpr (!PINGPONG) {
            if constexpr (HAS_NEXT) read_k((unsigned)st_nxt * STAGE_BYTES, kf);
            if constexpr (kEarlyV && !HAS_NEXT) read_v();
        }

        // phase A: QKᵀ(it+1) on the matrix pipe ‖ exp(it) on the vector pipe, pinned as one MFMA
        // followed by three v_exp_f32 per gap (8 + 3·8 issue cycles fill the MFMA's 32).
        auto exp_at = [&](int e) {  // e in [0, 32*RB): query block e/32, score e%32
            if (MHA_ABL & (ABL_NO_EXP | ABL_NO_SOFTMAX)) return;
            const int rb = e >> 5, i = e & 31;
            if (i < 16) c0[rb][i] = __builtin_amdgcn_exp2f(c0[rb][i]);
            else c1[rb][i - 16] = __builtin_amdgcn_exp2f(c1[rb][i - 16]);
        };
        if constexpr (HAS_NEXT) {
            const f16x8 ab0 = mask_next ? a_bias_tile(it + 1, 0) : a_bias;
            const f16x8 ab1 = mask_next ? a_bias_tile(it + 1, 1) : a_bias;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 10; ++i)
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) {
                    qk_step(i, kf, ab0, ab1, n0[rb], n1[rb], rb);
                    // Vᵀ reads queue behind the K reads (phase A carries all fragment reads).
                    if (!PINGPONG && kEarlyV && i == 2 && rb == 0) read_v();
                    const int g = i * RB + rb;
                    exp_at(3 * g);
                    exp_at(3 * g + 1);
                    exp_at(3 * g + 2);
                    __builtin_amdgcn_sched_barrier(0);
                }
            TCLK(ck[1]);
#pragma unroll
            for (int e = 30 * RB; e < 32 * RB; ++e) exp_at(e);
        } else {
#pragma unroll
            for (int e = 0; e < 32 * RB; ++e) exp_at(e);
        }
        f16x8 p[RB][2][2];  // P (f16) as the B operand: registers 8ss..8ss+7 of a 32x32 tile = k-step ss
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                p[rb][0][0][e] = (f16)c0[rb][e];
                p[rb][0][1][e] = (f16)c0[rb][8 + e];
                p[rb][1][0][e] = (f16)c1[rb][e];
                p[rb][1][1][e] = (f16)c1[rb][8 + e];
            }

        // phase B: Oᵀ += Vᵀ·Pᵀ (it) and the row sums on the matrix pipe ‖ row max (it+1) (and, in
        // the one-barrier form, the LDS refill of super-tile it+3: its stage held tile it-1).
        if constexpr (!PINGPONG) {
            if constexpr (!kEarlyV) read_v();
            if (!(MHA_ABL & ABL_NO_REFILL) && may_write) write(st_fill, wr);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) {
                    if (MHA_ABL & ABL_NO_PV) {
                        keep_live(vfa[j][ss]);
                        keep_live(vfb[j][ss]);
                        keep_live(p[rb][j][ss]);
                    } else {
                        o0[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[j][ss], p[rb][j][ss], o0[rb], 0, 0, 0);
                        o1[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[j][ss], p[rb][j][ss], o1[rb], 0, 0, 0);
                    }
                    if (!(MHA_ABL & ABL_NO_SOFTMAX))
                        l_acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, p[rb][j][ss], l_acc[rb], 0, 0, 0);
                }
        if constexpr (HAS_NEXT) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                if (MHA_ABL & ABL_NO_SOFTMAX) mxn[rb] = 0.f;
                else mxn[rb] = xhalf_max(tree_max(n0[rb], n1[rb]));
            }
        }

        TCLK(ck[2]);
#ifdef MHA_STEPSTAMPS
        if (HAS_NEXT) {  // previous full step's phases (its clocks have returned by now)
            ck_sum[0] += ck_prev[1] - ck_prev[0];
            ck_sum[1] += ck_prev[2] - ck_prev[1];
            ck_sum[2] += ck_prev[3] - ck_prev[2];
            ck_sum[3] += 1;
        }
#endif
        if (!(MHA_ABL & ABL_NO_BARRIER)) __syncthreads();
        TCLK(ck[3]);
#ifdef MHA_STEPSTAMPS
        if (HAS_NEXT) {
            for (int i = 0; i < 4; ++i) ck_prev[i] = ck[i];
        }
#endif
        st_cur = st_nxt;
    };

    // Scores ping-pong between two named register sets (no runtime-indexed arrays, no copies).
    f32x16 sA0[RB], sA1[RB], sB0[RB], sB1[RB];
    float mxA[RB], mxB[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) mxA[rb] = mxB[rb] = 0.f;
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (n_iter > 0) {
        if (tail && n_iter == 1)
            qk(0u, a_bias_tile(0, 0), a_bias_tile(0, 1), sA0, sA1);
        else
            qk(0u, a_bias, a_bias, sA0, sA1);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) mxA[rb] = xhalf_max(tree_max(sA0[rb], sA1[rb]));
    }
    if constexpr (NSTAGE == 1) {
        if (n_iter > 0) step(0, sA0, sA1, mxA, sB0, sB1, mxB, F_{}, false, stgA, stgA, false, false);
    } else {
    if (n_iter > 1) write(1, stgB);
    if constexpr (NSTAGE == 4) {
        if (n_iter > 3) issue(3, stgB);
        if (n_iter > 2) write(2, stgA);
    }
    if (n_iter > 1) __syncthreads();
    // The set the first step writes from (super-tile NSTAGE-1) and the one it issues into.
    Raw8<TIn>(&stg0)[NLOAD] = NSTAGE == 4 ? stgB : stgA;
    Raw8<TIn>(&stg1)[NLOAD] = NSTAGE == 4 ? stgA : stgB;
#ifndef MHA_PRIO
#define MHA_PRIO 0
#endif
    // (static priority for the second-dispatched half of an 8-wave workgroup: diagnostic switch)
    if (MHA_PRIO && NT == 512 && wave >= 4) __builtin_amdgcn_s_setprio(1);
    // Ping-pong offset: the second half starts one phase late (one extra barrier before the loop,
    // matched by one extra barrier of the first half after it).
    const bool late_half = PINGPONG && wave >= 4;
    if (late_half) __syncthreads();
    int it = 0;
    // Steady state: tiles it+1 and it+2 exist and neither is the (possibly partial) last one.
    // Refill issue / write are unconditional here (see step).
    for (; it + 3 < n_iter; it += 2) {
        step(it, sA0, sA1, mxA, sB0, sB1, mxB, T_{}, false, stg0, stg1, true, true);
        step(it + 1, sB0, sB1, mxB, sA0, sA1, mxA, T_{}, false, stg1, stg0, true, true);
    }
    // Tail (at most 3 iterations): same step with the mask flag live; scores and the pending
    // staging set move back after each step.
    for (; it + 1 < n_iter; ++it) {
        step(it, sA0, sA1, mxA, sB0, sB1, mxB, T_{}, tail && (it + 2 == n_iter), stg0, stg1, it + NSTAGE < n_iter,
             it + NSTAGE - 1 < n_iter);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            sA0[rb] = sB0[rb];
            sA1[rb] = sB1[rb];
            mxA[rb] = mxB[rb];
        }
#pragma unroll
        for (int i = 0; i < NLOAD; ++i) stg0[i] = stg1[i];
    }
    if (it < n_iter) step(it, sA0, sA1, mxA, sB0, sB1, mxB, F_{}, false, stg0, stg1, false, false);
    if (PINGPONG && !late_half) __syncthreads();
    }  // NSTAGE > 1
    STAMP(2);

    // ---- epilogue ----
    // Every wave stages its Oᵀ accumulators as fp32 rows (at its own max) plus (m, l) in LDS;
    // then all threads merge the KW key-split partials of a row and write whole 16-byte row
    // chunks (a wave stores complete rows: coalesced, few store instructions).
    // A wave that saw no key (all of its tiles past nkv) gets m = -inf (weight 0). The test uses
    // the cross-half total: the halves hold disjoint keys but the SAME query's m and O dims.
    float* ol = reinterpret_cast<float*>(smem);     // [KW][BLOCK_M][OROW]
    float* mlb = ol + KW * BLOCK_M * OROW;          // [KW][BLOCK_M][2]
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        if (qbad[rb]) {  // wave-uniform, rare
            const float pois = inv_or_nan(1.f, qbad[rb], r);  // NaN on a bad query's lanes, else 1
            o0[rb] *= pois;
            o1[rb] *= pois;
        }
        const float L_w = l_acc[rb][0];  // the row-sum MFMA already spans both half-waves
        const float m_w = (L_w > 0.f) ? m_run[rb] : -INFINITY;
        const int row = qw * 32 * RB + 32 * rb + r;
        float* dst = ol + (kw * BLOCK_M + row) * OROW;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d = 8 * g4 + 4 * hh;
            *reinterpret_cast<f32x4*>(dst + d) =
                f32x4{o0[rb][4 * g4], o0[rb][4 * g4 + 1], o0[rb][4 * g4 + 2], o0[rb][4 * g4 + 3]};
            *reinterpret_cast<f32x4*>(dst + 32 + d) =
                f32x4{o1[rb][4 * g4], o1[rb][4 * g4 + 1], o1[rb][4 * g4 + 2], o1[rb][4 * g4 + 3]};
        }
        if (hh == 0) *reinterpret_cast<float2*>(mlb + (kw * BLOCK_M + row) * 2) = make_float2(m_w, L_w);
    }
    __syncthreads();
    STAMP(3);

    // Thread -> (row, chunk of 8 dims); 8 threads per row, NT/8 rows per pass. Stores are 16-B
    // buffer stores through per-head descriptors (cache policy MHA_ST_AUX / MHA_PART_AUX).
    const int q_base = qtile * BLOCK_M;
    const __amdgpu_buffer_rsrc_t o_rs =
        make_rsrc(reinterpret_cast<TOut*>(ca.o) + (size_t)bh * nq * kHeadDim, (unsigned)(nq * kHeadDim * sizeof(TOut)));
    const __amdgpu_buffer_rsrc_t po_rs =
        make_rsrc(reinterpret_cast<TOut*>(ca.part_o) + (size_t)bh * ca.splits * nq * kHeadDim,
                  (unsigned)(ca.splits * nq * kHeadDim * sizeof(TOut)));
    // In-launch combine: every split's workgroup publishes its partial write-through (sc1) and
    // takes a ticket; the group's last arriver reads all the group's partials back and writes O
    // (same arithmetic and order as the combine kernel, so both forms give the same bits). Visibility follows MI355X_MICROARCH.md "Valid forms" (table
    // row 1): all partial bytes stored sc1 and drained (vmcnt(0)) before one lane's agent-scope
    // add, every load of them an sc1 buffer load, the other waves behind a barrier.
    const bool fused = a.tickets != nullptr && ca.splits > 1;
    const __amdgpu_buffer_rsrc_t pml_rs =
        make_rsrc(ca.part_ml + (size_t)bh * ca.splits * nq, (unsigned)(ca.splits * nq * sizeof(float2)));
    // Epilogue items: (row, chunk of DPT dims). DPT = 8 while a pass has no more threads than
    // items; workgroups with twice as many threads as 8-dim items (32-row (1,8)) use 4-dim chunks
    // so every thread merges and stores.
    constexpr int DPT = BLOCK_M * 8 >= NT ? 8 : 4;
    constexpr int CPR = kHeadDim / DPT;  // chunks per row
    constexpr int EITEMS = BLOCK_M * CPR;
    constexpr int EPASS = (EITEMS + NT - 1) / NT;
    static_assert(EITEMS % NT == 0, "epilogue items must tile the workgroup");
    using RawD = typename std::conditional<DPT == 8, Raw8<TOut>, Raw4<TOut>>::type;
    // merge of the KW key-wave partials of (row, dims c..c+DPT-1) staged in LDS
    auto merge_waves = [&](int row, int c, float& M, float& L, f32x4& acc0, f32x4& acc1) {
        M = -INFINITY;
        float2 ml[KW];
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            ml[k] = *reinterpret_cast<const float2*>(mlb + (k * BLOCK_M + row) * 2);
            M = fmaxf(M, ml[k].x);
        }
        acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
        acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
        L = 0.f;
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const float w = (ml[k].x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml[k].x - M);
            L += w * ml[k].y;
            const float* src = ol + (k * BLOCK_M + row) * OROW + c;
            acc0 += w * *reinterpret_cast<const f32x4*>(src);
            if constexpr (DPT == 8) acc1 += w * *reinterpret_cast<const f32x4*>(src + 4);
        }
    };
#pragma unroll
    for (int pass = 0; pass < EPASS; ++pass) {
        const int idx = pass * NT + tid;
        const int row = idx / CPR;
        const int chunk = idx % CPR;
        const int c = chunk * DPT;
        const int q = q_base + row;
        float M, L;
        f32x4 acc0, acc1;
        merge_waves(row, c, M, L, acc0, acc1);
        if (q < nq && !(MHA_ABL & ABL_NO_STORE)) {
            if (ca.splits == 1) {
                const float inv = 1.f / L;
                store_dims<TOut, DPT, MHA_ST_AUX>(o_rs, (unsigned)((q * kHeadDim + c) * sizeof(TOut)), acc0 * inv,
                                                  acc1 * inv);
            } else {
                // Partial O_s / l_s in the output precision (fp16 halves the partial traffic of
                // the fp16 path; the fp32-output path keeps fp32), merged with weights l_s·2^(m_s-M).
                const unsigned prow = (unsigned)(split * nq + q);
                const float inv = (L > 0.f) ? 1.f / L : 0.f;
                const unsigned poff = prow * (unsigned)(kHeadDim * sizeof(TOut)) + c * (unsigned)sizeof(TOut);
                if (fused) {
                    store_dims<TOut, DPT, kSC1>(po_rs, poff, acc0 * inv, acc1 * inv);
                    if (chunk == 0)
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(M, L)), pml_rs,
                                                              prow * (unsigned)sizeof(float2), 0, kSC1);
                } else {
                    store_dims<TOut, DPT, MHA_PART_AUX>(po_rs, poff, acc0 * inv, acc1 * inv);
                    if (chunk == 0) ca.part_ml[((size_t)bh * ca.splits) * nq + prow] = make_float2(M, L);
                }
            }
        }
    }
    if (fused) {  // workgroup-uniform
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        unsigned* last_word = reinterpret_cast<unsigned*>(smem + EPI_BYTES - 16);
        if (tid == 0) {
            unsigned* t = a.tickets + (j - split);
            const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned last = old + 1 == (unsigned)ca.splits;
            if (last) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *last_word = last;
        }
        __syncthreads();
        STAMP(5);
        if (*last_word) {
#pragma unroll
            for (int pass = 0; pass < EPASS; ++pass) {
                const int idx = pass * NT + tid;
                const int row = idx / CPR;
                const int c = (idx % CPR) * DPT;
                const int q = q_base + row;
                if (q >= nq) continue;
                // every split's partial as stored (its own too), merged in split order exactly as
                // the combine kernel does: the result does not depend on which split came last
                float2 ml[kMaxSplits];
                RawD pv[kMaxSplits];
#pragma unroll
                for (int s2 = 0; s2 < kMaxSplits; ++s2) {
                    if (s2 < ca.splits) {
                        const unsigned prow = (unsigned)(s2 * nq + q);
                        ml[s2] = __builtin_bit_cast(
                            float2, __builtin_amdgcn_raw_buffer_load_b64(pml_rs, prow * (unsigned)sizeof(float2), 0, kSC1));
                        const unsigned off = prow * (unsigned)(kHeadDim * sizeof(TOut)) + c * (unsigned)sizeof(TOut);
                        if constexpr (DPT == 8) bload8_aux<kSC1>(pv[s2], po_rs, off);
                        else bload4_aux<kSC1>(pv[s2], po_rs, off);
                    }
                }
                float Mt = -INFINITY;
#pragma unroll
                for (int s2 = 0; s2 < kMaxSplits; ++s2)
                    if (s2 < ca.splits) Mt = fmaxf(Mt, ml[s2].x);
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                float L = 0.f;
#pragma unroll
                for (int s2 = 0; s2 < kMaxSplits; ++s2) {
                    if (s2 < ca.splits) {
                        const float w = split_weight(ml[s2], Mt);
                        L += w;
                        if constexpr (DPT == 8) {
                            f32x4 lo, hi;
                            raw8_to_f32(pv[s2], lo, hi);
                            split_accumulate(acc0, w, lo);
                            split_accumulate(acc1, w, hi);
                        } else {
                            split_accumulate(acc0, w, raw4_to_f32(pv[s2]));
                        }
                    }
                }
                const float inv = 1.f / L;
                if (!(MHA_ABL & ABL_NO_STORE))
                    store_dims<TOut, DPT, MHA_ST_AUX>(o_rs, (unsigned)((q * kHeadDim + c) * sizeof(TOut)),
                                                      split_scale(acc0, inv), split_scale(acc1, inv));
            }
        }
    }
    STAMP(4);
#ifdef MHA_STEPSTAMPS
    if (lane == 0) {
        unsigned long long* dst = a.stamps + (1 << 16) + ((size_t)blockIdx.x * 8 + wave) * 4;
        // the first accumulated step has zero deltas (ck_prev unset): subtract it out on the host
        for (int i = 0; i < 4; ++i) dst[i] = ck_sum[i];
    }
    (void)ck_first;
#endif
}

// ----------------------------------------------------------------------------------------
// Split-KV combine: O = Σ_s w_s Ô_s / Σ_s w_s with w_s = l_s·2^(m_s - M) (m in log2 units) and
// Ô_s = O_s / l_s the partial as stored (TOut precision). One thread per (row, 4-dim chunk).
// Block b serves XCD b % 8: it combines rows whose partials the main kernel produced on that same XCD (same bijective block order), so the reads hit L2. All
// partials of a row are loaded in one round trip (S <= kMaxSplits).
// ----------------------------------------------------------------------------------------

struct CombineCall {
    const void* part_o;
    const float2* part_ml;
    void* out;
    int nq;
    int splits;
    int qtiles;       // query blocks per (batch, head) of the main kernel
    int pad_;
};
// Block b of the combine grid serves XCD x = b % 8 (k = b / 8): blocks k in
// [kbeg[x][i], kbeg[x][i+1]) serve call i, starting at query group gbeg[x][i] (the first group
// whose first split block ran on XCD x). A block is 16 rows of one query group (block_m is a
// multiple of 16), so the call, the group and its (batch*head, query block) are block-uniform.
struct CombineArgs {
    CombineCall c[kMaxCalls];
    int kbeg[8][kMaxCalls + 1];
    int gbeg[8][kMaxCalls];
    int n_calls;
    int block_m_log2;  // rows per query block = 1 << block_m_log2
    int per_xcd;       // combine blocks per XCD
    int main_blocks;   // single-call form: grid of the main kernel
    int groups0;       // single-call form: query groups of call 0
};

template <typename T>
__device__ __forceinline__ f32x4 load4f(const T* p) {
    if constexpr (sizeof(T) == 2) {
        const f16x4 h = *reinterpret_cast<const f16x4*>(p);
        return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    } else {
        return *reinterpret_cast<const f32x4*>(p);
    }
}

// MULTI = false (one call): the XCD's first group is computed from the main grid in scalar
// arithmetic (no dependent kernarg table lookups); MULTI = true reads the per-XCD table.
template <typename TOut, bool MULTI>
__global__ __launch_bounds__(256) void mha_hd64_combine_kernel(CombineArgs c) {
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    CombineCall cc = c.c[0];
    int kb = 0, gb;
    if constexpr (MULTI) {
        int ci = -1;
#pragma unroll
        for (int i = 0; i < kMaxCalls; ++i)
            if (i < c.n_calls && k >= c.kbeg[x][i] && k < c.kbeg[x][i + 1]) ci = i;
        if (ci < 0) return;
        kb = c.kbeg[x][0];
        gb = c.gbeg[x][0];
#pragma unroll
        for (int i = 1; i < kMaxCalls; ++i)
            if (ci == i) {
                cc = c.c[i];
                kb = c.kbeg[x][i];
                gb = c.gbeg[x][i];
            }
    } else {
        const int T = c.main_blocks, q8 = T >> 3, r8 = T & 7;
        const int jlo = x * q8 + min(x, r8), jhi = (x + 1) * q8 + min(x + 1, r8);
        const int groups = c.groups0;
        const int glo = min(groups, (jlo + cc.splits - 1) / cc.splits);
        const int ghi = min(groups, (jhi + cc.splits - 1) / cc.splits);
        if (k >= ((ghi - glo) << c.block_m_log2) / 16) return;
        gb = glo;
    }
    const int row0 = (k - kb) * 16;                       // first row of this block in the segment
    const int g = gb + (row0 >> c.block_m_log2);          // block-uniform query group
    const int bh = g / cc.qtiles, qt = g - bh * cc.qtiles;
    const int q = (qt << c.block_m_log2) + (row0 & ((1 << c.block_m_log2) - 1)) + ((int)threadIdx.x >> 4);
    if (q >= cc.nq) return;
    const int chunk = threadIdx.x & 15;
    const size_t base = (size_t)bh * cc.splits * cc.nq + q;
    const TOut* po = reinterpret_cast<const TOut*>(cc.part_o);
    float2 ml[kMaxSplits];
    f32x4 v[kMaxSplits];
#pragma unroll
    for (int s = 0; s < kMaxSplits; ++s) {
        if (s < cc.splits) {
            const size_t pr = base + (size_t)s * cc.nq;
            ml[s] = cc.part_ml[pr];
            v[s] = load4f<TOut>(po + pr * kHeadDim + chunk * 4);
        }
    }
    float M = -INFINITY;
#pragma unroll
    for (int s = 0; s < kMaxSplits; ++s)
        if (s < cc.splits) M = fmaxf(M, ml[s].x);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
#pragma unroll
    for (int s = 0; s < kMaxSplits; ++s) {
        if (s < cc.splits) {
            const float w = split_weight(ml[s], M);
            L += w;
            split_accumulate(acc, w, v[s]);
        }
    }
    const f32x4 o = split_scale(acc, 1.f / L);
    TOut* out = reinterpret_cast<TOut*>(cc.out) + ((size_t)bh * cc.nq + q) * kHeadDim + chunk * 4;
    store4<TOut>(out, o[0], o[1], o[2], o[3]);
}

template <typename TIn, typename TOut, int QW, int KW, int RB, bool MULTI>
hipError_t launch_fwd(const FwdArgs& a, int grid, hipStream_t stream) {
    hipLaunchKernelGGL((mha_hd64_fwd_kernel<TIn, TOut, QW, KW, RB, MULTI>), dim3(grid), dim3(64 * QW * KW), 0, stream,
                       a);
    return hipGetLastError();
}

// Grouped launches (several calls) exist for the shapes the planner picks on its own.
template <typename TIn, typename TOut>
hipError_t launch_fwd_shape(const FwdArgs& a, int grid, int qw, int kw, int rb, hipStream_t stream) {
    if (a.n_calls > 1) {
        switch (rb * 64 + qw * 8 + kw) {
            case 64 + 4 * 8 + 1: return launch_fwd<TIn, TOut, 4, 1, 1, true>(a, grid, stream);  // > 256 128-row blocks
            case 64 + 2 * 8 + 2: return launch_fwd<TIn, TOut, 2, 2, 1, true>(a, grid, stream);
            case 64 + 4 * 8 + 2: return launch_fwd<TIn, TOut, 4, 2, 1, true>(a, grid, stream);
            case 128 + 2 * 8 + 2: return launch_fwd<TIn, TOut, 2, 2, 2, true>(a, grid, stream);
            case 64 + 2 * 8 + 4: return launch_fwd<TIn, TOut, 2, 4, 1, true>(a, grid, stream);
            case 64 + 1 * 8 + 8: return launch_fwd<TIn, TOut, 1, 8, 1, true>(a, grid, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (rb * 64 + qw * 8 + kw) {
        case 64 + 4 * 8 + 1: return launch_fwd<TIn, TOut, 4, 1, 1, false>(a, grid, stream);
        case 64 + 2 * 8 + 2: return launch_fwd<TIn, TOut, 2, 2, 1, false>(a, grid, stream);
        case 64 + 1 * 8 + 2: return launch_fwd<TIn, TOut, 1, 2, 1, false>(a, grid, stream);
        case 64 + 4 * 8 + 2: return launch_fwd<TIn, TOut, 4, 2, 1, false>(a, grid, stream);
        case 64 + 2 * 8 + 4: return launch_fwd<TIn, TOut, 2, 4, 1, false>(a, grid, stream);
        case 64 + 1 * 8 + 4: return launch_fwd<TIn, TOut, 1, 4, 1, false>(a, grid, stream);
        case 64 + 1 * 8 + 8: return launch_fwd<TIn, TOut, 1, 8, 1, false>(a, grid, stream);
        case 128 + 2 * 8 + 2: return launch_fwd<TIn, TOut, 2, 2, 2, false>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

template <typename TOut>
hipError_t launch_combine(const CombineArgs& c, hipStream_t stream) {
    if (c.n_calls > 1)
        hipLaunchKernelGGL((mha_hd64_combine_kernel<TOut, true>), dim3(8 * c.per_xcd), dim3(256), 0, stream, c);
    else
        hipLaunchKernelGGL((mha_hd64_combine_kernel<TOut, false>), dim3(8 * c.per_xcd), dim3(256), 0, stream, c);
    return hipGetLastError();
}

bool valid_shape(int qw, int kw, int rb) {
    if (rb == 2) return qw == 2 && kw == 2;
    return rb == 1 && ((qw == 4 && kw == 1) || (qw == 2 && kw == 2) || (qw == 1 && kw == 2) || (qw == 4 && kw == 2) ||
                       (qw == 2 && kw == 4) || (qw == 1 && kw == 4) || (qw == 1 && kw == 8));
}

unsigned long long* g_stamps = nullptr;  // diagnostic builds (MHA_STAMPS) only

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

void set_stamp_buffer(void* p) { g_stamps = reinterpret_cast<unsigned long long*>(p); }

// ---- arrival tickets of the in-launch combine ----
// Every ticket a launch uses is zero when it starts and zero when it ends (the last arriver of
// each group resets its own), so a ticket array needs no per-call reset as long as no two launches
// that use it run concurrently:
//  * eager launches: one array per (device, stream) -- launches on one stream are serialised;
//  * launches recorded under stream capture: a slice of their own, carved from a per-device arena
//    (an instantiated graph never runs concurrently with itself, while two graphs captured on one
//    stream may be replayed side by side).
// Arrays are created only outside capture (hipMalloc + memset, then a one-time stream sync for the
// arena); a launch that finds no tickets combines in the second kernel instead. Nothing is freed
// (a launch in flight or a graph may still reference it). A half-used arena is replaced at the
// next eager launch (tickets_for), at most kMaxArenas times per device: memory for tickets is
// bounded by (kMaxArenas + 1) x 4 MiB per device plus the per-stream arrays; past the cap, captures
// that find the arena full use the combine kernel (same bits). So an EAGER split launch may
// allocate device memory (never more than that bound); it does so with this thread's capture mode
// exchanged to relaxed, so a global-mode capture running on another thread stays valid.
namespace {
int g_fused = -1;  // -1: unset (env MHA_HD64_FUSED_COMBINE, default on), 0 off, 1 on
std::mutex g_ticket_mu;
std::map<std::pair<int, hipStream_t>, std::pair<unsigned*, int>> g_tickets;
struct Arena {
    unsigned* base = nullptr;
    int cap = 0;
    int used = 0;
    int replaced = 0;
};
std::map<int, Arena> g_arena;
thread_local int g_last_combine = 0;  // this thread's last launch: 0 no split, 1 in-launch, 2 kernel
constexpr int kArenaTickets = 1 << 20;  // 4 MiB per device
constexpr int kMaxArenas = 4;           // replacements per device
// Scoped relaxed capture mode for this thread: allocation calls stay legal (and do not invalidate
// another thread's global-mode capture) while any capture is in progress in the process.
struct RelaxedCapture {
    hipStreamCaptureMode prev = hipStreamCaptureModeRelaxed;
    RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&prev); }
    ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&prev); }
};
}  // namespace

int last_combine_form() { return g_last_combine; }

namespace {
std::atomic<int> g_concurrency{1};
}
int concurrency_hint() { return g_concurrency.load(std::memory_order_relaxed); }
int set_concurrency_hint(int streams) { return g_concurrency.exchange(std::max(1, streams)); }

void set_fused_combine(int enable) {
    std::lock_guard<std::mutex> lk(g_ticket_mu);
    g_fused = enable ? 1 : 0;
}

static bool fused_enabled() {
    std::lock_guard<std::mutex> lk(g_ticket_mu);
    if (g_fused < 0) {
        const char* e = std::getenv("MHA_HD64_FUSED_COMBINE");
        g_fused = (e && e[0] == '0') ? 0 : 1;
    }
    return g_fused == 1;
}

static unsigned* zeroed_tickets(int count, hipStream_t stream) {
    unsigned* p = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&p), (size_t)count * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, (size_t)count * sizeof(unsigned), stream) != hipSuccess) {
        (void)hipFree(p);
        return nullptr;
    }
    return p;
}

static unsigned* tickets_for(hipStream_t stream, int count) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_ticket_mu);
    Arena& ar = g_arena[dev];
    if (cs != hipStreamCaptureStatusNone) {  // a slice owned by this recorded launch
        const int n = (count + 63) & ~63;
        if (!ar.base || ar.used + n > ar.cap) return nullptr;
        unsigned* p = ar.base + ar.used;
        ar.used += n;
        return p;
    }
    // First eager launch on this device: the arena for later captures. An arena more than half
    // carved is replaced by a fresh one at the next eager launch (the old one stays allocated: graphs
    // recorded from it may still run), at most kMaxArenas times, so captures run out only after
    // 512 Ki tickets recorded with no eager launch in between.
    RelaxedCapture relaxed;
    if (!ar.base || (ar.used > ar.cap / 2 && ar.replaced < kMaxArenas)) {
        unsigned* fresh = zeroed_tickets(kArenaTickets, stream);
        if (fresh && hipStreamSynchronize(stream) == hipSuccess) {
            if (ar.base) ++ar.replaced;  // (counted only once a fresh arena is installed)
            ar.base = fresh;
            ar.cap = kArenaTickets;
            ar.used = 0;
        } else {
            if (fresh) (void)hipFree(fresh);  // a failed attempt leaks nothing
            if (!ar.base) ar.cap = 0;
        }
    }
    auto& slot = g_tickets[{dev, stream}];
    if (slot.first && slot.second >= count) return slot.first;
    const int cap = std::max(count, 4096);
    unsigned* p = zeroed_tickets(cap, stream);
    if (!p) return nullptr;
    slot = {p, cap};
    return p;
}

size_t split_workspace_bytes(const Call& c, int splits) {
    if (splits <= 1) return 0;
    const size_t rows = (size_t)c.batch * c.heads * splits * c.nq;
    const size_t o_bytes = rows * kHeadDim * sizeof(float);  // fp32 bound (fp16 partials use half)
    return align256(o_bytes) + align256(rows * sizeof(float2));
}

static bool direct_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("MHA_HD64_DIRECT");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Tiles of 64 keys per wave of the single-pass kernels for this launch, or 0 if they do not apply:
// fp16 input, every call's keys within 8 waves x 2 tiles (x 2 passes for 32-row blocks), and at most max_wgs workgroups of `rows`
// query rows. 16-row blocks: at most 256 (one per CU, one round). 32-row blocks: at most 768 —
// up to three rounds of 256 still beat the LDS ring's plans there (tools/batch_sweep.py, graph
// replay, us per launch, 32-row kernel vs planner's ring plan: B=3 N=1024 10.3 vs 18.1, B=6 15.3 vs
// 19.7, B=6 N=512 6.3 vs 9.5, B=12 N=512 8.7 vs 13.5; at 1024 blocks the ring wins: B=8 N=1024
// 15.5 vs 21.0, B=16 N=512 10.4 vs 11.2). Past one round with 512 < nkv <= 1024 the 32-row kernel
// runs its two-workgroups-per-CU form (launch_direct): B=3 8.86 vs 10.28 for one per CU (ring
// 10.43), B=4 9.41 vs 10.68 (10.77), B=6 13.15 vs 15.23 (14.11); B=8 16.85 vs ring 15.33.
constexpr long kDirectMaxWgs16 = 256, kDirectMaxWgs32 = 768;
static int direct_tiles_for(const Call* calls, int n, InType in, bool forced, int rows = 32) {
    if (in != InType::F16 || (!forced && !direct_enabled())) return 0;
    long wgs = 0;
    int tiles = 1;
    // keys per call: <= 2048 (tiles 3, 4: the two-pass forms, 4 waves x 2 x 4 tiles)
    const int max_tiles = 4;
    for (int i = 0; i < n; ++i) {
        if (calls[i].nkv > 8 * max_tiles * kTileKV) return 0;
        tiles = std::max(tiles, (calls[i].nkv + 8 * kTileKV - 1) / (8 * kTileKV));
        wgs += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + rows - 1) / rows);
    }
    // two-pass forms (tiles 3, 4), one round: 16-row blocks up to 256, 32-row blocks from 96 on (tools/batch_sweep.py, us per launch, two-pass 16-row / 32-row
    // kernel vs ring plan: 2048^2 B=1 - / 9.87 vs 13.04, B=2 - / 17.6 vs 17.3; 1536^2 B=1 - / 8.13
    // vs 11.12; Nq x Nkv 1024x2048 7.40 / 8.57 vs 10.74, 768x2048 6.79 / 8.38 vs 10.24,
    // 512x2048 6.68 / 8.33 vs 7.95, 256x2048 6.61 / 8.31 vs 7.69, 1024x1536 6.32 / 8.05 vs 9.84)
    // Past one round the 32-row kernel's two-workgroups-per-CU form (4 passes x 2 tiles) takes
    // over up to 768 blocks (vs the ring plan: 2x4x2048^2 16.1 vs 17.8, 3x 21.7 vs 23.3; 2x4x1536^2
    // 12.0 vs 13.5, 3x 18.0 vs 17.7, 4x 18.6 vs 18.7; 4x4x1024x2048 15.0 vs 17.8).
    if (tiles > 2 && !forced && (rows == 16 ? wgs > 256 : wgs < 96)) return 0;
    const long max_wgs = rows == 16 ? kDirectMaxWgs16 : kDirectMaxWgs32;
    return (forced || wgs <= max_wgs) ? tiles : 0;
}

// The 16-row single-pass kernel first (default; MHA_HD64_DIRECT_ROWS=32 keeps 32-row blocks)
static bool direct16_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("MHA_HD64_DIRECT_ROWS");
        return !(e && e[0] == '3');
    }();
    return on;
}

// The persistent streaming kernel (mha_hd64_stream.hip) for fp16 launches of more than one round
// of 128-row blocks (MHA_HD64_STREAM=1 / set_stream_mode(1), the default; 0: never). Round 4's
// branch-free step loop: 16 batched 1x4x1024^2 calls 23.6 vs 26.0 us for the ring kernel, 32
// calls 44.2 vs 49.8 (profiles/r04/stream_check.jsonl).
std::atomic<int> g_stream_mode{-1};
int stream_env() {
    int v = g_stream_mode.load();
    if (v < 0) {
        const char* e = std::getenv("MHA_HD64_STREAM");
        int expect = -1;
        g_stream_mode.compare_exchange_strong(expect, (e && e[0] == '0') ? 0 : 1);
        v = g_stream_mode.load();
    }
    return v;
}
static bool stream_auto(const Call* calls, int n, InType in) {
    if (in != InType::F16 || stream_env() <= 0) return false;
    long blocks128 = 0;
    for (int i = 0; i < n; ++i) blocks128 += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + 127) / 128);
    return blocks128 > 256;
}

GroupPlan plan_group(const Call* calls, int n, size_t ws_bytes, int force_q_waves, int force_kv_waves,
                     int force_splits, InType in) {
    GroupPlan p{};
    if (force_q_waves == kForceStream || (force_q_waves == 0 && stream_auto(calls, n, in))) {
        if (in == InType::F16) {
            // 8 waves (256-row items, one workgroup per CU: the two waves of a SIMD stay in step, no
            // co-resident imbalance) when their last round of 256 items is at least 3/4 full; else
            // 4 (128-row items, two per CU: the older workgroup of a CU takes the extra items of a
            // partial round). tools/stream_check.py, 1024^2 calls per launch, us: 12 calls 20.0 vs
            // 21.1, 16: 22.5 vs 23.4, 24: 38.5 vs 34.0, 32: 43.3 vs 44.7, 64: 81.1 vs 84.3.
            // force_kv_waves 4 / 8 (forced plan 23) picks one.
            long blocks256 = 0;
            for (int i = 0; i < n; ++i) blocks256 += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + 255) / 256);
            const long rounds8 = (blocks256 + 255) / 256;
            const int nw = (force_q_waves == kForceStream && (force_kv_waves == 4 || force_kv_waves == 8))
                               ? force_kv_waves
                               : (4 * (256 * rounds8 - blocks256) <= 256 ? 8 : 4);
            p.q_waves = nw;  // items of 32·nw rows
            p.kv_waves = nw;  // (reported by the plan query)
            p.rows_per_wave = 32;
            p.stream = 1;
            for (int i = 0; i < n; ++i) {
                p.splits[i] = 1;
                p.tiles_per_split[i] = 1;
            }
            return p;
        }
        force_q_waves = 0;  // fp32 inputs: the planner's choice
    }
    // 16-row blocks first: a launch of at most 256 of them runs every block on its own CU. Under a
    // concurrency hint >= 2 (several streams of independent calls) a call takes 32-row blocks on
    // half the CUs instead (launch_direct: two-per-CU form from hint 3), so the streams overlap.
    if (force_q_waves == kForceDirect16 ||
        (force_q_waves == 0 && direct16_enabled() && concurrency_hint() < 2)) {
        const int dt = direct_tiles_for(calls, n, in, force_q_waves == kForceDirect16, 16);
        if (dt > 0) {
            p.q_waves = 1;
            p.kv_waves = 4;
            p.rows_per_wave = 16;
            p.direct_tiles = dt;
            for (int i = 0; i < n; ++i) {
                p.splits[i] = 1;
                p.tiles_per_split[i] = 1;
            }
            return p;
        }
        if (force_q_waves == kForceDirect16) force_q_waves = 0;  // not applicable: the planner's choice
    }
    if (force_q_waves == kForceDirect || force_q_waves == 0) {
        const int dt = direct_tiles_for(calls, n, in, force_q_waves == kForceDirect);
        if (dt > 0) {
            p.q_waves = 1;
            p.kv_waves = 8;
            p.rows_per_wave = 32;
            p.direct_tiles = dt;
            for (int i = 0; i < n; ++i) {
                p.splits[i] = 1;
                p.tiles_per_split[i] = 1;
            }
            return p;
        }
        if (force_q_waves == kForceDirect) force_q_waves = 0;  // not applicable: the planner's choice
    }
    // Forced shapes (test/bench hook): q_waves >= 10 selects 64-row waves (RB = 2) of q_waves - 10.
    int rb = force_q_waves >= 10 ? 2 : 1;
    int qw = force_q_waves >= 10 ? force_q_waves - 10 : force_q_waves, kw = force_kv_waves;
    if (!valid_shape(qw, kw, rb)) {
        rb = 1;
        long blocks128 = 0;
        for (int i = 0; i < n; ++i) blocks128 += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + 127) / 128);
        // (bench.py --sweep, profiles/r01/ring_plan_sweep.json; eager us per launch)
        if (blocks128 > 256) {
            // more than one round of 128-row blocks: 4 waves (48 KiB LDS, several workgroups per
            // CU) beat (4,2)'s 8 (96 KiB, one per CU): 1024^2 B=16 29.3 vs 33.1, 2048^2 B=8 51.5
            // vs 57.1, 1536^2 B=8 36.3 vs 40.8
            qw = 4;
            kw = 1;
        } else if (blocks128 > 128) {
            // one round of 128-row blocks: (4,2), no cross-WG split (1536^2 B=3 21.6 vs 29.0 for
            // the (2,2) split plans, B=4 22.6 vs 29.8; 1024^2 B=8 18.8 vs 19.6 for (4,1))
            qw = 4;
            kw = 2;
        } else {
            qw = 2;
            kw = 2;
            // A launch that does not fill the chip with 64-row blocks: one super-tile per split
            // (single-stage LDS ring, straight-line body) while the grid stays within one
            // residency round. First choice (1,8): 32 rows x 512 keys per workgroup (128 KiB
            // LDS, one workgroup per CU, <= 256 of them): half the splits of (2,4), so half the
            // partial round trip; else (2,4): 64 rows x 256 keys (72 KiB, two per CU, <= 512).
            long g64 = 0, wgs4 = 0, wgs8 = 0;
            bool fits4 = true, fits8 = true;
            for (int i = 0; i < n; ++i) {
                const long b = (long)calls[i].batch * calls[i].heads;
                const long g = b * ((calls[i].nq + 63) / 64);
                const long st4 = (calls[i].nkv + 255) / 256, st8 = (calls[i].nkv + 511) / 512;
                fits4 = fits4 && st4 <= kMaxSplits;
                fits8 = fits8 && st8 <= kMaxSplits;
                g64 += g;
                wgs4 += g * st4;
                wgs8 += b * ((calls[i].nq + 31) / 32) * st8;
            }
            if (g64 < 256 && fits8 && wgs8 <= 256) {
                qw = 1;
                kw = 8;
            } else if (g64 < 256 && fits4 && wgs4 <= 512) {
                kw = 4;
            }
        }
    }
    p.q_waves = qw;
    p.kv_waves = kw;
    p.rows_per_wave = 32 * rb;
    const int block_m = 32 * qw * rb;
    long groups = 0;
    for (int i = 0; i < n; ++i)
        groups += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + block_m - 1) / block_m);
    // splits: as many as keep the grid within one round of 256 workgroups (a second partial
    // round costs more than the split saves: 1536^2 B=1 (2,2) 3-way 19.1 vs 2-way 13.9 us)
    int want = force_splits > 0 ? force_splits : (int)std::max(1L, 256 / std::max(1L, groups));
    want = std::max(1, std::min(want, kMaxSplits));
    if (kw >= 4) {
        // single-super-tile shapes: every split must be exactly one super-tile (their LDS ring
        // has one stage); otherwise (too many keys, or no workspace for the partials) use (2,2).
        size_t off = 0;
        bool ok = true;
        for (int i = 0; i < n; ++i) {
            const int super_total = std::max(1, (calls[i].nkv + 64 * kw - 1) / (64 * kw));
            ok = ok && super_total <= kMaxSplits;
            p.splits[i] = super_total;
            p.tiles_per_split[i] = 1;
            p.ws_offset[i] = off;
            off += split_workspace_bytes(calls[i], super_total);
        }
        p.ws_needed = off;
        if (ok && off <= ws_bytes) return p;
        return plan_group(calls, n, ws_bytes, 2, 2, force_splits, in);
    }
    for (;;) {
        size_t off = 0;
        for (int i = 0; i < n; ++i) {
            const int super_total = std::max(1, (calls[i].nkv + 64 * kw - 1) / (64 * kw));
            const int w = std::min(want, super_total);
            p.tiles_per_split[i] = (super_total + w - 1) / w;
            p.splits[i] = (super_total + p.tiles_per_split[i] - 1) / p.tiles_per_split[i];
            p.ws_offset[i] = off;
            off += split_workspace_bytes(calls[i], p.splits[i]);
        }
        p.ws_needed = off;
        if (want <= 1 || off <= ws_bytes) break;
        --want;
    }
    return p;
}

LaunchPlan plan_call(const Call& c, size_t ws_bytes, int force_q_waves, int force_kv_waves, int force_splits,
                     InType in) {
    const GroupPlan g = plan_group(&c, 1, ws_bytes, force_q_waves, force_kv_waves, force_splits, in);
    LaunchPlan p{};
    p.q_waves = g.q_waves;
    p.kv_waves = g.kv_waves;
    p.rows_per_wave = g.rows_per_wave;
    p.splits = g.splits[0];
    p.tiles_per_split = g.tiles_per_split[0];
    p.ws_needed = g.ws_needed;
    p.direct_tiles = g.direct_tiles;
    p.stream = g.stream;
    return p;
}

// ---- Float boundary onto the single-pass kernels ----
// fp32 Q/K/V of launches the single-pass kernels take (as fp16) are rounded to fp16 (RNE, the
// reference's convert kernel …fp16in_fp32out.cu:706-804 without its padding) into the caller's
// workspace by one elementwise launch, then run there; the LDS-ring kernel converts on load instead.
namespace {
constexpr int kConvMax = 3 * kMaxCalls;
struct ConvArgs {
    const float* src[kConvMax];
    f16* dst[kConvMax];
    unsigned end8[kConvMax];  // prefix sums of each tensor's element count / 8
    int count;
};

__global__ __launch_bounds__(256) void convert_f32_f16_kernel(ConvArgs c) {
    const unsigned g = blockIdx.x * 256u + threadIdx.x;
    int t = 0;
#pragma unroll
    for (int i = 0; i < kConvMax - 1; ++i) t += (int)((i < c.count - 1) & (g >= c.end8[i]));
    if (g >= c.end8[t]) return;
    const unsigned idx = g - (t ? c.end8[t - 1] : 0u);
    const f32x4* s = reinterpret_cast<const f32x4*>(c.src[t]) + 2 * (size_t)idx;
    const f32x4 lo = s[0], hi = s[1];
    const f16x4 a = __builtin_convertvector(lo, f16x4), b = __builtin_convertvector(hi, f16x4);
    reinterpret_cast<f16x8*>(c.dst[t])[idx] = f16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

bool f32_convert_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("MHA_HD64_F32_CONVERT");
        return !(e && e[0] == '0');
    }();
    return on;
}
// fp32 inputs rounded inside the 16-row kernel (one launch) where its one-pass forms apply
// (MHA_HD64_F32_INKERNEL=0 or set_f32_inkernel(0): the convert launch + fp16 kernel instead)
std::atomic<int> g_f32_inkernel{-1};
bool f32_inkernel_enabled() {
    int v = g_f32_inkernel.load();
    if (v < 0) {
        const char* e = std::getenv("MHA_HD64_F32_INKERNEL");
        int expect = -1;
        g_f32_inkernel.compare_exchange_strong(expect, (e && e[0] == '0') ? 0 : (e && e[0] == '2') ? 2 : 1);
        v = g_f32_inkernel.load();
    }
    return v >= 1;
}
// 2 (MHA_HD64_F32_INKERNEL=2 / set_f32_inkernel(2)): the two-pass forms (1024 < nkv <= 2048) round
// fp32 in the kernel too. Diagnostic: measured slower than convert + fp16 kernel.
bool f32_inkernel_two_pass() { return f32_inkernel_enabled() && g_f32_inkernel.load() == 2; }
}  // namespace

void set_f32_inkernel(int enable) { g_f32_inkernel.store(enable <= 0 ? 0 : enable >= 2 ? 2 : 1); }
int set_stream_mode(int mode) {
    const int prev = stream_env();
    g_stream_mode.store(mode ? 1 : 0);
    return prev;
}

static hipError_t launch_group_chunk(const Call* calls, int n, InType in, OutType out, void* workspace,
                                     size_t ws_bytes, hipStream_t stream, int force_q_waves, int force_kv_waves,
                                     int force_splits, int phase_mask);

// Whether an fp32-input launch whose fp16 plan is p16 takes the convert launch + that fp16 kernel
// (true) or the ring kernel rounding fp32 on load (false). The 32-row single-pass kernel after a
// convert loses to the ring kernel past one round of its blocks and at short key ranges, where
// the ring kernel's 128-row blocks share each K/V tile over four query waves (tools/f32_routes.py,
// profiles/r03/f32_routes.jsonl, us per launch, convert + 32-row kernel vs ring: 4x4x1024^2 16.4
// vs 13.9, 4x4x512^2 8.7 vs 7.6; kept: 2x4x1024^2 10.4 vs 12.8, 2x4x2048^2 22.4 vs 22.1).
static bool f32_convert_route(const Call* calls, int n, const GroupPlan& p16) {
    if (p16.stream) return true;
    if (p16.direct_tiles == 0) return false;
    if (p16.rows_per_wave == 16) return true;  // the 16-row kernel's two-pass forms (nkv > 1024)
    long blocks = 0;
    int max_nkv = 0;
    for (int i = 0; i < n; ++i) {
        blocks += (long)calls[i].batch * calls[i].heads * ((calls[i].nq + 31) / 32);
        max_nkv = std::max(max_nkv, calls[i].nkv);
    }
    return blocks <= 256 && max_nkv > 512;
}

// The convert + single-pass form of an fp32-input launch, or hipErrorNotSupported when it does
// not apply (not the planner's choice, no single-pass plan for these shapes, workspace too small).
static hipError_t launch_f32_via_f16(const Call* calls, int n, OutType out, void* workspace, size_t ws_bytes,
                                     hipStream_t stream, int phase_mask) {
    if (!f32_convert_enabled() || !workspace) return hipErrorNotSupported;
    const GroupPlan p16 = plan_group(calls, n, 0, 0, 0, 0, InType::F16);
    if (!f32_convert_route(calls, n, p16)) return hipErrorNotSupported;
    Call c16[kMaxCalls];
    ConvArgs cv{};
    size_t off = 0;
    unsigned total8 = 0;
    char* ws = reinterpret_cast<char*>(workspace);
    for (int i = 0; i < n; ++i) {
        c16[i] = calls[i];
        if (calls[i].nq <= 0 || calls[i].batch <= 0 || calls[i].heads <= 0) continue;
        const size_t bh = (size_t)calls[i].batch * calls[i].heads;
        const size_t elems[3] = {bh * calls[i].nq * kHeadDim, bh * calls[i].nkv * kHeadDim,
                                 bh * calls[i].nkv * kHeadDim};
        const void* src[3] = {calls[i].q, calls[i].k, calls[i].v};
        const void** dstp[3] = {&c16[i].q, &c16[i].k, &c16[i].v};
        for (int j = 0; j < 3; ++j) {
            const size_t bytes = align256(elems[j] * sizeof(f16));
            if (off + bytes > ws_bytes) return hipErrorNotSupported;
            total8 += (unsigned)(elems[j] / 8);
            cv.src[cv.count] = reinterpret_cast<const float*>(src[j]);
            cv.dst[cv.count] = reinterpret_cast<f16*>(ws + off);
            cv.end8[cv.count] = total8;
            ++cv.count;
            *dstp[j] = ws + off;
            off += bytes;
        }
    }
    if (total8 > 0 && (phase_mask & 1)) {
        hipLaunchKernelGGL(convert_f32_f16_kernel, dim3((total8 + 255) / 256), dim3(256), 0, stream, cv);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_group_chunk(c16, n, InType::F16, out, nullptr, 0, stream, 0, 0, 0, phase_mask);
}

static hipError_t launch_group_chunk(const Call* calls, int n, InType in, OutType out, void* workspace,
                                     size_t ws_bytes, hipStream_t stream, int force_q_waves, int force_kv_waves,
                                     int force_splits, int phase_mask) {
    bool in32_direct = false;  // fp32 inputs into the 16-row kernel's one-pass forms
    GroupPlan p{};
    if (in == InType::F32 && force_q_waves == 0 && force_kv_waves == 0 && force_splits == 0) {
        if (f32_inkernel_enabled() && f32_convert_enabled()) {
            const GroupPlan p16 = plan_group(calls, n, 0, 0, 0, 0, InType::F16);
            // one-pass forms only (nkv <= 1024): the two-pass form rounding fp32 in the kernel
            // measured slower than convert + fp16 kernel (1x4x1024x2048 11.32 vs 10.75 us,
            // 512x1536 9.78 vs 9.24; profiles/r02/float_inkernel.jsonl)
            in32_direct = p16.direct_tiles > 0 && p16.direct_tiles <= (f32_inkernel_two_pass() ? 4 : 2) &&
                          p16.rows_per_wave == 16;
            if (in32_direct) p = p16;
        }
        if (!in32_direct) {
            const hipError_t e = launch_f32_via_f16(calls, n, out, workspace, ws_bytes, stream, phase_mask);
            if (e != hipErrorNotSupported) return e;
        }
    }
    if (!in32_direct) p = plan_group(calls, n, workspace ? ws_bytes : 0, force_q_waves, force_kv_waves, force_splits, in);
    FwdArgs a{};
    CombineArgs cb{};
    a.stamps = g_stamps;
    int blocks = 0, n_live = 0;
    bool any_split = false;
    for (int i = 0; i < n; ++i) {
        const Call& c = calls[i];
        if (c.nq <= 0 || c.batch <= 0 || c.heads <= 0) continue;  // nothing to compute
        CallArgs& ca = a.c[n_live];
        ca.q = c.q;
        ca.k = c.k;
        ca.v = c.v;
        ca.o = c.o;
        ca.nq = c.nq;
        ca.nkv = c.nkv;
        ca.splits = p.splits[i];
        ca.tiles_per_split = p.tiles_per_split[i];
        ca.bh = c.batch * c.heads;
        const int block_m = p.rows_per_wave == 16 ? 16 : 32 * p.q_waves * (p.rows_per_wave / 32);
        ca.qtiles = (c.nq + block_m - 1) / block_m;
        ca.block_begin = blocks;
        if (ca.splits > 1) {
            const size_t rows = (size_t)ca.bh * ca.splits * c.nq;
            char* base = reinterpret_cast<char*>(workspace) + p.ws_offset[i];
            ca.part_o = base;
            ca.part_ml = reinterpret_cast<float2*>(base + align256(rows * kHeadDim * sizeof(float)));
            any_split = true;
        }
        CombineCall& cc = cb.c[n_live];
        cc.part_o = ca.part_o;
        cc.part_ml = ca.part_ml;
        cc.out = c.o;
        cc.nq = c.nq;
        cc.splits = ca.splits;
        cc.qtiles = ca.qtiles;
        blocks += ca.qtiles * ca.bh * ca.splits;
        ++n_live;
    }
    if (n_live == 0) return hipSuccess;
    a.n_calls = n_live;
    a.total_blocks = blocks;
    const int rbw = p.rows_per_wave / 32;
    if (p.stream) {  // persistent streaming kernel: no split, no workspace
        g_last_combine = 0;
        if (!(phase_mask & 1)) return hipSuccess;
        return launch_stream(a, p.q_waves, out == OutType::F32, stream);
    }
    if (p.direct_tiles > 0) {  // single-pass kernel: no split, no workspace
        g_last_combine = 0;
        if (!(phase_mask & 1)) return hipSuccess;
        return p.rows_per_wave == 16 ? launch_direct16(a, blocks, p.direct_tiles, out == OutType::F32, stream, in32_direct)
                                     : launch_direct(a, blocks, p.direct_tiles, out == OutType::F32, stream);
    }
    // Split calls combine inside the main launch when a ticket array is available (phase_mask 3,
    // the production form); otherwise (or MHA_HD64_FUSED_COMBINE=0) in the combine kernel.
    if (any_split && (phase_mask & 3) == 3 && fused_enabled()) a.tickets = tickets_for(stream, blocks);
    g_last_combine = !any_split ? 0 : (a.tickets ? 1 : 2);
    hipError_t e = hipSuccess;
    if (phase_mask & 1) {
        if (in == InType::F16) {
            e = (out == OutType::F16) ? launch_fwd_shape<f16, f16>(a, blocks, p.q_waves, p.kv_waves, rbw, stream)
                                      : launch_fwd_shape<f16, float>(a, blocks, p.q_waves, p.kv_waves, rbw, stream);
        } else {
            e = (out == OutType::F16) ? launch_fwd_shape<float, f16>(a, blocks, p.q_waves, p.kv_waves, rbw, stream)
                                      : launch_fwd_shape<float, float>(a, blocks, p.q_waves, p.kv_waves, rbw, stream);
        }
    }
    if (e != hipSuccess || !any_split || !(phase_mask & 2) || a.tickets) return e;
    // Combine grid: for every XCD x, the groups (of calls that split) whose first split block
    // ran on x (same bijective order as the main kernel), 16 rows per block.
    cb.n_calls = n_live;
    const int block_m = 32 * p.q_waves * rbw;
    cb.block_m_log2 = block_m == 32 ? 5 : (block_m == 64 ? 6 : 7);
    auto xb = [&](int xx) {
        const int q8 = blocks >> 3, r8 = blocks & 7;
        return xx < r8 ? xx * (q8 + 1) : r8 * (q8 + 1) + (xx - r8) * q8;
    };
    auto fg = [](int j, int b0, int S) { return j <= b0 ? 0 : (j - b0 + S - 1) / S; };
    int per_xcd = 0;
    for (int x = 0; x < 8; ++x) {
        const int jlo = xb(x), jhi = xb(x + 1);
        int kk = 0;
        for (int i = 0; i < n_live; ++i) {
            cb.kbeg[x][i] = kk;
            const CallArgs& ca = a.c[i];
            if (ca.splits <= 1) {
                cb.gbeg[x][i] = 0;
                continue;
            }
            const int groups = ca.qtiles * ca.bh;
            const int glo = std::min(groups, fg(jlo, ca.block_begin, ca.splits));
            const int ghi = std::min(groups, fg(jhi, ca.block_begin, ca.splits));
            cb.gbeg[x][i] = glo;
            kk += (ghi - glo) * block_m / 16;
        }
        for (int i = n_live; i <= kMaxCalls; ++i) cb.kbeg[x][i] = kk;
        per_xcd = std::max(per_xcd, kk);
    }
    cb.per_xcd = std::max(1, per_xcd);
    cb.main_blocks = blocks;
    cb.groups0 = a.c[0].qtiles * a.c[0].bh;
    return (out == OutType::F16) ? launch_combine<f16>(cb, stream) : launch_combine<float>(cb, stream);
}

hipError_t launch_group(const Call* calls, int n, InType in, OutType out, void* workspace, size_t ws_bytes,
                        hipStream_t stream, int force_q_waves, int force_kv_waves, int force_splits,
                        int phase_mask) {
    // Chunks of kMaxCalls calls share one launch; each chunk reuses the workspace (stream order).
    for (int i = 0; i < n; i += kMaxCalls) {
        const hipError_t e = launch_group_chunk(calls + i, std::min(kMaxCalls, n - i), in, out, workspace, ws_bytes,
                                                stream, force_q_waves, force_kv_waves, force_splits, phase_mask);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// What launch_group_chunk uses for one chunk (same decisions, in the same order).
static size_t chunk_workspace_bytes(const Call* calls, int n, InType in) {
    if (in == InType::F32 && f32_convert_enabled()) {
        const GroupPlan p16 = plan_group(calls, n, 0, 0, 0, 0, InType::F16);
        const bool in32_direct = f32_inkernel_enabled() && p16.direct_tiles > 0 &&
                                 p16.direct_tiles <= (f32_inkernel_two_pass() ? 4 : 2) && p16.rows_per_wave == 16;
        if (in32_direct) return 0;
        if (f32_convert_route(calls, n, p16)) {  // convert launch into the workspace, then the fp16 kernel
            size_t off = 0;
            for (int i = 0; i < n; ++i) {
                if (calls[i].nq <= 0 || calls[i].batch <= 0 || calls[i].heads <= 0) continue;
                const size_t bh = (size_t)calls[i].batch * calls[i].heads;
                off += align256(bh * calls[i].nq * kHeadDim * sizeof(f16)) +
                       2 * align256(bh * calls[i].nkv * kHeadDim * sizeof(f16));
            }
            return off;
        }
    }
    return plan_group(calls, n, (size_t)-1, 0, 0, 0, in).ws_needed;
}

size_t group_workspace_bytes(const Call* calls, int n, InType in) {
    size_t need = 0;
    for (int i = 0; i < n; i += kMaxCalls)
        need = std::max(need, chunk_workspace_bytes(calls + i, std::min(kMaxCalls, n - i), in));
    return need;
}

hipError_t launch_attention(const Call& c, InType in, OutType out, void* workspace, size_t ws_bytes,
                            hipStream_t stream, int force_q_waves, int force_kv_waves, int force_splits,
                            int phase_mask) {
    return launch_group_chunk(&c, 1, in, out, workspace, ws_bytes, stream, force_q_waves, force_kv_waves,
                              force_splits, phase_mask);
}

}  // namespace mha_hd64
