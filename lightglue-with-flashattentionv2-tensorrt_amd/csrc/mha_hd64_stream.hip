// mha_hd64_stream.hip — persistent streaming FlashAttention forward, head_dim = 64, for gfx950
// (MI355X): the throughput form of the MHAHeadDim64 operator.
//
// Same operator as mha_hd64_kernels.hip (O = softmax(Q·Kᵀ·0.125)·V per (batch, head); reference
// lightglue_attention_plugin/attention_headdim_64_fp16in_fp16out.cu:253-733 and
// …fp16in_fp32out.cu:253-703, oracle lightglue_pytorch_no_plugin/lightglue.py:75-85) for launches
// that carry more 128-row query blocks than one round of the chip holds: batched image-pair
// streams (many calls stacked in the batch dimension) and grouped matcher layers.
//
// Where the LDS-ring kernel pays per workgroup (Q + first super-tile burst, key-wave merge,
// output burst, dispatch), this kernel pays per launch:
//  * item = (call, batch·head, 128-row query block) with ALL of its keys. Workgroup = 4 waves,
//    one per SIMD, each wave 32 query rows; 80 KiB LDS and <= 256 VGPRs, so two workgroups share
//    a CU and every SIMD runs one wave of each: one wave's softmax (vector and transcendental
//    pipes) beside the other's MFMAs, with no barrier between the two;
//  * persistent: grid = min(items, 512); the workgroups of one XCD walk that XCD's contiguous
//    share of the items (consecutive query blocks of one head: its K/V is read through one L2)
//    with stride;
//  * K and V stream by LDS-DMA (`buffer_load_dwordx4 … lds`, 1 KiB per wave instruction, the XOR
//    swizzles applied on the source address) into a 4-slot ring of 64-key tiles, three tiles ahead
//    of the compute, CONTINUOUSLY across item seams: the loader moves on to the next item's keys
//    while the current item finishes. The next item's Q arrives by DMA in a 16 KiB region during
//    the current item's first step; its first QKᵀ runs in the current item's last step. An item
//    seam costs the output stores and a few register moves; nothing waits for a fresh burst;
//  * per step t (64 keys, one barrier), deferred P·V: the matrix pipe runs QKᵀ of tile t+1
//    (v_mfma_f32_32x32x16_f16, Sᵀ = K·Qᵀ so a lane holds one query) and then Oᵀ += Vᵀ·Pᵀ of tile
//    t−1 (P packed to fp16 in the previous step, Vᵀ by ds_read_b64_tr_b16) + its row sums, while
//    the vector pipes run exp2 and the fp16 pack of tile t and the row max of tile t+1; so no
//    MFMA waits for the exponentials of its own step. The ring slot of every operand is a
//    compile-time constant (the loop body is unrolled over the 4 slots);
//  * the running max rides in the QKᵀ chains' C operand (a register block holding −m, read, never
//    written: the MFMA emits s·c − m), so a probability is one v_exp_f32 and there is no bias
//    k-step; lazy rescale (threshold 8, log2 units) as the other kernels;
//  * epilogue per item: 1/l, fp16 pack, v_permlane32_swap pairs → 16-B row-segment stores
//    (cdna_hip_programming.md T21); rows past nq and keys past nkv are bounded by the buffer
//    descriptors (no pad / unpad).
// The DMA is inline asm with hand-counted waits (lds_dma16, mha_hd64_device.h).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

// Diagnostic build (-DMHA_STREAM_STAMPS, tools/stream_stamps.py): per wave, the s_memtime cycles
// of every step summed by segment (0 refill issue, 1 decision / seam, 2 phase A issue, 3 phase B
// issue, 4 the counted DMA wait, 5 the barrier) and the step count, written at exit to
// a.stamps[(blockIdx.x * NW + wave) * 16 + k]; k = 8..11: s_memtime / s_memrealtime (100 MHz) at
// kernel entry and exit (the in-kernel clock, MI355X_MICROARCH.md DVFS item 6). The stamps return through lgkmcnt and are summed after
// the next barrier, where nothing else is outstanding on that counter.
#ifdef MHA_STREAM_STAMPS
#define SSTAMP(i) asm volatile("s_memtime %0" : "=s"(ck_[i])::"memory")
#else
#define SSTAMP(i) \
    do {          \
    } while (0)
#endif

// Ablation switches (diagnostic builds only; results are wrong by construction): bit 0 no K/V
// DMA in the steady loop, 1 no exponentials, 2 no step barrier, 3 no K/V fragment reads in the
// loop (registers stand in), 4 no P packing / row-max vector work.
#ifndef MHA_STREAM_ABL
#define MHA_STREAM_ABL 0
#endif

#ifndef MHA_STREAM_FENCE
#define MHA_STREAM_FENCE 1  // 0: no scheduling fences in the step (the compiler interleaves freely)
#endif
#define STREAM_FENCE()                                          \
    do {                                                        \
        if (MHA_STREAM_FENCE) __builtin_amdgcn_sched_barrier(0); \
    } while (0)

#ifndef MHA_STREAM_PRIO
#define MHA_STREAM_PRIO 0  // A/B hook: s_setprio 1 for the odd workgroups
#endif

namespace mha_hd64 {
namespace {

// NW = waves per workgroup: 4 (128-row items, two workgroups per CU) or 8 (256-row items, one
// per CU: the two waves of a SIMD share one K/V stream, half the DMA pieces per wave and step)
constexpr int kStreamSlot = 2 * kTileBytes;           // K image, then V image
template <int NW> constexpr int stream_rows() { return 32 * NW; }
// ring slots (80 KiB LDS with the Q region: two workgroups per CU); the refill of a step lands
// before that step's barrier (one step ahead of its first read)
template <int NW> constexpr int stream_slots() { return 4; }
template <int NW> constexpr int stream_lds() { return stream_slots<NW>() * kStreamSlot + stream_rows<NW>() * 128; }
template <int NW> constexpr int stream_max_grid() { return NW == 8 ? 256 : 512; }

// Call ci's arguments, field by field with compile-time indices (a runtime index into the
// kernarg table would copy it to scratch).
template <bool MULTI>
__device__ __forceinline__ int stream_call(const FwdArgs& a, int j) {
    int ci = 0;
    if constexpr (MULTI) {
#pragma unroll
        for (int i = 1; i < kMaxCalls; ++i) ci += (int)((i < a.n_calls) & (j >= a.c[i].block_begin));
    }
    return ci;
}
#define MHA_SEL(field)                                                                  \
    [&]() {                                                                             \
        auto v_ = a.c[0].field;                                                         \
        if constexpr (MULTI) {                                                          \
            _Pragma("unroll") for (int i_ = 1; i_ < kMaxCalls; ++i_) if (ci == i_) v_ = a.c[i_].field; \
        }                                                                               \
        return v_;                                                                      \
    }()

// One item's scalar description (batch·head offsets applied).
struct StreamItem {
    const char* q;
    const char* k;
    const char* v;
    char* o;
    int nq;
    int nkv;
    int q0;  // first query row of the block
};

template <bool MULTI, int OSZ, int NW>
__device__ __forceinline__ StreamItem stream_item(const FwdArgs& a, int j) {
    const int ci = stream_call<MULTI>(a, j);
    const int nq = MHA_SEL(nq), nkv = MHA_SEL(nkv), qtiles = MHA_SEL(qtiles);
    const int jl = j - MHA_SEL(block_begin);
    const int bh = jl / qtiles, qtile = jl - bh * qtiles;
    StreamItem it;
    it.q = reinterpret_cast<const char*>(MHA_SEL(q)) + (size_t)bh * nq * (kHeadDim * 2);
    it.k = reinterpret_cast<const char*>(MHA_SEL(k)) + (size_t)bh * nkv * (kHeadDim * 2);
    it.v = reinterpret_cast<const char*>(MHA_SEL(v)) + (size_t)bh * nkv * (kHeadDim * 2);
    it.o = reinterpret_cast<char*>(MHA_SEL(o)) + (size_t)bh * nq * (kHeadDim * OSZ);
    it.nq = nq;
    it.nkv = nkv;
    it.q0 = qtile * stream_rows<NW>();
    return it;
}

// Buffer descriptor from wave-uniform values, made provably uniform (T20): every buffer op on it
// keeps its descriptor in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return make_rsrc((const void*)(((unsigned long long)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
}

// Every VMEM op of the wave except the N youngest (the tile pieces issued this step) done.
template <int N>
__device__ __forceinline__ void stream_wait() {
    static_assert(N == 0 || N == 2 || N == 4, "pieces per wave and tile");
    if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// fp16 Q scaled by 0.125·log2(e): each half rounded once from the fp32 product (v_fma_mix), the
// same bits as the other kernels' (f16)((float)q * kScaleLog2).
__device__ __forceinline__ f16x8 stream_scale_q(f16x8 raw) {
    const u32x4 in = __builtin_bit_cast(u32x4, raw);
    const float sc = kScaleLog2;
    u32x4 outv;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "=&v"(outv[w])
            : "v"(in[w]), "v"(sc));
    return __builtin_bit_cast(f16x8, outv);
}

typedef f16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f16x2 f16x2_pack(float a, float b) { return f16x2{(f16)a, (f16)b}; }

// Scores and row max of one 64-key tile (two 32-key halves): the state that rotates per step.
struct StreamScores {
    f32x16 s0, s1;  // Sᵀ halves: keys 0..31 / 32..63 of the tile, query = lane % 32
    float mx;       // row max (both half-waves), relative to the running max (absolute on a
                    // block's first tile)
    bool rs;        // some query of the wave exceeds the running max by > kRescaleThr (wave-uniform)
};

template <typename TOut, bool MULTI, int NW>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 1 : 2) void mha_hd64_stream_kernel(FwdArgs a) {
    constexpr int OSZ = (int)sizeof(TOut);
    constexpr int PW = 16 / NW;               // DMA pieces per wave and tile (16 KiB of K and V)
    constexpr int NS = stream_slots<NW>();    // ring slots
    constexpr int QOFF = NS * kStreamSlot;    // Q region
    constexpr int WAITN = 0;                  // the step's own refill lands before its barrier
    __shared__ __attribute__((aligned(1024))) char smem[stream_lds<NW>()];
    lds_char* const lds = (lds_char*)smem;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave

#ifdef MHA_STREAM_STAMPS
    unsigned long long ck_entry[2];
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_entry[0]), "=s"(ck_entry[1])::"memory");
#endif
    // This workgroup's items: XCD x = blockIdx % 8 owns the contiguous range [jb, je) of the
    // T items (the other kernels' XCD-aware split); its G workgroups take every G-th item from
    // their local index.
    const int T = a.total_blocks;
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8);
    const int je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    int j = jb + loc;
    if (j >= je) return;  // (grid <= items: never)
#if MHA_STREAM_PRIO
    if constexpr (NW == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // (wave is readfirstlane'd: a scalar branch)
    } else {
        // 1: odd workgroups; 2: the second half of the grid (the second workgroup dispatched to a CU)
        if (MHA_STREAM_PRIO == 1 ? (__builtin_amdgcn_readfirstlane(blockIdx.x) & 1)
                                 : (__builtin_amdgcn_readfirstlane(blockIdx.x) >= gridDim.x / 2))
            __builtin_amdgcn_s_setprio(1);
    }
#endif

    // ---- per-lane constant addressing ----
    // K image (A operand of Sᵀ = K·Qᵀ): dim step s, half-wave hh reads chunk 2s + hh of key row r
    // (keys 0..31) and r + 32 (keys 32..63, + 4 KiB: the swizzle repeats every 16 rows). The Q
    // region has the same image (row = query).
    unsigned k_addr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = (unsigned)k_off(r, 2 * s + hh);
    const unsigned q_addr = (unsigned)(QOFF + 32 * wave * 128);  // + k_addr[s]
    // V image (A operand of Oᵀ = Vᵀ·Pᵀ via ds_read_b64_tr_b16): as the LDS-ring kernel's.
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const unsigned v_addr0 = (unsigned)(v_lane + 64 * vb + kTileBytes);        // dims 0..31
    const unsigned v_addr1 = (unsigned)(v_lane + 64 * (1 - vb) + kTileBytes);  // dims 32..63
    // DMA: piece p of a tile = rows 8p..8p+7, lane L writes LDS chunk L&7 of row 8p + L/8 and reads
    // the source chunk the image puts there. Wave w moves the K and V pieces w (and w + 4 with 4
    // waves) of every tile and Q pieces w + NW·i (the K swizzle repeats every 16 rows: one lane
    // offset per wave).
    const unsigned dma_k = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7)) << 4));
    const unsigned dma_v = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ (((lane >> 4) & 1) << 2)) << 4));
    // Row sums on the matrix pipe (the LDS-ring kernel's selector): l_acc = sel · P per k-step.
    const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
    const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};

    // ---- loader: the tile stream over this workgroup's items ----
    int l_j = j, l_t = 0, l_nt;
    __amdgpu_buffer_rsrc_t k_l, v_l;
    auto loader_item = [&](int jj) {
        const StreamItem it = stream_item<MULTI, OSZ, NW>(a, jj);
        l_nt = (it.nkv + kTileKV - 1) / kTileKV;
        k_l = stream_rsrc(it.k, (unsigned)it.nkv * kHeadDim * 2);
        v_l = stream_rsrc(it.v, (unsigned)it.nkv * kHeadDim * 2);
    };
    loader_item(j);
    // piece i of the loader's tile into `slot`: NW = 4: K w, K w+4, V w, V w+4; NW = 8: K w, V w
    const unsigned m0w = (unsigned)__builtin_amdgcn_readfirstlane(lds0 + (unsigned)wave * 1024u);
    const unsigned sow = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wave * 1024u);
    auto issue_piece = [&](int slot, int i) {
        const int kv = i / (PW / 2), hi = i % (PW / 2);  // V image?, second row block?
        const unsigned m = m0w + (unsigned)(slot * kStreamSlot + kv * kTileBytes + hi * 4096);
        const unsigned so = (unsigned)l_t * kTileBytes + sow + (unsigned)(hi * 4096);
        lds_dma16(m, kv ? dma_v : dma_k, kv ? v_l : k_l, so);
    };
    // the cursor moves on to the stream's next tile; past the last item the pieces read from an
    // empty descriptor (zeros into a slot nobody reads), so every step issues exactly PW and the
    // counted waits stay exact
    auto advance = [&]() {
        if (++l_t == l_nt) {
            l_t = 0;
            l_j += G;
            if (l_j < je) {
                loader_item(l_j);
            } else {
                l_nt = 1 << 20;
                k_l = stream_rsrc(nullptr, 0u);
                v_l = k_l;
            }
        }
    };
    auto issue = [&](int slot) {
#pragma unroll
        for (int i = 0; i < PW; ++i) issue_piece(slot, i);
        advance();
    };
    // Q rows of item `it` into the Q region (pieces w + NW·i, i = 0..3, of this wave)
    auto issue_q_piece = [&](const StreamItem& it, int i) {
        const __amdgpu_buffer_rsrc_t q_rs = stream_rsrc(it.q, (unsigned)it.nq * kHeadDim * 2);
        const unsigned m = m0w + (unsigned)QOFF + 1024u * NW * i;
        const unsigned so = (unsigned)it.q0 * 128u + sow + 1024u * NW * i;
        lds_dma16(m, dma_k, q_rs, so);
    };
    auto issue_q = [&](const StreamItem& it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) issue_q_piece(it, i);
    };
    // Q fragments of this wave's rows from the Q region, scaled
    f16x8 qf[4];
    // (returns the mask of the wave's queries with a non-finite Q, whose fragments it zeroes)
    auto read_q = [&]() -> unsigned {
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = stream_scale_q(lds_read16(lds, q_addr + k_addr[s]));
        return q_nonfinite_fix(qf);
    };

    // ---- compute state ----
    StreamItem cur = stream_item<MULTI, OSZ, NW>(a, j);
    int nt = (cur.nkv + kTileKV - 1) / kTileKV;
    bool has_next = j + G < je;
    StreamItem nxt = stream_item<MULTI, OSZ, NW>(a, has_next ? j + G : j);
    StreamItem prv = cur;       // the item whose last PV is pending (stored after the next first step)
    bool has_prv = false;
    unsigned qbad = 0, qbad_next = 0, qbad_prv = 0;  // non-finite query masks (current / next / previous item)
    int t = 0;                  // tile of the current item
    f32x16 cm;                  // -m (the QKᵀ chains' C operand)
    f32x16 o0 = {}, o1 = {};    // Oᵀ: dims 0..31 / 32..63, query on the lane
    f32x4 l_acc = {0.f, 0.f, 0.f, 0.f};  // row sums (every element: the lane's query)
    StreamScores sA, sB;
    f16x8 pA[2][2], pB[2][2];   // P (fp16) of a tile: B operand of k-step (jj, ss) of Oᵀ = Vᵀ·Pᵀ
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) pB[jj][ss] = f16x8{};  // the first step's "previous" P

    auto mask_tile = [&](StreamScores& s, int lim) {  // keys >= lim of the tile -> -inf
        const int l4 = lim - 4 * hh;  // element i holds key (i & 3) + 8 (i >> 2) + 4 hh (+ 32 in s1)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int key = (i & 3) + 8 * (i >> 2);
            s.s0[i] = key >= l4 ? -INFINITY : s.s0[i];
            s.s1[i] = key + 32 >= l4 ? -INFINITY : s.s1[i];
        }
    };
    // V fragments (A operand of Oᵀ = Vᵀ·Pᵀ) of the tile in `slot`, key half jj
    f16x8 vfa[2][2], vfb[2][2];
    auto read_v = [&](int slot, int jj) {
        if (MHA_STREAM_ABL & 8) {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                vfa[jj][ss] = qf[(jj + ss) & 3];
                vfb[jj][ss] = qf[(jj + ss + 1) & 3];
            }
            return;
        }
        const unsigned vbase = (unsigned)slot * kStreamSlot;
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            const unsigned rowc = vbase + 128u * (32 * jj + 16 * ss);
            vfa[jj][ss] = cat8(tr_read(lds, v_addr0 + rowc), tr_read(lds, v_addr0 + rowc + 8 * 128));
            vfb[jj][ss] = cat8(tr_read(lds, v_addr1 + rowc), tr_read(lds, v_addr1 + rowc + 8 * 128));
        }
    };
    auto pv_mfma = [&](int k, const f16x8 (&pv)[2][2], int part) {  // k-step k: 0 o0, 1 o1, 2 row sums
        const int jj = k >> 1, ss = k & 1;
        if (part == 0) o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], pv[jj][ss], o0, 0, 0, 0);
        else if (part == 1) o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], pv[jj][ss], o1, 0, 0, 0);
        else l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, pv[jj][ss], l_acc, 0, 0, 0);
    };
    // O = Oᵀ / l of item `it` (rows past nq: dropped by the descriptor)
    auto epilogue = [&](const StreamItem& it, unsigned qbad_it) {
        const float inv = inv_or_nan(l_acc[0], qbad_it, r);  // a non-finite query row: NaN
        const __amdgpu_buffer_rsrc_t o_rs = stream_rsrc(it.o, (unsigned)it.nq * kHeadDim * OSZ);
        const unsigned row = (unsigned)(it.q0 + 32 * wave + r);
        if constexpr (OSZ == 2) {
            // lane (query, hh) holds dims 8k + 4hh .. +3 of group k (o0: k 0..3, o1: 4..7);
            // v_permlane32_swap pairs (k, k+1) so each lane holds 8 consecutive dims (T21)
            u32x2 rk[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x16& o = k < 4 ? o0 : o1;
                const int b = 4 * (k & 3);
                const f16x4 h = f16x4{(f16)(o[b] * inv), (f16)(o[b + 1] * inv), (f16)(o[b + 2] * inv),
                                      (f16)(o[b + 3] * inv)};
                rk[k] = __builtin_bit_cast(u32x2, h);
            }
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
#pragma unroll
                for (int w = 0; w < 2; ++w) {
                    const auto sw = __builtin_amdgcn_permlane32_swap(rk[k][w], rk[k + 1][w], false, false);
                    rk[k][w] = sw[0];
                    rk[k + 1][w] = sw[1];
                }
                const u32x4 v = u32x4{rk[k][0], rk[k][1], rk[k + 1][0], rk[k + 1][1]};
                __builtin_amdgcn_raw_buffer_store_b128(v, o_rs, row * 128u + (unsigned)(8 * k + 8 * hh) * 2u, 0,
                                                       MHA_ST_AUX);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x16& o = k < 4 ? o0 : o1;
                const int b = 4 * (k & 3);
                const f32x4 v = f32x4{o[b] * inv, o[b + 1] * inv, o[b + 2] * inv, o[b + 3] * inv};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), o_rs,
                                                       row * 256u + (unsigned)(8 * k + 4 * hh) * 4u, 0, MHA_ST_AUX);
            }
        }
    };

    // prologue: Q of the first item and tiles 0 .. NS-3 of the stream, landed; the V image of slot
    // NS-1 zeroed: the first step's PV of "tile -1" (P = 0) reads it before any DMA fills it
    issue_q(cur);
#pragma unroll
    for (int i = 0; i < NS - 2; ++i) issue(i);
#pragma unroll
    for (unsigned off = (unsigned)tid * 16u; off < (unsigned)kTileBytes; off += 64u * NW * 16u)
        lds_write16(lds, (NS - 1) * kStreamSlot + kTileBytes + off, f16x8{});
    stream_wait<WAITN>();
    __builtin_amdgcn_s_barrier();
    qbad = read_q();
    {
        f16x8 kf[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            kf[2 * s] = lds_read16(lds, k_addr[s]);
            kf[2 * s + 1] = lds_read16(lds, k_addr[s] + 4096u);
        }
        const f32x16 zero = {};
        sA.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[0], qf[0], zero, 0, 0, 0);
        sA.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[1], qf[0], zero, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < 4; ++s) {
            sA.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s], qf[s], sA.s0, 0, 0, 0);
            sA.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + 1], qf[s], sA.s1, 0, 0, 0);
        }
        if (cur.nkv < kTileKV) mask_tile(sA, cur.nkv);
        sA.mx = xhalf_max(tree_max(sA.s0, sA.s1));
        sA.rs = false;
    }
    __builtin_amdgcn_s_barrier();  // every wave's Q reads done before step 0 refills the Q region
#ifdef MHA_STREAM_STAMPS
    unsigned long long ck_pro;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_pro)::"memory");
    unsigned long long ck_epi = 0;
    unsigned long long ck_[7] = {}, ck_sum[7] = {};
    bool ck_live = false;
#endif

    // One step (global tile g = tile t of the current item), deferred-PV pipeline: the matrix pipe
    // runs QKᵀ of tile t + 1 and Oᵀ += Vᵀ·Pᵀ of tile t - 1 (P from the last step, V still in its
    // slot) while the vector pipe exponentiates and packs tile t and takes the row max of tile t + 1:
    // no dependency between the step's MFMAs and its vector work, so every MFMA gap carries about
    // two exponentials and one other vector op. c: scores of tile t; n: of tile t + 1; pp: P of
    // tile t - 1 (consumed); pn: P of tile t (produced). Returns false once the workgroup is done.
    auto step = [&](auto slot_c, StreamScores& c, StreamScores& n, const f16x8 (&pp)[2][2], f16x8 (&pn)[2][2]) -> bool {
        // ring slots as compile-time constants (the loop is unrolled over the NS = 4 slots): every
        // LDS address folds into the instruction's offset field, every M0 into one scalar add
        constexpr int S = decltype(slot_c)::value;     // tile t
        constexpr int NSL = (S + 1) % NS;              // tile t + 1 (K)
        constexpr int VSL = (S + NS - 1) % NS;         // tile t - 1 (V)
        constexpr int FSL = (S + 2) % NS;              // refill: tile t + 2, into tile t - 2's slot
#ifdef MHA_STREAM_STAMPS
        if (ck_live) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(ck_[0]), "+s"(ck_[1]), "+s"(ck_[2]), "+s"(ck_[3]), "+s"(ck_[4]),
                         "+s"(ck_[5]), "+s"(ck_[6])::"memory");
            for (int i_ = 0; i_ < 6; ++i_) ck_sum[i_] += ck_[i_ + 1] - ck_[i_];
            ck_sum[6] += 1;
        }
        ck_live = true;
#endif
        SSTAMP(0);
        const bool first = t == 0;
        const bool last = t + 1 == nt;
        const bool seam = last && has_next;  // the next tile is the next item's first
        const int nlim = !last ? min(kTileKV, cur.nkv - kTileKV * (t + 1)) : min(kTileKV, nxt.nkv);

        // online-softmax decision for tile t. A rescale (rare) moves the max now for tile t and is
        // applied to O and l at the end of the step, after tile t - 1's PV (at the old max) is in.
        float alpha = 1.f;
        const bool rescale = !first && c.rs;
        if (first) {
            const float d = (c.mx < kEmptyMax) ? 0.f : c.mx;  // (a fully masked tile: m = 0)
            cm = splat16(-d);
            c.s0 -= d;
            c.s1 -= d;
        } else if (rescale) {  // wave-uniform
            const float d = fmaxf(c.mx, 0.f);
            alpha = __builtin_amdgcn_exp2f(-d);
            cm -= d;
            c.s0 -= d;
            c.s1 -= d;
        }
        if (seam) {  // the next item's Q (C = 0: its max is set at its first step)
            if (first) {  // a one-tile item: its successor's Q now, landed everywhere before the reads
                asm volatile("" ::: "memory");
                issue_q(nxt);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            qbad_next = read_q();
            cm = f32x16{};
        }
        if (first && !seam) issue_q(nxt);  // the next item's Q: the region is free since the last seam
        SSTAMP(1);

        constexpr unsigned kbase = (unsigned)NSL * kStreamSlot;
        f16x8 kf[8];
        auto read_k = [&](int s) {
            if (MHA_STREAM_ABL & 8) {
                kf[2 * s] = qf[s];
                kf[2 * s + 1] = qf[(s + 1) & 3];
                return;
            }
            kf[2 * s] = lds_read16(lds, kbase + k_addr[s]);
            kf[2 * s + 1] = lds_read16(lds, kbase + k_addr[s] + 4096u);
        };
        // (every exponential and pack is tied in place: the results are consumed only by the next
        // step, and the compiler would otherwise sink them to one burst where no MFMA runs)
        auto exp2 = [&](int e) {  // two exponentials of tile t: elements 2e, 2e + 1
            if (MHA_STREAM_ABL & 2) return;
            f32x16& x = e < 8 ? c.s0 : c.s1;
            const int u = (2 * e) & 15;
            x[u] = __builtin_amdgcn_exp2f(x[u]);
            x[u + 1] = __builtin_amdgcn_exp2f(x[u + 1]);
            float a0 = x[u], a1 = x[u + 1];
            asm volatile("" : "+v"(a0), "+v"(a1));
            x[u] = a0;
            x[u + 1] = a1;
        };
        auto cvt = [&](int g, int part) {  // P of k-step group g = (jj, ss): 2 of its 8 values
            const int jj = g >> 1, ss = g & 1;
            if (MHA_STREAM_ABL & 16) {
                if (part == 0) pn[jj][ss] = qf[g];
                return;
            }
            const f32x16& x = jj ? c.s1 : c.s0;
            unsigned w = __builtin_bit_cast(unsigned, f16x2_pack(x[8 * ss + 2 * part], x[8 * ss + 2 * part + 1]));
            asm volatile("" : "+v"(w));
            u32x4 pw = __builtin_bit_cast(u32x4, pn[jj][ss]);
            pw[part] = w;
            pn[jj][ss] = __builtin_bit_cast(f16x8, pw);
        };
        float mt[4];
        auto maxk = [&](int k) {  // partial row max of tile t + 1, k-step k
            const f32x16& x = k < 2 ? n.s0 : n.s1;
            if (MHA_STREAM_ABL & 16) {
                mt[k] = x[k];
                return;
            }
            const int b = 8 * (k & 1);
            const float u = max3f(x[b], x[b + 1], x[b + 2]);
            const float v = max3f(x[b + 3], x[b + 4], x[b + 5]);
            mt[k] = max3f(u, v, fmaxf(x[b + 6], x[b + 7]));
        };

        // QKᵀ(t + 1) MFMAs, each gap: two exponentials of tile t (+ a pack or an LDS read batch)
        SSTAMP(2);
        STREAM_FENCE();
        read_k(0);
        read_k(1);
        exp2(0);
        exp2(1);
        STREAM_FENCE();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int s = i >> 1;
            if ((i & 1) == 0) n.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i], qf[s], s == 0 ? cm : n.s0, 0, 0, 0);
            else n.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i], qf[s], s == 0 ? cm : n.s1, 0, 0, 0);
            exp2(2 + i);  // elements 4 .. 19
            if (i == 0) {
                read_k(2);
                read_k(3);
            }
            if (i == 3) read_v(VSL, 0);
            if (i == 5) read_v(VSL, 1);
            // the refill (tile t + 2) between the QKᵀ MFMAs: lands before this step's barrier
            if ((i & 1) == 0 && (i >> 1) < PW && !(MHA_STREAM_ABL & 1)) issue_piece(FSL, i >> 1);
            if (i >= 4) cvt(0, i - 4);  // P group (0,0) = elements 0..7
            STREAM_FENCE();
        }
        SSTAMP(3);
        // Oᵀ += Vᵀ·Pᵀ of tile t - 1 and its row sums, each gap: exponentials / packs of tile t, the
        // row max of tile t + 1, the refill's DMA pieces (~60+ issue cycles each)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pv_mfma(k, pp, 0);
            if (k < 3) exp2(10 + 2 * k);  // elements 20 .. 31 (with the next line)
            if (k == 0) cvt(1, 0);
            if (k == 1) cvt(1, 2);
            if (k == 2) cvt(2, 0);
            if (k == 3) cvt(2, 2);
            STREAM_FENCE();
            pv_mfma(k, pp, 1);
            if (k < 3) exp2(11 + 2 * k);
            if (k == 0) cvt(1, 1);
            if (k == 1) cvt(1, 3);
            if (k == 2) cvt(2, 1);
            if (k == 3) cvt(2, 3);
            maxk(k);
            STREAM_FENCE();
            pv_mfma(k, pp, 2);
            if (k == 3) {
                cvt(3, 0);
                cvt(3, 1);
            }
            STREAM_FENCE();
        }
        cvt(3, 2);
        cvt(3, 3);
        if (nlim < kTileKV) {  // wave-uniform, once per block with a partial last tile
            asm volatile("" ::: "memory");  // (a real branch: no if-conversion onto every step)
            mask_tile(n, nlim);
            mt[0] = mt[1] = mt[2] = mt[3] = tree_max(n.s0, n.s1);
        }
        n.mx = xhalf_max(fmaxf(max3f(mt[0], mt[1], mt[2]), mt[3]));
        n.rs = __builtin_amdgcn_ballot_w64(n.mx > kRescaleThr) != 0;
        // P of tile t is consumed only by the next step: without this tie the compiler sinks the
        // exponentials and packs past the barrier, where no MFMA runs beside them
        asm volatile("" : "+v"(pn[0][0]), "+v"(pn[0][1]), "+v"(pn[1][0]), "+v"(pn[1][1]));
        advance();
        if (rescale) {  // tile t - 1's PV went in at the old max: now O and l follow the new one
            o0 *= alpha;
            o1 *= alpha;
            l_acc *= alpha;
        }
        SSTAMP(4);

        // tile t + 2 landed (the younger pieces are the refill's), then every wave's
        stream_wait<WAITN>();
        SSTAMP(5);
        if (!(MHA_STREAM_ABL & 4)) __builtin_amdgcn_s_barrier();
        SSTAMP(6);

        if (first && has_prv) {  // the previous item's last PV went in this step: store it
#ifdef MHA_STREAM_STAMPS
            unsigned long long e0, e1;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e0)::"memory");
#endif
            epilogue(prv, qbad_prv);
            o0 = f32x16{};
            o1 = f32x16{};
            l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
            has_prv = false;
#ifdef MHA_STREAM_STAMPS
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e1)::"memory");
            ck_epi += e1 - e0;
#endif
        }
        if (!last) {
            ++t;
            return true;
        }
        if (!has_next) {
            // flush: the last tile's PV (its V is in the slot just passed), then the last store
            read_v(S, 0);
            read_v(S, 1);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pv_mfma(k, pn, 0);
                pv_mfma(k, pn, 1);
                pv_mfma(k, pn, 2);
            }
            epilogue(cur, qbad);
            return false;
        }
        prv = cur;
        has_prv = true;
        qbad_prv = qbad;
        qbad = qbad_next;
        j += G;
        cur = nxt;
        nt = (cur.nkv + kTileKV - 1) / kTileKV;
        t = 0;
        has_next = j + G < je;
        nxt = stream_item<MULTI, OSZ, NW>(a, has_next ? j + G : j);
        return true;
    };

    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;
    static_assert(NS == 4, "the loop is unrolled over 4 ring slots");
    for (;;) {
        if (!step(C0{}, sA, sB, pB, pA)) break;
        if (!step(C1{}, sB, sA, pA, pB)) break;
        if (!step(C2{}, sA, sB, pB, pA)) break;
        if (!step(C3{}, sB, sA, pA, pB)) break;
    }
    // drain: the loader's trailing (empty) pieces and the output stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef MHA_STREAM_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long ck_exit[2];
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_exit[0]), "=s"(ck_exit[1])::"memory");
    if (lane == 0 && a.stamps) {
        unsigned long long* dst = a.stamps + ((size_t)blockIdx.x * NW + wave) * 16;
        for (int i_ = 0; i_ < 7; ++i_) dst[i_] = ck_sum[i_];
        dst[8] = ck_entry[0];
        dst[9] = ck_entry[1];
        dst[10] = ck_exit[0];
        dst[11] = ck_exit[1];
        dst[12] = ck_pro;
        dst[13] = ck_epi;
    }
#endif
}
#undef MHA_SEL

template <typename TOut, int NW>
hipError_t launch_stream_t(const FwdArgs& a, int grid, hipStream_t stream) {
    if (a.n_calls > 1)
        hipLaunchKernelGGL((mha_hd64_stream_kernel<TOut, true, NW>), dim3(grid), dim3(64 * NW), 0, stream, a);
    else
        hipLaunchKernelGGL((mha_hd64_stream_kernel<TOut, false, NW>), dim3(grid), dim3(64 * NW), 0, stream, a);
    return hipGetLastError();
}

}  // namespace

int stream_grid(int items, int waves) {
    const int cap = waves == 8 ? stream_max_grid<8>() : stream_max_grid<4>();
    return items < cap ? items : cap;
}

hipError_t launch_stream(const FwdArgs& a, int waves, bool out_f32, hipStream_t stream) {
    const int grid = stream_grid(a.total_blocks, waves);
    if (grid <= 0) return hipSuccess;
    if (waves == 8) return out_f32 ? launch_stream_t<float, 8>(a, grid, stream) : launch_stream_t<f16, 8>(a, grid, stream);
    return out_f32 ? launch_stream_t<float, 4>(a, grid, stream) : launch_stream_t<f16, 4>(a, grid, stream);
}

}  // namespace mha_hd64
