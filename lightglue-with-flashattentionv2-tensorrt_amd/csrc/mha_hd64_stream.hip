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
//  * per step (64 keys, one barrier): phase A = QKᵀ of the next tile (v_mfma_f32_32x32x16_f16,
//    Sᵀ = K·Qᵀ so a lane holds one query) ‖ exp2 of this tile; phase B = Oᵀ += Vᵀ·Pᵀ of this tile
//    (P straight from the score registers, Vᵀ by ds_read_b64_tr_b16) + row sums on the matrix pipe
//    ‖ row max of the next tile;
//  * the running max rides in the QKᵀ chains' C operand (a register block holding −m, read, never
//    written: the MFMA emits s·c − m), so a probability is one v_exp_f32 and there is no bias
//    k-step; lazy rescale (threshold 8, log2 units) as the other kernels;
//  * epilogue per item: 1/l, fp16 pack, v_permlane32_swap pairs → 16-B row-segment stores
//    (cdna_hip_programming.md T21); rows past nq and keys past nkv are bounded by the buffer
//    descriptors (no pad / unpad).
// The DMA is inline asm with hand-counted waits: the compiler, seeing LDS-DMA builtins, drains
// every one in flight before the first transposing LDS read (it cannot tell them apart).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

// Diagnostic build (-DMHA_STREAM_STAMPS, tools/stream_stamps.py): per wave, the s_memtime cycles
// of every step summed by segment (0 refill issue, 1 decision / seam, 2 phase A issue, 3 phase B
// issue, 4 the counted DMA wait, 5 the barrier) and the step count, written at exit to
// a.stamps[(blockIdx.x * 4 + wave) * 8 + k]. The stamps return through lgkmcnt and are summed after
// the next barrier, where nothing else is outstanding on that counter.
#ifdef MHA_STREAM_STAMPS
#define SSTAMP(i) asm volatile("s_memtime %0" : "=s"(ck_[i])::"memory")
#else
#define SSTAMP(i) \
    do {          \
    } while (0)
#endif

#ifndef MHA_STREAM_PRIO
#define MHA_STREAM_PRIO 0  // A/B hook: s_setprio 1 for the odd workgroups
#endif

namespace mha_hd64 {
namespace {

constexpr int kStreamWaves = 4;
constexpr int kStreamRows = 32 * kStreamWaves;     // query rows per item
constexpr int kStreamSlots = 4;                    // LDS ring slots (64-key tiles)
constexpr int kStreamSlot = 2 * kTileBytes;        // K image, then V image
constexpr int kStreamQ = kStreamSlots * kStreamSlot;  // Q region (128 rows, K-style swizzle)
constexpr int kStreamLds = kStreamQ + kStreamRows * 128;
constexpr int kStreamMaxGrid = 512;                // two workgroups per CU

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

template <bool MULTI, int OSZ>
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
    it.q0 = qtile * kStreamRows;
    return it;
}

// One 1-KiB LDS-DMA piece: 64 lanes x 16 B from rs at voff + soff into LDS [m0, m0 + 1 KiB).
// M0 is written inside the statement (the compiler keeps no value in M0 across asm statements
// here). The compiler does not see this LDS write: every read of a slot is ordered behind the
// issuing waves' counted vmcnt and the workgroup barrier.
__device__ __forceinline__ void stream_dma(unsigned m0, unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned soff) {
    // (wave-uniform by construction; readfirstlane pins values the compiler computed on the
    // vector unit into SGPRs, as the "s" constraints need)
    m0 = __builtin_amdgcn_readfirstlane(m0);
    soff = __builtin_amdgcn_readfirstlane(soff);
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %3 offen lds"
        :
        : "s"(m0), "v"(voff), "s"(rs), "s"(soff)
        : "memory");
}

// Buffer descriptor from wave-uniform values, made provably uniform (T20): every buffer op on it
// keeps its descriptor in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return make_rsrc((const void*)(((unsigned long long)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
}

// Every VMEM op of the wave except the 4 youngest (the tile issued at this step's start) done.
__device__ __forceinline__ void stream_wait4() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }

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

// Scores and row max of one 64-key tile (two 32-key halves): the state that rotates per step.
struct StreamScores {
    f32x16 s0, s1;  // Sᵀ halves: keys 0..31 / 32..63 of the tile, query = lane % 32
    float mx;       // row max (both half-waves), relative to the running max (absolute on a
                    // block's first tile)
};

template <typename TOut, bool MULTI>
__global__ __launch_bounds__(64 * kStreamWaves, 2) void mha_hd64_stream_kernel(FwdArgs a) {
    constexpr int OSZ = (int)sizeof(TOut);
    __shared__ __attribute__((aligned(1024))) char smem[kStreamLds];
    lds_char* const lds = (lds_char*)smem;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave

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
    if (__builtin_amdgcn_readfirstlane(blockIdx.x) & 1) __builtin_amdgcn_s_setprio(1);
#endif

    // ---- per-lane constant addressing ----
    // K image (A operand of Sᵀ = K·Qᵀ): dim step s, half-wave hh reads chunk 2s + hh of key row r
    // (keys 0..31) and r + 32 (keys 32..63, + 4 KiB: the swizzle repeats every 16 rows). The Q
    // region has the same image (row = query).
    unsigned k_addr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = (unsigned)k_off(r, 2 * s + hh);
    const unsigned q_addr = (unsigned)(kStreamQ + 32 * wave * 128);  // + k_addr[s]
    // V image (A operand of Oᵀ = Vᵀ·Pᵀ via ds_read_b64_tr_b16): as the LDS-ring kernel's.
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const unsigned v_addr0 = (unsigned)(v_lane + 64 * vb + kTileBytes);        // dims 0..31
    const unsigned v_addr1 = (unsigned)(v_lane + 64 * (1 - vb) + kTileBytes);  // dims 32..63
    // DMA: piece p of a tile = rows 8p..8p+7, lane L writes LDS chunk L&7 of row 8p + L/8 and reads
    // the source chunk the image puts there. Wave w moves K and V pieces w and w + 4 of every tile
    // and Q pieces w, w + 4, w + 8, w + 12 (the K swizzle repeats every 16 rows: one lane offset).
    const unsigned dma_k = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7)) << 4));
    const unsigned dma_v = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ (((lane >> 4) & 1) << 2)) << 4));
    // Row sums on the matrix pipe (the LDS-ring kernel's selector): l_acc = sel · P per k-step.
    const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
    const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};

    // ---- loader: the tile stream over this workgroup's items ----
    int l_j = j, l_t = 0, l_nt;
    __amdgpu_buffer_rsrc_t k_l, v_l;
    auto loader_item = [&](int jj) {
        const StreamItem it = stream_item<MULTI, OSZ>(a, jj);
        l_nt = (it.nkv + kTileKV - 1) / kTileKV;
        k_l = stream_rsrc(it.k, (unsigned)it.nkv * kHeadDim * 2);
        v_l = stream_rsrc(it.v, (unsigned)it.nkv * kHeadDim * 2);
    };
    loader_item(j);
    // the loader's tile into `slot` (4 DMA pieces per wave), then the cursor moves on; past the
    // last item the pieces read from an empty descriptor (zeros into a slot nobody reads), so every
    // step issues exactly 4 and the counted waits stay exact
    auto issue = [&](int slot) {
        const unsigned m = lds0 + (unsigned)slot * kStreamSlot + (unsigned)wave * 1024u;
        const unsigned so = (unsigned)l_t * kTileBytes + (unsigned)wave * 1024u;
        stream_dma(m, dma_k, k_l, so);
        stream_dma(m + 4096u, dma_k, k_l, so + 4096u);
        stream_dma(m + kTileBytes, dma_v, v_l, so);
        stream_dma(m + kTileBytes + 4096u, dma_v, v_l, so + 4096u);
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
    // Q rows of item `it` into the Q region (4 pieces per wave)
    auto issue_q = [&](const StreamItem& it) {
        const __amdgpu_buffer_rsrc_t q_rs = stream_rsrc(it.q, (unsigned)it.nq * kHeadDim * 2);
        const unsigned m = lds0 + (unsigned)kStreamQ + (unsigned)wave * 1024u;
        const unsigned so = (unsigned)it.q0 * 128u + (unsigned)wave * 1024u;
#pragma unroll
        for (int i = 0; i < 4; ++i) stream_dma(m + 4096u * i, dma_k, q_rs, so + 4096u * i);
    };
    // Q fragments of this wave's rows from the Q region, scaled
    f16x8 qf[4];
    auto read_q = [&]() {
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = stream_scale_q(lds_read16(lds, q_addr + k_addr[s]));
    };

    // ---- compute state ----
    StreamItem cur = stream_item<MULTI, OSZ>(a, j);
    int nt = (cur.nkv + kTileKV - 1) / kTileKV;
    bool has_next = j + G < je;
    StreamItem nxt = stream_item<MULTI, OSZ>(a, has_next ? j + G : j);
    int t = 0;        // tile of the current item
    int gslot = 0;    // ring slot of the current tile
    f32x16 cm;        // -m (the QKᵀ chains' C operand)
    f32x16 o0 = {}, o1 = {};  // Oᵀ: dims 0..31 / 32..63, query on the lane
    f32x4 l_acc = {0.f, 0.f, 0.f, 0.f};  // row sums (every element: the lane's query)
    StreamScores sA, sB;

    auto mask_tile = [&](StreamScores& s, int lim) {  // keys >= lim of the tile -> -inf
        const int l4 = lim - 4 * hh;  // element i holds key (i & 3) + 8 (i >> 2) + 4 hh (+ 32 in s1)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int key = (i & 3) + 8 * (i >> 2);
            s.s0[i] = key >= l4 ? -INFINITY : s.s0[i];
            s.s1[i] = key + 32 >= l4 ? -INFINITY : s.s1[i];
        }
    };

    // prologue: Q of the first item and tiles 0..2 of the stream; Q and tiles 0, 1 landed
    issue_q(cur);
    issue(0);
    issue(1);
    issue(2);
    stream_wait4();
    __builtin_amdgcn_s_barrier();
    read_q();
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
    }
    __builtin_amdgcn_s_barrier();  // every wave's Q reads done before step 0 refills the Q region

    // One step = tile t of the current item, its scores in c; the next tile's scores into n.
    // Returns false once the workgroup's last item is stored.
#ifdef MHA_STREAM_STAMPS
    unsigned long long ck_[7] = {}, ck_sum[7] = {};
    bool ck_live = false;
#endif
    auto step = [&](StreamScores& c, StreamScores& n) -> bool {
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
        const bool seam = last && has_next;   // the next tile is the next item's first
        const int nlim = !last ? min(kTileKV, cur.nkv - kTileKV * (t + 1)) : min(kTileKV, nxt.nkv);
        const int nslot = (gslot + 1) & 3;
        if (first) issue_q(nxt);  // the Q region is free since the last item's seam step
        issue((gslot + 3) & 3);   // the slot of tile t - 1: free since the last barrier
        SSTAMP(1);

        // online-softmax decision for tile t
        if (first) {
            const float d = (c.mx < kEmptyMax) ? 0.f : c.mx;  // (a fully masked tile: m = 0)
            cm = splat16(-d);
            c.s0 -= d;
            c.s1 -= d;
        } else if (__builtin_amdgcn_ballot_w64(c.mx > kRescaleThr) != 0) {  // wave-uniform, rare
            const float d = fmaxf(c.mx, 0.f);
            const float alpha = __builtin_amdgcn_exp2f(-d);
            o0 *= alpha;
            o1 *= alpha;
            l_acc *= alpha;
            cm -= d;
            c.s0 -= d;
            c.s1 -= d;
        }
        if (seam) {  // the next item's Q (C = 0: its max is set at its first step)
            if (first) {  // a one-tile item: the Q pieces issued above, landed everywhere
                stream_wait4();
                __builtin_amdgcn_s_barrier();
            }
            read_q();
            cm = f32x16{};
        }

        // phase A: QKᵀ of the next tile on the matrix pipe ‖ exp2 of this tile, in a fixed order
        // (fences): 8 exps up front while the first K fragments land, then one MFMA + 3 v_exp_f32
        // per gap; the second half of K and the V fragments are read between the MFMAs (shorter
        // register lifetimes). The QKᵀ runs unconditionally: on the workgroup's very last step it
        // scores a slot nobody uses (no branch splits the interleave).
        const unsigned kbase = (unsigned)nslot * kStreamSlot;
        const unsigned vbase = (unsigned)gslot * kStreamSlot;
        auto exp_at = [&](int e) {
            if (e < 16) c.s0[e] = __builtin_amdgcn_exp2f(c.s0[e]);
            else c.s1[e - 16] = __builtin_amdgcn_exp2f(c.s1[e - 16]);
        };
        f16x8 kf[8];
        auto read_k = [&](int s) {
            kf[2 * s] = lds_read16(lds, kbase + k_addr[s]);
            kf[2 * s + 1] = lds_read16(lds, kbase + k_addr[s] + 4096u);
        };
        f16x8 vfa[2][2], vfb[2][2];
        auto read_v = [&](int jj) {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const unsigned rowc = vbase + 128u * (32 * jj + 16 * ss);
                vfa[jj][ss] = cat8(tr_read(lds, v_addr0 + rowc), tr_read(lds, v_addr0 + rowc + 8 * 128));
                vfb[jj][ss] = cat8(tr_read(lds, v_addr1 + rowc), tr_read(lds, v_addr1 + rowc + 8 * 128));
            }
        };
        SSTAMP(2);
        __builtin_amdgcn_sched_barrier(0);
        read_k(0);
        read_k(1);
#pragma unroll
        for (int e = 0; e < 8; ++e) exp_at(e);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int s = i >> 1;
            if ((i & 1) == 0) n.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i], qf[s], s == 0 ? cm : n.s0, 0, 0, 0);
            else n.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[i], qf[s], s == 0 ? cm : n.s1, 0, 0, 0);
            exp_at(8 + 3 * i);
            exp_at(9 + 3 * i);
            exp_at(10 + 3 * i);
            if (i == 1) {
                read_k(2);
                read_k(3);
            }
            if (i == 3) read_v(0);
            if (i == 5) read_v(1);
            __builtin_amdgcn_sched_barrier(0);
        }
        // P (f16) as the B operand: registers 8ss..8ss+7 of a 32x32 tile = k-step ss
        f16x8 p[2][2];
        auto cvt_p = [&](int jj, int ss) {
            const f32x16& x = jj ? c.s1 : c.s0;
#pragma unroll
            for (int e = 0; e < 8; ++e) p[jj][ss][e] = (f16)x[8 * ss + e];
        };

        SSTAMP(3);
        // phase B: Oᵀ += Vᵀ·Pᵀ and the row sums ‖ row max of the next tile (and the P packing one
        // k-step ahead)
        cvt_p(0, 0);
        __builtin_amdgcn_sched_barrier(0);
        float mt[4];  // partial maxima of the next tile's scores (v_max3 tree, 4 per k-step)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int jj = k >> 1, ss = k & 1;
            o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], p[jj][ss], o0, 0, 0, 0);
            if (k < 3) cvt_p((k + 1) >> 1, (k + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
            o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], p[jj][ss], o1, 0, 0, 0);
            {
                const f32x16& x = k < 2 ? n.s0 : n.s1;
                const int b = 8 * (k & 1);
                const float u = max3f(x[b], x[b + 1], x[b + 2]);
                const float v = max3f(x[b + 3], x[b + 4], x[b + 5]);
                mt[k] = max3f(u, v, fmaxf(x[b + 6], x[b + 7]));
            }
            __builtin_amdgcn_sched_barrier(0);
            l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, p[jj][ss], l_acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (nlim < kTileKV) {  // wave-uniform, once per block with a partial last tile
            asm volatile("" ::: "memory");  // (a real branch: no if-conversion onto every step)
            mask_tile(n, nlim);
            mt[0] = mt[1] = mt[2] = mt[3] = tree_max(n.s0, n.s1);
        }
        n.mx = xhalf_max(fmaxf(max3f(mt[0], mt[1], mt[2]), mt[3]));

        // tile t + 2 landed (the 4 pieces of tile t + 3 are the younger ops), then every wave's
        SSTAMP(4);
        stream_wait4();
        SSTAMP(5);
        __builtin_amdgcn_s_barrier();
        SSTAMP(6);
        gslot = (gslot + 1) & 3;

        if (!last) {
            ++t;
            return true;
        }
        // epilogue: O = Oᵀ / l for the block's rows (rows past nq: dropped by the descriptor)
        {
            const float inv = 1.f / l_acc[0];
            const __amdgpu_buffer_rsrc_t o_rs = stream_rsrc(cur.o, (unsigned)cur.nq * kHeadDim * OSZ);
            const unsigned row = (unsigned)(cur.q0 + 32 * wave + r);
            if constexpr (OSZ == 2) {
                // lane (query, hh) holds dims 8k + 4hh .. +3 of group k (o0: k 0..3, o1: 4..7);
                // v_permlane32_swap pairs (k, k+1) so each lane holds 8 consecutive dims
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
        }
        if (!has_next) return false;
        o0 = f32x16{};
        o1 = f32x16{};
        l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
        j += G;
        cur = nxt;
        nt = (cur.nkv + kTileKV - 1) / kTileKV;
        t = 0;
        has_next = j + G < je;
        nxt = stream_item<MULTI, OSZ>(a, has_next ? j + G : j);
        return true;
    };

    while (step(sA, sB) && step(sB, sA)) {
    }
    // drain: the loader's trailing (empty) pieces and the output stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef MHA_STREAM_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0 && a.stamps) {
        unsigned long long* dst = a.stamps + ((size_t)blockIdx.x * 4 + wave) * 8;
        for (int i_ = 0; i_ < 7; ++i_) dst[i_] = ck_sum[i_];
    }
#endif
}
#undef MHA_SEL

template <typename TOut>
hipError_t launch_stream_t(const FwdArgs& a, int grid, hipStream_t stream) {
    if (a.n_calls > 1)
        hipLaunchKernelGGL((mha_hd64_stream_kernel<TOut, true>), dim3(grid), dim3(64 * kStreamWaves), 0, stream, a);
    else
        hipLaunchKernelGGL((mha_hd64_stream_kernel<TOut, false>), dim3(grid), dim3(64 * kStreamWaves), 0, stream, a);
    return hipGetLastError();
}

}  // namespace

int stream_grid(int items) { return items < kStreamMaxGrid ? items : kStreamMaxGrid; }

hipError_t launch_stream(const FwdArgs& a, bool out_f32, hipStream_t stream) {
    const int grid = stream_grid(a.total_blocks);
    if (grid <= 0) return hipSuccess;
    return out_f32 ? launch_stream_t<float>(a, grid, stream) : launch_stream_t<f16>(a, grid, stream);
}

}  // namespace mha_hd64
