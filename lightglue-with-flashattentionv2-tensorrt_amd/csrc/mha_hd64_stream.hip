// mha_hd64_stream.hip — persistent streaming FlashAttention forward, head_dim = 64, for gfx950
// (MI355X): the throughput form of the MHAHeadDim64 operator.
//
// Same operator as mha_hd64_kernels.hip (O = softmax(Q·Kᵀ·0.125)·V per (batch, head); reference
// lightglue_attention_plugin/attention_headdim_64_fp16in_fp16out.cu:253-733 and
// …fp16in_fp32out.cu:253-703, oracle lightglue_pytorch_no_plugin/lightglue.py:75-85) for launches
// that carry more 128-row query blocks than one round of the chip holds: batched image-pair
// streams (many calls stacked in the batch dimension) and grouped matcher layers of several pairs.
//
// Structure (round 4). The steady step is the one tools/mb_step.hip measures in isolation
// (profiles/r04/mb_step.txt): with every ingredient in it (MFMAs, exponentials, packs, row max,
// LDS fragment reads, LDS-DMA refill, one barrier) a 32-row wave-step costs ≈1500 cycles at two
// waves per SIMD, 77 % of the matrix pipe. The round-3 form of this kernel ran the same step in
// ≈2660 cycles (in-kernel stamps, profiles/r04/stream_stamps.jsonl): item-seam logic inside
// every step (first / last / seam / tail-mask branches) made the compiler split the step into
// many blocks, sink the row max out of the MFMA interleave and copy state at the joins. Here:
//  * item = (call, batch·head, 32·NW-row query block) with ALL of its keys; workgroup = NW waves,
//    32 query rows each, <= 256 VGPRs. NW = 4: 128-row items, 80 KiB LDS, two workgroups per CU,
//    so every SIMD runs one wave of each; NW = 8: 256-row items, 160 KiB LDS, one workgroup per
//    CU whose two waves per SIMD share every K/V tile (half the DMA per wave, no second workgroup
//    losing issue arbitration to the first). The planner takes NW = 8 when its last round of
//    items is at least 3/4 full;
//  * persistent and XCD-aware: grid = min(items, 512); the workgroups of XCD x walk a contiguous
//    range of items (consecutive query blocks of one head: its K/V is read through one L2);
//  * the pipeline runs across items without a seam: an item's LAST step computes QKᵀ of the next
//    item's tile 0 (with that item's Q and C = 0; its exact row max becomes the next running max),
//    and the next item's FIRST step does the P·V of this item's last tile and then its epilogue,
//    whose output stores it issues after its own refill so that its counted wait leaves them in
//    flight. So every step is a full step: the FIRST step, pairs of MIDDLE steps in a loop whose
//    body has no branch but the rare rescale, tail steps that mask keys past nkv, the LAST step.
//    Tiles per item are rounded up to an even count (the padding tile is fully masked), so the
//    middle loop alternates two named register states;
//  * step t: the matrix pipe runs QKᵀ of tile t+1 (v_mfma_f32_32x32x16_f16, Sᵀ = K·Qᵀ, a lane
//    holds one query) and then Oᵀ += Vᵀ·Pᵀ of tile t−1 (P packed to fp16 in the previous step,
//    Vᵀ by ds_read_b64_tr_b16) + its row sums (v_mfma_f32_16x16x32_f16), while the vector pipe
//    exponentiates and packs tile t and takes the row max of tile t+1 — one exponential pair per
//    MFMA gap; no MFMA waits for the vector work of its own step;
//  * the running max rides in the QKᵀ chains' C operand (−m in every element), so a probability
//    is one v_exp_f32; lazy rescale (threshold 8, log2 units): the decision for tile t is taken at
//    the start of step t from the max of the previous step, O and l follow after P·V of tile t−1
//    (which is still at the old max: cdna_hip_programming.md T13's safe order);
//  * K and V stream by LDS-DMA (`buffer_load_dwordx4 … lds`, 1 KiB per wave instruction, XOR
//    swizzles applied on the source address) into a ring of 64-key tiles (NW 4: 4 slots, 2 tiles
//    ahead; NW 8: 8 slots, 4 ahead; slot = global tile index mod slots, a runtime value: one
//    scalar add per DMA, one vector add per fragment base), CONTINUOUSLY across items: a loader
//    cursor (StreamLoader) runs `lead` tiles ahead of the compute side, into the next item (or
//    several short ones). Each wave DMAs its own 32 Q rows of the next item during the first
//    step, so no wave waits for another's Q;
//  * epilogue per item: 1/l, fp16 pack, v_permlane32_swap pairs → 16-B row-segment stores
//    (cdna_hip_programming.md T21); rows past nq and keys past nkv are bounded by the buffer
//    descriptors (no pad / unpad).
// The DMA is inline asm with hand-counted waits (lds_dma16 / lds_dma16_s, mha_hd64_device.h;
// wait states audited on the built library by tools/check_dma_hazards.py): in the 4-wave form
// every step ends with this wave's DMAs landed (vmcnt(0)) and one workgroup barrier; in the 8-wave
// form every second step ends with all but the newest tile's DMAs landed and one barrier.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "mha_hd64_device.h"
#include "mha_hd64_internal.h"

// Diagnostic build (-DMHA_STREAM_STAMPS, tools/stream_stamps.py): per wave, s_memtime cycles by
// part, written at exit to a.stamps[(blockIdx.x * 4 + wave) * 48 + k]: 0 item prologues, 1 first
// steps, 2 middle-loop steps, 3 tail + last steps + epilogues, 6 middle steps counted, 14 items,
// 8..11 s_memtime / s_memrealtime (100 MHz) at entry and exit (the in-kernel clock,
// MI355X_MICROARCH.md DVFS item 6), 12 the end of the kernel prologue; 16 + k chained segments
// (SEG(k): 0 item advance, 1 next Q issue, 2..5 FIRST step phase A / phase B / mask+max+epilogue
// +wait / barrier, 6..9 the same for middle steps, 10..13 tail steps, 14 to the last step, 15 read_q,
// 16..19 the LAST step).
#ifdef MHA_STREAM_STAMPS
#define SCLK(var) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory")
// chained segments: sg[k] += cycles since the previous SEG stamp (written to slots 16 + k)
#define SEG(k)                                      \
    do {                                            \
        unsigned long long t_;                      \
        SCLK(t_);                                   \
        sg[k] += (unsigned)(t_ - ck_last);          \
        ck_last = t_;                               \
    } while (0)
#else
#define SCLK(var) \
    do {          \
    } while (0)
#define SEG(k) \
    do {       \
    } while (0)
#endif
constexpr int kStreamStampSlots = 48;  // per wave, diagnostic builds

namespace mha_hd64 {
namespace {

// NW waves per workgroup (4: 128-row items, two workgroups per CU; 8: 256-row items sharing each
// K/V tile, one workgroup per CU)
template <int NW>
constexpr int stream_rows() { return 32 * NW; }  // query rows per item
constexpr int kSSlot = 2 * kTileBytes;            // one ring slot: K image, then V image (16 KiB)
// ring slots and lead (the refill of step t is global tile t + lead): NW 4: 4 slots, lead 2, a
// barrier every step (80 KiB: two workgroups per CU); NW 8: 8 slots, lead 4, a barrier every second
// step (160 KiB, the whole LDS)
template <int NW>
constexpr int stream_slots() { return NW == 8 ? 8 : 4; }
template <int NW>
constexpr int stream_lead() { return NW == 8 ? 4 : 2; }
template <int NW>
constexpr int stream_q_off() { return stream_slots<NW>() * kSSlot; }  // Q region: the item's rows
template <int NW>
constexpr int stream_lds() { return stream_q_off<NW>() + stream_rows<NW>() * 128; }  // 80 / 160 KiB
template <int NW>
constexpr int stream_max_grid() { return NW == 4 ? 512 : 256; }  // one residency round

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

// Buffer descriptor from wave-uniform values, made provably uniform (T20): every buffer op on it
// keeps its descriptor in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return make_rsrc((const void*)(((unsigned long long)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
}

// One item's scalar description for the compute side (batch·head offsets applied): its Q and O
// descriptors, key count, first query row and tile count.
struct StreamItem {
    __amdgpu_buffer_rsrc_t q, o;
    int nkv;
    int q0;  // first query row of the block
    int nt;  // 64-key tiles, rounded up to an even count (the padding tile reads zeros, masked)
};
// The loader's cursor: K/V descriptors of the item whose tiles it issues, its next local tile, its
// tile count and its index. It runs `lead` tiles ahead of the compute side, across item seams
// (over several short items if need be).
struct StreamLoader {
    __amdgpu_buffer_rsrc_t k, v;
    int lt, nt, j;
};

__device__ __forceinline__ int stream_tiles(int nkv) { return ((nkv + 2 * kTileKV - 1) / (2 * kTileKV)) * 2; }

template <bool MULTI, int OSZ, int NW>
__device__ __forceinline__ StreamItem stream_item(const FwdArgs& a, int j, bool live) {
    const int ci = stream_call<MULTI>(a, j);
    const int nq = MHA_SEL(nq), nkv = MHA_SEL(nkv), qtiles = MHA_SEL(qtiles);
    const int jl = j - MHA_SEL(block_begin);
    const int bh = jl / qtiles, qtile = jl - bh * qtiles;
#ifdef MHA_STREAM_L2Q  // diagnostic: every item reads the first query block (L2-resident)
    const int bhq = 0;
#else
    const int bhq = bh;
#endif
    const char* q = reinterpret_cast<const char*>(MHA_SEL(q)) + (size_t)bhq * nq * (kHeadDim * 2);
    char* o = reinterpret_cast<char*>(MHA_SEL(o)) + (size_t)bh * nq * (kHeadDim * OSZ);
    StreamItem it;
    // (a dead item — past the workgroup's last — gets an empty Q descriptor: its DMA reads zeros)
    it.q = stream_rsrc(q, live ? (unsigned)nq * kHeadDim * 2 : 0u);
    it.o = stream_rsrc(o, (unsigned)nq * kHeadDim * OSZ);
    it.nkv = nkv;
#ifdef MHA_STREAM_L2Q
    it.q0 = 0;
#else
    it.q0 = qtile * stream_rows<NW>();
#endif
    it.nt = stream_tiles(nkv);
    return it;
}

template <bool MULTI>
__device__ __forceinline__ StreamLoader stream_kv(const FwdArgs& a, int j, bool live) {
    const int ci = stream_call<MULTI>(a, j);
    const int nkv = MHA_SEL(nkv), qtiles = MHA_SEL(qtiles);
    const int bh = (j - MHA_SEL(block_begin)) / qtiles;
#ifdef MHA_STREAM_L2KV  // diagnostic: every item streams the first head's K/V (L2-resident)
    const int bhk = 0;
#else
    const int bhk = bh;
#endif
    const char* k = reinterpret_cast<const char*>(MHA_SEL(k)) + (size_t)bhk * nkv * (kHeadDim * 2);
    const char* v = reinterpret_cast<const char*>(MHA_SEL(v)) + (size_t)bhk * nkv * (kHeadDim * 2);
    StreamLoader ld;
    // (past the workgroup's last item: empty descriptors, zeros into the ring, forever)
    const unsigned kvb = live ? (unsigned)nkv * kHeadDim * 2 : 0u;
    ld.k = stream_rsrc(k, kvb);
    ld.v = stream_rsrc(v, kvb);
    ld.lt = 0;
    ld.nt = live ? stream_tiles(nkv) : (1 << 30);
    ld.j = j;
    return ld;
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

// Scores and row max of one 64-key tile (two 32-key halves): the state that alternates per step.
struct StreamScores {
    f32x16 s0, s1;  // Sᵀ halves: keys 0..31 / 32..63 of the tile, query = lane % 32
    float mx;       // row max (both half-waves) relative to the running max
    bool rs;        // some query of the wave exceeds the running max by > kRescaleThr (wave-uniform)
};

// Speculative running max (-DMHA_STREAM_SPEC=1: an A/B build, not shipped): an item's running max is
// its tile 0's and never moves, so the middle and tail steps carry no row max of the next tile, no
// rescale decision and no rescale (≈ 20 of the step's ≈ 44 non-exponential vector instructions).
// Exact while no later score exceeds it by 2^16 (the fp16 P would overflow; below that fp16's
// relative precision does not depend on magnitude and the row sums and O accumulate in fp32). An
// overflow makes the row sum +Inf (NaN keys, or the partner row of the row-sum MFMA: NaN), which the
// epilogue sees: the item is marked, and at the end of the kernel the wave recomputes its rows of
// every marked item with an exact online softmax (exact_item below) through its own ring slot.
// Round 6 measurements (profiles/r06/stream_spec_*.jsonl, lazy -> spec): random inputs 32 calls
// 44.0 -> 41.3 us (tools/spec_rare_cost.py), but bench.py's 32 / 64-call lines 41.4 -> 41.2 and
// 76.1 -> 75.4 us only; one spike key per head 44.3 -> 70.1 us (gain 3) and 45.0 -> 94.9 (gain 6:
// secondary overflows mark nearly every item); and the seeded matcher's batched forwards, whose
// attention rows do overflow (tools/matcher_nan_probe.py), 1.278 -> 1.361 ms at P = 8, 2.333 ->
// 2.553 at P = 16. A re-run costs a whole item, so no rare path makes a marked fraction f cheaper
// than ≈ 1 + 1.3 f; the lazy form below stays the default.
#ifndef MHA_STREAM_SPEC
#define MHA_STREAM_SPEC 0
#endif

template <typename TOut, bool MULTI, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void mha_hd64_stream_kernel(FwdArgs a) {
    constexpr int OSZ = (int)sizeof(TOut);
    constexpr int kPW = 8 / NW;  // DMA pieces (1 KiB, 8 rows) per wave of each 8 KiB K or V image
    constexpr int kPiece = 2 * kPW;  // DMA pieces per wave and tile (K and V)
    constexpr unsigned kSM = (unsigned)stream_slots<NW>() - 1u;  // ring slot = global tile & kSM
    constexpr int L = stream_lead<NW>();  // the refill of step t: global tile t + L
    __shared__ __attribute__((aligned(1024))) char smem[stream_lds<NW>()];
    lds_char* const lds = (lds_char*)smem;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int r = lane & 31;   // query column of the MFMA tiles
    const int hh = lane >> 5;  // half-wave

#ifdef MHA_STREAM_STAMPS
    unsigned long long ck_entry[2], ck_pro = 0, ck_t0 = 0, ck_t1 = 0;
    unsigned long long ck_sum[4] = {0, 0, 0, 0}, ck_mid = 0, ck_items = 0, ck_last = 0;
    unsigned sg[24];
#pragma unroll
    for (int i_ = 0; i_ < 24; ++i_) sg[i_] = 0;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_entry[0]), "=s"(ck_entry[1])::"memory");
#endif
    // This workgroup's items: XCD x = blockIdx % 8 owns the contiguous range [jb, je) of the T
    // items; its G workgroups take every G-th item from their local index (at least one each).
    const int T = a.total_blocks;
    const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
    const int q8 = T >> 3, r8 = T & 7;
    const int jb = xcd * q8 + min(xcd, r8);
    const int je = jb + q8 + (xcd < r8 ? 1 : 0);
    const int G = ((int)gridDim.x - xcd + 7) >> 3;
    int j = jb + loc;
    if (j >= je) return;  // (grid <= items: never)

    // ---- per-lane constant addressing ----
    // K image (A operand of Sᵀ = K·Qᵀ): dim step s, half-wave hh reads chunk 2s + hh of key row r
    // (keys 0..31) and r + 32 (keys 32..63, + 4 KiB: the swizzle repeats every 16 rows). The Q
    // region has the same image (row = query of the item).
    unsigned k_addr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = (unsigned)k_off(r, 2 * s + hh);
    const unsigned q_base = (unsigned)(stream_q_off<NW>() + 32 * wave * 128);
    // V image (A operand of Oᵀ = Vᵀ·Pᵀ via ds_read_b64_tr_b16): as the LDS-ring kernel's.
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const unsigned v_addr0 = (unsigned)(v_lane + 64 * vb + kTileBytes);        // dims 0..31
    const unsigned v_addr1 = (unsigned)(v_lane + 64 * (1 - vb) + kTileBytes);  // dims 32..63
    // DMA: piece p of an image = rows 8p..8p+7; lane L writes LDS chunk L&7 of row 8p + L/8 and
    // reads the source chunk the image puts there. The K / Q swizzle depends on p's parity; wave w
    // moves K and V pieces w, w + 4 of every tile and Q pieces 4w..4w+3 (its own 32 rows).
    auto dma_kq = [&](int parity) {
        return (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ ((4 * parity + (lane >> 4)) & 7)) << 4));
    };
    const unsigned dma_k = dma_kq(wave & 1);
    const unsigned dma_q0 = dma_kq(0), dma_q1 = dma_kq(1);
    const unsigned dma_v = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ (((lane >> 4) & 1) << 2)) << 4));
    const unsigned m0w = (unsigned)__builtin_amdgcn_readfirstlane(lds0 + (unsigned)wave * 1024u);
    const unsigned sow = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wave * 1024u);
    // Row sums on the matrix pipe (the LDS-ring kernel's selector): l_acc = sel · P per k-step.
    const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
    const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};

    // The loader's K and V pieces of its current tile into ring slot `slot` (pieces wave + NW·h of
    // each image, 8 KiB apart per image), then its cursor moves on (past an item's last tile: the
    // workgroup's next item, or an empty one past the last)
    StreamLoader ld = stream_kv<MULTI>(a, j, true);
    auto issue_tile = [&](unsigned slot) {
        const unsigned m = m0w + slot * (unsigned)kSSlot;
        const unsigned so = (unsigned)ld.lt * (unsigned)kTileBytes + sow;
#pragma unroll
        for (int h = 0; h < kPW; ++h) {
            const unsigned ho = (unsigned)(h * NW * 1024);
            lds_dma16(m + ho, dma_k, ld.k, so + ho);
            lds_dma16(m + (unsigned)kTileBytes + ho, dma_v, ld.v, so + ho);
        }
    };
    auto ld_advance = [&]() {
        if (++ld.lt >= ld.nt) {  // (wave-uniform, once per item)
            const int jn = ld.j + G;
            ld = stream_kv<MULTI>(a, jn < je ? jn : ld.j, jn < je);
            ld.j = jn;
        }
    };
    // this wave's 32 Q rows of an item into its part of the Q region
    const unsigned q_m0 = (unsigned)__builtin_amdgcn_readfirstlane(lds0 + q_base);
    auto issue_q = [&](const StreamItem& it) {
        const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(it.q0 + 32 * wave) * 128u);
#pragma unroll
        for (int i = 0; i < 4; ++i) lds_dma16(q_m0 + 1024u * i, (i & 1) ? dma_q1 : dma_q0, it.q, so + 1024u * i);
    };

    // ---- state ----
    StreamItem cur = stream_item<MULTI, OSZ, NW>(a, j, true);
    StreamItem nxt = stream_item<MULTI, OSZ, NW>(a, j + G < je ? j + G : j, j + G < je);
    unsigned gb = 0;  // global tile index of the current item's tile 0 (ring slot = index & kSM)
    f16x8 qf[4];
    f32x16 cm;                  // −m (the QKᵀ chains' C operand)
    f32x16 o0, o1;              // Oᵀ: dims 0..31 / 32..63, query on the lane
    f32x4 l_acc;                // row sums (every element: the lane's query)
    StreamScores sA, sB;
    f16x8 pA[2][2], pB[2][2];   // P (fp16) of a tile: B operand of k-step (jj, ss) of Oᵀ = Vᵀ·Pᵀ

    // kernel prologue: the first item's Q and global tiles 0 .. L − 1 issued; Q and tiles 0, 1
    // landed everywhere (NW 8: tiles 2, 3 issued after the first barrier and still in flight; the
    // first item's FIRST step waits for tile 2 before its barrier); the V image of the last slot and pB zeroed: the first FIRST step's
    // P·V of "tile −1" adds 0·0 (that slot's first refill is tile kSM, issued after a barrier)
    // (NW 8: tiles 0, 1 with Q, tiles 2, 3 after the first barrier: the whole chip's burst before
    // the first barrier is smaller; 16 calls 24.5 vs 25.3 us, profiles/r04/stream_prologue_split.jsonl)
    constexpr int L0 = NW == 8 ? 2 : L;
    issue_q(cur);
#pragma unroll
    for (int i = 0; i < L0; ++i) {
        issue_tile((unsigned)i);
        ld_advance();
    }
#pragma unroll
    for (unsigned off = (unsigned)tid * 16u; off < (unsigned)kTileBytes; off += 64u * NW * 16u)
        lds_write16(lds, kSM * (unsigned)kSSlot + (unsigned)kTileBytes + off, f16x8{});
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) pB[jj][ss] = f16x8{};
    // Q and tile 0 first: tile 0's QKᵀ below runs while tile 1 lands
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((L0 - 1) * kPiece) : "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = L0; i < L; ++i) {
        issue_tile((unsigned)i);
        ld_advance();
    }
#ifdef MHA_STREAM_STAMPS
    SCLK(ck_pro);
    ck_last = ck_pro;
#endif

    auto mask_tile = [&](StreamScores& s, int lim) {  // keys >= lim of the tile -> -inf
        int l4 = lim - 4 * hh;  // element i holds key (i & 3) + 8 (i >> 2) + 4 hh (+ 32 in s1)
        // (opaque: with one call per launch nkv is loop-invariant, and the compiler would hoist the
        // 32 compares out of the item loop as 64 SGPRs of lane masks, spilled to VGPR lanes)
        asm volatile("" : "+v"(l4));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int key = (i & 3) + 8 * (i >> 2);
            s.s0[i] = key >= l4 ? -INFINITY : s.s0[i];
            s.s1[i] = key + 32 >= l4 ? -INFINITY : s.s1[i];
        }
    };
    f16x8 kf[8];
    auto read_k = [&](unsigned kbase, int s) {
        kf[2 * s] = lds_read16(lds, kbase + k_addr[s]);
        kf[2 * s + 1] = lds_read16(lds, kbase + k_addr[s] + 4096u);
    };
    f16x8 vfa[2][2], vfb[2][2];
    auto read_v = [&](unsigned vbase, int jj) {
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            const unsigned rowc = vbase + 128u * (32 * jj + 16 * ss);
            vfa[jj][ss] = cat8(tr_read(lds, v_addr0 + rowc), tr_read(lds, v_addr0 + rowc + 8 * 128));
            vfb[jj][ss] = cat8(tr_read(lds, v_addr1 + rowc), tr_read(lds, v_addr1 + rowc + 8 * 128));
        }
    };
    // SPEC: the items (ordinal k of this workgroup's walk, bit min(k, 63)) with a row sum that
    // overflowed (or a NaN key), recomputed exactly at the end
    unsigned long long dirty = 0;
    // O = Oᵀ / l of an item (rows past nq: dropped by the descriptor)
    auto epilogue = [&](__amdgpu_buffer_rsrc_t o_rs, int q0, unsigned qbad_it, int ord) {
        if constexpr (MHA_STREAM_SPEC) {
            // the bits behind an empty asm (-fno-honor-nans folds a float class test). Not an asm
            // v_mov: the flush's epilogue follows the last row-sum MFMA directly, and the hazard
            // recognizer puts no wait states before an instruction inside inline asm — such a move
            // read the register before the MFMA had written it (an overflow missed, its rows left
            // NaN; tools/check_mfma_hazards.py audits the library for it)
            unsigned lb = __builtin_bit_cast(unsigned, l_acc[0]);
            asm volatile("" : "+v"(lb));
            const bool over = (lb & 0x7f800000u) == 0x7f800000u && !((qbad_it >> r) & 1u);
            if (__builtin_amdgcn_ballot_w64(over) != 0) dirty |= 1ull << (ord < 63 ? ord : 63);
        }
        const float inv = inv_or_nan(l_acc[0], qbad_it, r);  // a non-finite query row: NaN
        const unsigned row = (unsigned)(q0 + 32 * wave + r);
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

    // The previous item's output (its epilogue runs in the next item's FIRST step)
    bool prev = false;  // a previous item of this workgroup awaits its last P·V and epilogue
    __amdgpu_buffer_rsrc_t prv_o = cur.o;
    int prv_q0 = 0;
    unsigned qbad_prv = 0;
    int item_no = 0, prv_no = 0;  // ordinal of the current / previous item in this workgroup's walk

    // One step of the current item — every step is a full step of the pipeline: tile t's
    // exponentials; QKᵀ of global tile g + 1 (LAST: the next item's tile 0, with the next item's Q
    // and C = 0); P·V of global tile g − 1 (FIRST: the previous item's last tile, then that item's
    // epilogue — unless PREV is false: the workgroup's first item); the refill of global tile
    // g + L (the loader's cursor); the step's counted wait + barrier (NW 8: odd steps only; nt is
    // even, so every item starts on an even global tile). MASK: tile t + 1 may hold keys past nkv.
    // c: scores of tile t; n: of tile t + 1; pp: P of tile g − 1 (consumed); pn: P of tile t
    // (produced). One instantiation per kind (KIND: 0 FIRST, 1 / 4 MIDDLE odd / even t, 2 / 5 TAIL
    // odd / even t, 3 LAST), each called from one place: step variants in the arms of a branch
    // would share their first instructions, which the IR passes hoist above the branch — the whole
    // exponential block, out of the interleave.
    // FIRST always runs its P·V (the workgroup's first item: P = 0 against a zeroed V image) and
    // decides at run time whether an epilogue follows; TAIL and LAST mask at run time.
    auto step = [&](auto kind_c, int t, StreamScores& c, StreamScores& n, const f16x8 (&pp)[2][2],
                    f16x8 (&pn)[2][2]) {
        constexpr int KIND = decltype(kind_c)::value;
        constexpr bool FIRST = KIND == 0;
        constexpr bool PV = true;  // a P·V of global tile g − 1 in phase B
        constexpr bool LAST = KIND == 3;
        constexpr bool MASK = KIND != 1 && KIND != 4;  // tile t + 1 may hold keys past nkv
        constexpr bool BAR = NW == 4 || KIND == 1 || KIND == 2 || KIND == 3;  // (NW 8: odd t)
        // the row max of tile t + 1: every step of the lazy-rescale form; SPEC: the LAST step only
        // (the next item's tile 0 sets its running max)
        constexpr bool NEEDMAX = !MHA_STREAM_SPEC || LAST;
        const unsigned g = gb + (unsigned)t;
#ifdef MHA_STREAM_PRIO_BAL
        // NW 8, between two barriers: the first step at raised priority, the second at normal, so
        // the wave of a SIMD pair that finishes its first step ahead (the older one, on age) yields
        // the issue to the other until it catches up (experiment)
        if constexpr (NW == 8) __builtin_amdgcn_s_setprio(BAR ? 0 : 1);
#endif
        const unsigned kbase = ((g + 1u) & kSM) * (unsigned)kSSlot;  // K of tile t + 1
        const unsigned vbase = ((g - 1u) & kSM) * (unsigned)kSSlot;  // V of tile t − 1
        // FIRST: tile 0's scores came from a C = 0 chain (the previous item's last step, or the
        // kernel prologue); its exact row max becomes the item's running max
        // (m = 0 while every query's tile-0 max lies within ±kRescaleThr of 0: P <= 2^8 and the
        // largest P of a row >= 2^-8, no subtraction; else, rare, the exact max)
        if constexpr (FIRST) {
            cm = f32x16{};
            if (__builtin_amdgcn_ballot_w64(fabsf(c.mx) > kRescaleThr) != 0) {
                asm volatile("" ::: "memory");  // (a real branch)
                const float d = (c.mx < kEmptyMax) ? 0.f : c.mx;  // (never empty: nkv >= 1)
                cm = splat16(-d);
                c.s0 -= d;
                c.s1 -= d;
            }
        }
        // online-softmax decision for tile t (rare): the max moves now for tiles t, t + 1, ...;
        // O and l follow after tile t − 1's P·V (at the old max) is in
        float alpha = 1.f;
        const bool rescale = !MHA_STREAM_SPEC && !FIRST && c.rs;
        if (rescale) {
            asm volatile("" ::: "memory");  // (a real branch)
            const float d = fmaxf(c.mx, 0.f);
            alpha = __builtin_amdgcn_exp2f(-d);
            cm -= d;
            c.s0 -= d;
            c.s1 -= d;
        }
        // the refill: global tile g + L, the loader's current tile (of this item or a later one)
        const __amdgpu_buffer_rsrc_t rk_ = ld.k;
        const __amdgpu_buffer_rsrc_t rv_ = ld.v;
        const unsigned fm = m0w + ((g + (unsigned)L) & kSM) * (unsigned)kSSlot;
        const unsigned fso = (unsigned)ld.lt * (unsigned)kTileBytes + sow;
        auto dma = [&](int i) {  // piece i (< 2 kPW) of the refill: K w, (K w+4,) V w(, V w+4)
            const unsigned ho = (unsigned)((i % kPW) * NW * 1024);
            if (i < kPW) lds_dma16_s(fm + ho, dma_k, rk_, fso + ho);
            else lds_dma16_s(fm + (unsigned)kTileBytes + ho, dma_v, rv_, fso + ho);
        };

        // ---- vector work, a fixed order over the step's MFMA gaps ----
        auto exp_pair = [&](int e) {  // exponentials of tile t: elements 2e, 2e + 1
            f32x16& x = e < 8 ? c.s0 : c.s1;
            const int u = (2 * e) & 15;
            x[u] = __builtin_amdgcn_exp2f(x[u]);
            x[u + 1] = __builtin_amdgcn_exp2f(x[u + 1]);
            float a0 = x[u], a1 = x[u + 1];
            asm volatile("" : "+v"(a0), "+v"(a1));  // (tied in place: consumed only next step)
            x[u] = a0;
            x[u + 1] = a1;
        };
        auto cvt = [&](int q) {  // pack q (0..15): P group q / 4 = k-step (jj, ss), word q % 4
            const int grp = q >> 2, w = q & 3;
            const int jj = grp >> 1, ss = grp & 1;
            const f32x16& x = jj ? c.s1 : c.s0;
            unsigned v = __builtin_bit_cast(unsigned, f16x2{(f16)x[8 * ss + 2 * w], (f16)x[8 * ss + 2 * w + 1]});
            asm volatile("" : "+v"(v));
            u32x4 pw = __builtin_bit_cast(u32x4, pn[jj][ss]);
            pw[w] = v;
            pn[jj][ss] = __builtin_bit_cast(f16x8, pw);
        };
        float mt[4];
        auto maxk = [&](int k) {  // partial row max k of tile t + 1
            const f32x16& x = k < 2 ? n.s0 : n.s1;
            const int b = 8 * (k & 1);
            const float u = max3f(x[b], x[b + 1], x[b + 2]);
            const float v = max3f(x[b + 3], x[b + 4], x[b + 5]);
            float m = max3f(u, v, fmaxf(x[b + 6], x[b + 7]));
            asm volatile("" : "+v"(m));  // (a MASK step's run-time branch must not sink it)
            mt[k] = m;
        };
        // gap gi (0..19) of the step: an exponential pair, a pack of the group whose exponentials
        // are done, and (gaps 14..17, after the QKᵀ chains have drained) a partial row max
        auto fill = [&](int gi) {
            if (gi < 16) exp_pair(gi);
            if (gi >= 4 && gi < 20) cvt(gi - 4);
            if (NEEDMAX && gi >= 14 && gi < 18) maxk(gi - 14);
        };

        constexpr int SB = KIND == 0 ? 2 : (KIND == 1 || KIND == 4) ? 6 : KIND == 3 ? 16 : 10;  // (stamps)
        int gi = 0;
        // phase A: QKᵀ(t + 1), each gap an exponential pair (+ LDS reads, DMA pieces, packs). In
        // the LAST step, tile t + 1 is the next item's tile 0 (global tile g + 1, landed two
        // steps ago): its QKᵀ with the next item's Q (in qf by now) and C = 0, so the next item
        // starts at its FIRST step (the seam costs no separate prologue)
        read_k(kbase, 0);
        read_k(kbase, 1);
        const f32x16 zero16 = {};
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                {
                    f32x16& acc = kb ? n.s1 : n.s0;
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + kb], qf[s], s == 0 ? (LAST ? zero16 : cm) : acc,
                                                                 0, 0, 0);
                }
                fill(gi++);
                if (kb == 0) {
                    if (s < 2) read_k(kbase, s + 2);
                    if constexpr (PV) {
                        if (s == 1) read_v(vbase, 0);
                        if (s == 2) read_v(vbase, 1);
                    }
                    if (s < 2 * kPW) dma(s);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        SEG(SB);
        // phase B: Oᵀ += Vᵀ·Pᵀ(t − 1) and its row sums (each gap a pack, the rest of the
        // exponentials, the row max of tile t + 1)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int jj = k >> 1, ss = k & 1;
            if constexpr (PV) o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], pp[jj][ss], o0, 0, 0, 0);
            fill(gi++);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PV) o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], pp[jj][ss], o1, 0, 0, 0);
            fill(gi++);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PV) l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, pp[jj][ss], l_acc, 0, 0, 0);
            fill(gi++);
            __builtin_amdgcn_sched_barrier(0);
        }
        // P of tile t is consumed only by the next step: without this tie the compiler sinks the
        // exponentials and packs past the barrier, where no MFMA runs beside them
        asm volatile("" : "+v"(pn[0][0]), "+v"(pn[0][1]), "+v"(pn[1][0]), "+v"(pn[1][1]));
        SEG(SB + 1);
        if constexpr (MASK) {  // LAST: the next item's tile 0 (keys past its nkv)
            const int lim = LAST ? nxt.nkv : cur.nkv - kTileKV * (t + 1);  // keys of tile t + 1 (<= 0: none)
            if (lim < kTileKV) {  // (wave-uniform, rare: a partial or padding tile)
                asm volatile("" ::: "memory");
                mask_tile(n, lim);
                if constexpr (NEEDMAX) mt[0] = mt[1] = mt[2] = mt[3] = tree_max(n.s0, n.s1);
            }
        }
        if constexpr (NEEDMAX) n.mx = xhalf_max(fmaxf(max3f(mt[0], mt[1], mt[2]), mt[3]));
        if constexpr (!LAST && !MHA_STREAM_SPEC) n.rs = __builtin_amdgcn_ballot_w64(n.mx > kRescaleThr) != 0;
        if (rescale) {  // tile t − 1's P·V went in at the old max: O and l follow the new one
            asm volatile("" ::: "memory");
            o0 *= alpha;
            o1 *= alpha;
            l_acc *= alpha;
        }
        if constexpr (FIRST) {  // the previous item is complete: its output, then a fresh O and l
            if (prev) epilogue(prv_o, prv_q0, qbad_prv, prv_no);
            o0 = f32x16{};
            o1 = f32x16{};
            l_acc = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        SEG(SB + 2);
        // The step's wait and barrier. Loads (LDS-DMA pieces) complete in issue order; a count
        // below never lets an older store or Q piece stay in flight.
        if constexpr (NW == 4) {
            // this step's refill (tile t + 2, whose K the next step reads) has landed everywhere;
            // FIRST: the epilogue's stores and the next item's Q pieces too
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        } else if constexpr (BAR) {
            // (odd t) every refill up to the previous step's has landed (tiles up to t + 3: the K
            // read in the next two steps); this step's tile t + 4 stays in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPiece) : "memory");
            __builtin_amdgcn_s_barrier();
        } else if constexpr (FIRST) {
            if (!prev) {  // the workgroup's first item: the prologue's tile 2 is read next step
                // (in flight: the prologue's tile 3, the next item's Q pieces, this step's tile 4)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPiece + 4) : "memory");
                __builtin_amdgcn_s_barrier();
            }
        }
        SEG(SB + 3);
        ld_advance();
    };

    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    using K2 = std::integral_constant<int, 2>;
    using K3 = std::integral_constant<int, 3>;
    using K4 = std::integral_constant<int, 4>;
    using K5 = std::integral_constant<int, 5>;
    // Q fragments of an item's rows from the Q region (this wave's own rows: its own DMA, waited at
    // a step's end), scaled; the mask of non-finite query rows
    auto read_q = [&]() -> unsigned {
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = stream_scale_q(lds_read16(lds, q_base + k_addr[s]));
        return q_nonfinite_fix(qf);
    };
    // the first item's tile 0 (C = 0) and its exact row max, as a LAST step does for the others
    unsigned qbad = read_q();
    {
        f16x8 k0[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            k0[2 * s] = lds_read16(lds, k_addr[s]);
            k0[2 * s + 1] = lds_read16(lds, k_addr[s] + 4096u);
        }
        const f32x16 zero = {};
        sA.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0[0], qf[0], zero, 0, 0, 0);
        sA.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0[1], qf[0], zero, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < 4; ++s) {
            sA.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0[2 * s], qf[s], sA.s0, 0, 0, 0);
            sA.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(k0[2 * s + 1], qf[s], sA.s1, 0, 0, 0);
        }
        if (cur.nkv < kTileKV) mask_tile(sA, cur.nkv);
        sA.mx = xhalf_max(tree_max(sA.s0, sA.s1));
    }
    // tile 1 (read by the first FIRST step) landed everywhere
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((L - 2) * kPiece) : "memory");
    __builtin_amdgcn_s_barrier();
#ifdef MHA_STREAM_STAMPS
    SCLK(ck_t0);
    ck_sum[0] += ck_t0 - ck_pro;
#endif
    for (;;) {
        // the next item's Q rows of this wave, once its reads of the region have returned
        SEG(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_q(nxt);
        SEG(1);
        const int nt = cur.nt;
        const int nfull = cur.nkv / kTileKV;  // tiles without keys past nkv
        // step 0 (nt >= 2): with the previous item's last P·V and epilogue
        step(K0{}, 0, sA, sB, pB, pA);
#ifdef MHA_STREAM_STAMPS
        SCLK(ck_t1);
        ck_sum[1] += ck_t1 - ck_t0;
        ck_t0 = ck_t1;
#endif
        // middle steps in pairs (t odd, t + 1 even), no key past nkv in tiles t + 1, t + 2
        int t = 1;
        for (; t + 2 < nt && t + 2 < nfull; t += 2) {
            step(K1{}, t, sB, sA, pA, pB);
            step(K4{}, t + 1, sA, sB, pB, pA);
        }
#ifdef MHA_STREAM_STAMPS
        SCLK(ck_t1);
        ck_sum[2] += ck_t1 - ck_t0;
        ck_mid += (unsigned)(t - 1);
        ck_t0 = ck_t1;
#endif
        // the tail pairs: tiles past the full ones masked
        for (; t + 2 < nt; t += 2) {
            step(K2{}, t, sB, sA, pA, pB);
            step(K5{}, t + 1, sA, sB, pB, pA);
        }
        // the last step: beside tile nt − 2's P·V, the next item's tile 0 (its Q first: the
        // current item's fragments are no longer needed; NW 8 two-tile items: once this wave's DMA
        // of it, issued before the FIRST step, has landed); tile nt − 1's P·V and this item's
        // epilogue follow in the next item's FIRST step
        SEG(14);
        if (NW == 8 && nt == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned qbad_next = read_q();
        SEG(15);
        step(K3{}, t, sB, sA, pA, pB);
#ifdef MHA_STREAM_STAMPS
        SCLK(ck_t1);
        ck_sum[3] += ck_t1 - ck_t0;
        ck_items += 1;
        ck_t0 = ck_t1;
#endif
        prv_o = cur.o;
        prv_q0 = cur.q0;
        qbad_prv = qbad;
        prv_no = item_no++;
        prev = true;
        // ---- next item ----
        j += G;
        if (j >= je) break;
        gb += (unsigned)nt;
        cur = nxt;
        qbad = qbad_next;
        const bool more = j + G < je;
        nxt = stream_item<MULTI, OSZ, NW>(a, more ? j + G : j, more);
    }
    // SPEC's rare path: this wave's 32 rows of item jj, exactly — a running max per 64-key tile (exact
    // online softmax, rescale at every move) on the step's MFMA forms and fragment reads. Runs after
    // the workgroup's last barrier, when the ring is idle: the wave streams each K / V tile by LDS-DMA
    // into ring slot `wave` (its own: 16 KiB, the main loop's image layout and swizzles) and reads
    // the fragments as the steps do (read_k, read_v: ds_read_b128 / ds_read_b64_tr_b16); the next
    // tile's DMA is issued once the current one's fragments are in registers, so it lands under the
    // current tile's arithmetic. (Round 5's form loaded K fragments with 16-B and Vᵀ with 2-byte
    // global loads, one item ~90 us; profiles/r05/stream_spec_rare_cost.jsonl.)
    const unsigned xs_base = (unsigned)wave * (unsigned)kSSlot;
    const unsigned xs_m0 = (unsigned)__builtin_amdgcn_readfirstlane(lds0 + xs_base);
    auto exact_item = [&](int jj) {
        const StreamItem it = stream_item<MULTI, OSZ, NW>(a, jj, true);
        const StreamLoader kv = stream_kv<MULTI>(a, jj, true);
        auto load_tile = [&](int t) {  // pieces p = rows 8p..8p+7 of K and V (swizzles as issue_tile)
            const unsigned so = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(t * kTileBytes));
#pragma unroll
            for (int pc = 0; pc < 8; ++pc) {
                lds_dma16(xs_m0 + (unsigned)(pc * 1024), dma_kq(pc & 1), kv.k, so + (unsigned)(pc * 1024));
                lds_dma16(xs_m0 + (unsigned)(kTileBytes + pc * 1024), dma_v, kv.v, so + (unsigned)(pc * 1024));
            }
        };
        load_tile(0);
        const unsigned qrow = (unsigned)(it.q0 + 32 * wave + r);
#pragma unroll
        for (int s = 0; s < 4; ++s)
            qf[s] = stream_scale_q(__builtin_bit_cast(
                f16x8, __builtin_amdgcn_raw_buffer_load_b128(it.q, qrow * 128u + (unsigned)(2 * s + hh) * 16u, 0, 0)));
        const unsigned qb = q_nonfinite_fix(qf);
        float m = -INFINITY, l = 0.f;
        o0 = f32x16{};
        o1 = f32x16{};
        const int ntl = (it.nkv + kTileKV - 1) / kTileKV;
        for (int t = 0; t < ntl; ++t) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t landed (this wave's own DMA)
#pragma unroll
            for (int s = 0; s < 4; ++s) read_k(xs_base, s);
            read_v(xs_base, 0);
            read_v(xs_base, 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments in registers: the slot is free
            if (t + 1 < ntl) load_tile(t + 1);
            const unsigned kt = (unsigned)(t * kTileKV);
            StreamScores sc;
            const f32x16 zero = {};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                sc.s0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s], qf[s], s == 0 ? zero : sc.s0, 0, 0, 0);
                sc.s1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + 1], qf[s], s == 0 ? zero : sc.s1, 0, 0, 0);
            }
            if (it.nkv - (int)kt < kTileKV) mask_tile(sc, it.nkv - (int)kt);
            const float mn = fmaxf(m, xhalf_max(tree_max(sc.s0, sc.s1)));
            const float alpha = __builtin_amdgcn_exp2f(m - mn);  // (the first tile: exp2(-Inf) = 0)
            m = mn;
            float ls = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                sc.s0[i] = __builtin_amdgcn_exp2f(sc.s0[i] - m);
                sc.s1[i] = __builtin_amdgcn_exp2f(sc.s1[i] - m);
                ls += sc.s0[i] + sc.s1[i];
            }
            const auto lsw = __builtin_amdgcn_permlane32_swap(__float_as_uint(ls), __float_as_uint(ls), false, false);
            l = l * alpha + (__uint_as_float(lsw[0]) + __uint_as_float(lsw[1]));  // (own half + the other)
            o0 *= alpha;
            o1 *= alpha;
#pragma unroll
            for (int pj = 0; pj < 2; ++pj)
#pragma unroll
                for (int ps = 0; ps < 2; ++ps) {
                    const f32x16& x = pj ? sc.s1 : sc.s0;
                    f16x8 pk;
#pragma unroll
                    for (int e = 0; e < 8; ++e) pk[e] = (f16)x[8 * ps + e];
                    o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[pj][ps], pk, o0, 0, 0, 0);
                    o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[pj][ps], pk, o1, 0, 0, 0);
                }
        }
        l_acc = f32x4{l, l, l, l};
        epilogue(it.o, it.q0, qb, 63);
    };
    // flush: the last item's last tile (P in pB, V in its slot: no refill has reached it)
    {
        const unsigned vb_t = ((gb + (unsigned)cur.nt - 1u) & kSM) * (unsigned)kSSlot;
        read_v(vb_t, 0);
        read_v(vb_t, 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int jj = k >> 1, ss = k & 1;
            o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], pB[jj][ss], o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], pB[jj][ss], o1, 0, 0, 0);
            l_acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, pB[jj][ss], l_acc, 0, 0, 0);
        }
        epilogue(prv_o, prv_q0, qbad_prv, prv_no);
    }
    // drain: the loader's trailing (empty) pieces and the output stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (MHA_STREAM_SPEC) {
        // every wave is done with the ring (its flush read the last V image): slot w is wave w's
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#ifdef MHA_STREAM_RARE_ALL  // diagnostic: every item down the rare path
        dirty = ~0ull;
#endif
#ifdef MHA_STREAM_RARE_NONE  // diagnostic: the speculative output as it is
        dirty = 0;
#endif
        if (dirty) {  // (wave-uniform, rare) the exact rows of the marked items, over their stores
            asm volatile("" ::: "memory");
            const int j_first = jb + loc;
            for (int k = 0; j_first + k * G < je; ++k)
                if ((dirty >> (k < 63 ? k : 63)) & 1ull) exact_item(j_first + k * G);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
#ifdef MHA_STREAM_STAMPS
    unsigned long long ck_exit[2];
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_exit[0]), "=s"(ck_exit[1])::"memory");
    if (lane == 0 && a.stamps) {
        unsigned long long* dst = a.stamps + ((size_t)blockIdx.x * NW + wave) * kStreamStampSlots;
        for (int i_ = 0; i_ < 24; ++i_) dst[16 + i_] = sg[i_];
        for (int i_ = 0; i_ < 4; ++i_) dst[i_] = ck_sum[i_];
        dst[6] = ck_mid;
        dst[14] = ck_items;
        dst[8] = ck_entry[0];
        dst[9] = ck_entry[1];
        dst[10] = ck_exit[0];
        dst[11] = ck_exit[1];
        dst[12] = ck_pro;
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

// waves: 4 (128-row items) or 8 (256-row items); a.total_blocks counts items of that size
hipError_t launch_stream(const FwdArgs& a, int waves, bool out_f32, hipStream_t stream) {
    const int grid = stream_grid(a.total_blocks, waves);
    if (grid <= 0) return hipSuccess;
    if (waves == 8) return out_f32 ? launch_stream_t<float, 8>(a, grid, stream) : launch_stream_t<f16, 8>(a, grid, stream);
    return out_f32 ? launch_stream_t<float, 4>(a, grid, stream) : launch_stream_t<f16, 4>(a, grid, stream);
}

}  // namespace mha_hd64
