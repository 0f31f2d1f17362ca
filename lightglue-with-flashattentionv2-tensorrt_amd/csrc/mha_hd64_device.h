// mha_hd64_device.h — device-side types and helpers shared by the gfx950 attention kernels
// (mha_hd64_kernels.hip: the LDS-ring kernel and the split combine; mha_hd64_direct.hip: the
// single-pass kernel). Included by HIP translation units only.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mha_hd64_internal.h"

namespace mha_hd64 {
namespace {
typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
}  // namespace

constexpr float kScaleLog2 = 0.18033688011112042f;  // 0.125 * log2(e)
constexpr float kRescaleThr = 8.0f;                  // lazy-rescale threshold (log2 units)
constexpr int kTileKV = 64;                          // keys per LDS tile
constexpr int kTileBytes = kTileKV * kHeadDim * 2;   // 8 KiB fp16 tile

// One call of a launch (a launch carries up to kMaxCalls independent calls of any shapes: the
// grouped launcher runs self0+self1 or cross0->1+cross1->0 of a LightGlue layer as one launch).
constexpr int kMaxCalls = kGroupCalls;
constexpr int kMaxSplits = 16;  // KV splits per query group (combine loads them all in one round)
struct CallArgs {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    void* part_o;     // [bh][splits][nq][64] O_s / l_s in TOut precision (splits > 1 only)
    float2* part_ml;  // [bh][splits][nq] (m in log2 units, l)
    int nq;
    int nkv;
    int splits;
    int tiles_per_split;
    int qtiles;       // query blocks per (batch, head)
    int bh;           // batch * heads
    int block_begin;  // first block (in XCD-remapped order j) of this call
    int pad_;
};
struct FwdArgs {
    CallArgs c[kMaxCalls];
    int n_calls;
    int total_blocks;            // grid size (kept here so the first scalar-load round has it)
    unsigned long long* stamps;  // diagnostic builds only (MHA_STAMPS): 8 x u64 per workgroup
    // In-launch combine (non-null): one arrival ticket per query group, indexed by the group's
    // first block j; zero between launches (the last arriver resets its ticket).
    unsigned* tickets;
};

// Single-pass kernel (mha_hd64_direct.hip): 8 waves x tiles_per_wave 64-key tiles per 32-row block.
hipError_t launch_direct(const FwdArgs& a, int grid, int tiles_per_wave, bool out_f32, hipStream_t stream);
// 16-row single-pass kernel (mha_hd64_direct16.hip): 4 waves x 2*tiles_per_wave 64-key tiles.
// in_f32: fp32 Q/K/V rounded to fp16 inside the kernel (tiles_per_wave <= 2 only).
hipError_t launch_direct16(const FwdArgs& a, int grid, int tiles_per_wave, bool out_f32, hipStream_t stream,
                           bool in_f32 = false);
// Persistent streaming kernel (mha_hd64_stream.hip): 128-row items, all keys, fp16 Q/K/V;
// a.total_blocks = items (128-row blocks of every call, qtiles per call of 128 rows).
// waves = 4 (128-row items, two workgroups per CU) or 8 (256-row items, one per CU).
hipError_t launch_stream(const FwdArgs& a, int waves, bool out_f32, hipStream_t stream);
int stream_grid(int items, int waves);

namespace {
// Uniform (scalar) selection of call ci's arguments from the kernarg table (grouped launches).
__device__ __forceinline__ CallArgs pick_call(const FwdArgs& a, int ci) {
    CallArgs ca = a.c[0];
#pragma unroll
    for (int i = 1; i < kMaxCalls; ++i)
        if (ci == i) ca = a.c[i];
    return ca;
}

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
// Row max of the 32 scores of a lane as a v_max3_f32 tree (16 instructions: 11 + 4 + 1).
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ float tree_max(const f32x16& a, const f32x16& b) {
    float t[11];
#pragma unroll
    for (int i = 0; i < 5; ++i) t[i] = max3f(a[3 * i], a[3 * i + 1], a[3 * i + 2]);
    t[5] = max3f(a[15], b[0], b[1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) t[6 + i] = max3f(b[2 + 3 * i], b[3 + 3 * i], b[4 + 3 * i]);
    t[10] = fmaxf(b[14], b[15]);
    const float u0 = max3f(t[0], t[1], t[2]), u1 = max3f(t[3], t[4], t[5]);
    const float u2 = max3f(t[6], t[7], t[8]), u3 = fmaxf(t[9], t[10]);
    return fmaxf(max3f(u0, u1, u2), u3);
}
// LDS accesses through an explicit address-space-3 base and 32-bit byte offsets, so the
// compiler folds the compile-time part of every address into the DS instruction's offset field.
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) f16x8 lds_f16x8;

__device__ __forceinline__ f16x4 tr_read(lds_char* lds, unsigned byte_off) {
    const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds + byte_off));
    return __builtin_bit_cast(f16x4, v);
}
__device__ __forceinline__ f16x8 lds_read16(lds_char* lds, unsigned byte_off) {
    return *(lds_f16x8*)(lds + byte_off);
}
__device__ __forceinline__ void lds_write16(lds_char* lds, unsigned byte_off, f16x8 v) {
    *(lds_f16x8*)(lds + byte_off) = v;
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

// Diagnostic ablation switches (tools/ablate_build.sh builds each into lib/exp/; the shipped
// library defines none of them). Results of an ablated build are wrong by construction.
#ifndef MHA_ABL
#define MHA_ABL 0
#endif
#define ABL_NO_BARRIER 1
#define ABL_NO_REFILL 2
#define ABL_NO_EXP 4
#define ABL_NO_SOFTMAX 8
#define ABL_NO_PV 16
#define ABL_NO_QK 32
#define ABL_NO_GLOAD 64   // no K/V/Q global loads (LDS and Q hold garbage)
#define ABL_NO_STORE 128  // no output / partial stores
#define ABL_K_CONST 256   // K fragments from registers (no K LDS reads)
#define ABL_V_CONST 512   // V fragments from registers (no V LDS reads)
__device__ __forceinline__ void keep_live(const f16x8& x) { asm volatile("" ::"v"(x)); }

// In-kernel timestamps (diagnostic build -DMHA_STAMPS only): s_memtime after draining memory.
#ifdef MHA_STAMPS
#define STAMP(slot)                                                                                       \
    do {                                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                                \
        unsigned long long t_;                                                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                                \
        if (threadIdx.x == 0) a.stamps[blockIdx.x * 8 + (slot)] = t_;                                     \
    } while (0)
#else
#define STAMP(slot) \
    do {            \
    } while (0)
#endif

#ifndef MHA_ST_AUX
#define MHA_ST_AUX 0    // cache policy bits of the output stores (2 = nt, 16 = sc1)
#endif
#ifndef MHA_PART_AUX
#define MHA_PART_AUX 0  // cache policy bits of the split-partial stores
#endif

// Per-step phase clocks (diagnostic build -DMHA_STEPSTAMPS only): s_memtime at phase boundaries
// of every full loop step, summed per wave, waited for only at the next step's barrier.
#ifdef MHA_STEPSTAMPS
#define TCLK(var)                                  \
    do {                                           \
        __builtin_amdgcn_sched_barrier(0);         \
        var = __builtin_readcyclecounter();        \
        __builtin_amdgcn_sched_barrier(0);         \
    } while (0)
#else
#define TCLK(var) \
    do {          \
    } while (0)
#endif

#ifndef MHA_PINGPONG
#define MHA_PINGPONG 0  // measured neutral on the steady loop (vector-issue bound), and it makes the
                        // fp32-input 8-wave kernel spill: off by default, kept as a switch
#endif

constexpr float kMaskBias = -65504.f;  // fp16 lowest: a masked key's score, exp2 -> 0
constexpr float kEmptyMax = -30000.f;  // tile max below this: every key of the tile was masked

// Non-finite query rows. The matrix-pipe row sums multiply a partner query's fp16 P by a 0
// selector, and 0 * NaN = NaN would poison that partner's sum. So a query whose 64 dims hold a NaN
// or an Inf (spread over lanes l and l ^ 32 of the swapped QKᵀ layout: 4 x f16x8 each) has its Q
// fragments zeroed (its P stays finite) and its output row written as NaN, which is what the
// reference's math gives such a row. Returns the mask of the wave's 32 queries that are bad
// (wave-uniform). Integer tests only: the kernels are built with -fno-honor-nans.
__device__ __forceinline__ unsigned q_nonfinite_fix(f16x8 (&q)[4]) {
    // the sum of 32 finite fp16 values is finite (|s| <= 32 * 65504); four independent chains
    // (one per fragment), so the check is 4 dependent dot2 deep instead of 16
    float ps[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // (h2 built element-wise: a bit_cast of a vector element w[j] here compiles to w[0] four
        // times with this compiler)
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        ps[i] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            ps[i] = __builtin_amdgcn_fdot2(h2{q[i][2 * j], q[i][2 * j + 1]}, h2{(_Float16)1.f, (_Float16)1.f}, ps[i],
                                           false);
    }
    const float s = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    // the bits through an asm move: on a bit-cast float the compiler reads this test as an
    // fp-class test and, under -fno-honor-nans, drops its NaN half
    unsigned bits;
    asm volatile("v_mov_b32 %0, %1" : "=v"(bits) : "v"(s));
    const bool bad_lane = (bits & 0x7f800000u) == 0x7f800000u;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(bad_lane);
    const unsigned qm = (unsigned)m | (unsigned)(m >> 32);
    if (qm) {  // rare: zero the bad queries' fragments
        const bool bad = (qm >> (__lane_id() & 31)) & 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = bad ? f16x8{} : q[i];
    }
    return qm;
}
// 1 / l, or a quiet NaN for a bad query (opaque to the -fno-honor-nans folds)
__device__ __forceinline__ float inv_or_nan(float l, unsigned qm, int query) {
    unsigned b = __builtin_bit_cast(unsigned, 1.f / l);
    b = ((qm >> query) & 1u) ? 0x7fc00000u : b;
    float r = __builtin_bit_cast(float, b);
    asm volatile("" : "+v"(r));
    return r;
}

// Buffer loads (T8): a per-head descriptor whose record count is the head's byte size, so
// rows past nq / nkv read as zeros in hardware (no clamps, no 64-bit address math per load);
// the per-iteration key offset rides in the scalar soffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// One 1-KiB LDS-DMA piece (`buffer_load_dwordx4 … lds`: 64 lanes x 16 B from rs at voff + soff
// into LDS [m0, m0 + 1 KiB)) as inline asm, M0 written inside the statement. The compiler does not
// see this LDS write, so it adds no wait of its own: every read of the destination must follow the
// issuing wave's counted vmcnt (and a barrier for other waves' reads). (With the LDS-DMA builtin
// the compiler cannot tell the DMA's LDS writes from later ds_read_b64_tr_b16 reads of any address
// and drains EVERY DMA in flight, vmcnt(0), before the first transposing read.)
// m0 / soff are wave-uniform; readfirstlane pins values the compiler computed on the vector unit
// into the SGPRs the "s" constraints need. M0 is an explicit "{m0}" operand: the compiler writes
// it itself and knows the statement reads it (no value of its own is kept there across the asm).
// `s_nop 4` gives the 5 wait states a VMEM read of an SGPR (soffset, descriptor, M0) needs after a
// VALU (v_readfirstlane) or SALU wrote it — the compiler's hazard recognizer does not look inside
// the asm (as masked_load_dword below).
__device__ __forceinline__ void lds_dma16(unsigned m0, unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned soff) {
    m0 = __builtin_amdgcn_readfirstlane(m0);
    soff = __builtin_amdgcn_readfirstlane(soff);
    asm volatile(
        "s_nop 4\n\t"
        "buffer_load_dwordx4 %0, %1, %2 offen lds"
        :
        : "v"(voff), "s"(rs), "s"(soff), "{m0}"(m0)
        : "memory");
}
// The same with one wait state, for call sites whose M0, soffset and descriptor are SALU values
// (a SALU write of M0 needs 1 wait state before an LDS-DMA load; no VALU writes them): the hot
// refill of the streaming kernel. tools/check_dma_hazards.py audits every LDS-DMA load of the
// built library against both rules (tests/test_abi.py runs it).
__device__ __forceinline__ void lds_dma16_s(unsigned m0, unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned soff) {
    asm volatile(
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %0, %1, %2 offen lds"
        :
        : "v"(voff), "s"(rs), "s"(soff), "{m0}"(m0)
        : "memory");
}
// LDS byte address of a pointer into a __shared__ array (the value M0 takes)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
#ifndef MHA_DMA_ASM
#define MHA_DMA_ASM 1  // 0: the LDS-DMA builtin in the single-pass kernels (A/B hook)
#endif

// L2 prefetch for the single-pass kernels (issued by one wave per workgroup, before its own
// loads). A workgroup's DMA requests K of its first tiles at entry but V tile by tile once K(t)
// is in registers, and the later K tiles once K(0) has landed, so with inputs not already in the
// L2 those requests wait a second memory round trip. The `group` workgroups of one (batch, head)
// that the XCD-aware order puts on one XCD (consecutive query tiles) split that head's rows:
// workgroup r (= qtile % group) touches rows r + group·i, one dword per 128-B row, V always and K
// where the DMA asks late (row % WAVE_KEYS >= EARLY_KEYS). Only the fill matters (every row must
// be touched: every other row gains nothing, profiles/r02/prefetch_ab.txt); the returned dwords
// are kept live until the caller's first wait covers them (oldest loads of the wave). Masked
// lanes rather than out-of-range offsets: a full-wave load costs warm-input calls more.
//
// Register safety: the compiler does not track an asm load's pending VGPR write, so each load's
// destination must stay the SAME register from the asm statement to the covering wait. No load is
// therefore issued under a C-level branch (a join could merge the destination with its initial
// value through a copy and hand the original register to another value while the load is in
// flight): every statement is unconditional, the destination is a read-write ("+v") operand
// initialised to 0, and lane selection is an EXEC mask applied and restored inside the statement
// (waves other than the prefetching one run it with an empty mask).
struct L2Prefetch {
    unsigned k[2] = {0u, 0u}, v[2] = {0u, 0u};
};
// workgroups of one (batch, head) per XCD in the XCD-aware order (0: too few to split the rows)
__device__ __forceinline__ int prefetch_group(int total_blocks, int qtiles) {
    const int n = min(total_blocks >> 3, qtiles);
    return n >= 32 ? 32 : (n >= 16 ? 16 : 0);
}
// buffer_load_dword into `dst` on the lanes of `mask` only (EXEC saved and restored in the same
// statement). `s_nop 4`: the descriptor / mask SGPRs may come straight from a VALU write
// (readfirstlane, the ballot's v_cmp), which a VMEM / exec read must not follow within 5 states.
__device__ __forceinline__ void masked_load_dword(unsigned& dst, unsigned off, __amdgpu_buffer_rsrc_t rs,
                                                  unsigned long long mask) {
    unsigned long long saved;
    asm volatile(
        "s_nop 4\n\t"
        "s_and_saveexec_b64 %1, %4\n\t"
        "buffer_load_dword %0, %2, %3, 0 offen\n\t"
        "s_mov_b64 exec, %1"
        : "+v"(dst), "=&s"(saved)
        : "v"(off), "s"(rs), "s"(mask)
        : "memory", "scc");
}
// `active`: wave-uniform (the prefetching wave); the other waves issue empty-mask statements.
template <int WAVE_KEYS, int EARLY_KEYS>
__device__ __forceinline__ void l2_prefetch(L2Prefetch& pf, __amdgpu_buffer_rsrc_t k_rs, __amdgpu_buffer_rsrc_t v_rs,
                                            int nkv, int qtile, int group, int lane, bool active) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {  // nkv <= 2048: at most 128 rows per workgroup
        const int g = group > 0 ? group : 1;
        const int row = (qtile & (g - 1)) + g * (lane + 64 * c);
        const unsigned off = (unsigned)row * 128u;
        const bool live = active && group > 0 && row < nkv;
        const unsigned long long mk =
            __builtin_amdgcn_ballot_w64(EARLY_KEYS < WAVE_KEYS && live && row % WAVE_KEYS >= EARLY_KEYS);
        const unsigned long long mv = __builtin_amdgcn_ballot_w64(live);
        masked_load_dword(pf.k[c], off, k_rs, mk);
        masked_load_dword(pf.v[c], off, v_rs, mv);
    }
}
__device__ __forceinline__ void l2_prefetch_done(L2Prefetch& pf) {
    asm volatile("" : "+v"(pf.k[0]), "+v"(pf.k[1]), "+v"(pf.v[0]), "+v"(pf.v[1])::"memory");
}
// 8 consecutive output values (dims c8..c8+7 of one row) as one (f16) or two (f32) 16-B stores.
template <typename T, int AUX>
__device__ __forceinline__ void store8(__amdgpu_buffer_rsrc_t rs, unsigned voff, f32x4 a, f32x4 b) {
    if constexpr (sizeof(T) == 2) {
        const f16x8 h = f16x8{(f16)a[0], (f16)a[1], (f16)a[2], (f16)a[3], (f16)b[0], (f16)b[1], (f16)b[2], (f16)b[3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), rs, voff, 0, AUX);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rs, voff, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), rs, voff + 16, 0, AUX);
    }
}
__device__ __forceinline__ void bload8(Raw8<f16>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    r.x = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
__device__ __forceinline__ void bload8(Raw8<float>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    r.a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
    r.b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16, soff, 0));
}
// cache-policy bits of the buffer intrinsics' aux operand: sc1 (write-through store / L1-bypassing
// load; the inter-workgroup hand-off form of MI355X_MICROARCH.md)
constexpr int kSC1 = 16;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int AUX>
__device__ __forceinline__ void bload8_aux(Raw8<f16>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff) {
    r.x = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ void bload8_aux(Raw8<float>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff) {
    r.a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, AUX));
    r.b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16, 0, AUX));
}
// One split's term of the split merge, O += w_s·Ô_s, L += w_s with w_s = l_s·2^(m_s - M):
// shared by the combine kernel and the in-launch combine with contraction off, so both forms
// round identically (bitwise-equal outputs whichever runs).
__device__ __forceinline__ float split_weight(float2 ml, float M) {
#pragma clang fp contract(off)
    return (ml.x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ml.x - M) * ml.y;
}
__device__ __forceinline__ void split_accumulate(f32x4& acc, float w, f32x4 v) {
#pragma clang fp contract(off)
    acc = acc + w * v;
}
// (an fp32 product, then the output rounding: never fused into one mixed-precision FMA)
__device__ __forceinline__ f32x4 split_scale(f32x4 acc, float inv) {
#pragma clang fp contract(off)
    return acc * inv;
}
// 4-dim forms (workgroups with more threads than (row, 8-dim) items split rows into 16 chunks)
template <typename T> struct Raw4;
template <> struct Raw4<f16> { f16x4 x; };
template <> struct Raw4<float> { f32x4 a; };
template <int AUX>
__device__ __forceinline__ void bload4_aux(Raw4<f16>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff) {
    r.x = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ void bload4_aux(Raw4<float>& r, __amdgpu_buffer_rsrc_t rs, unsigned voff) {
    r.a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, AUX));
}
__device__ __forceinline__ f32x4 raw4_to_f32(const Raw4<f16>& r) {
    return f32x4{(float)r.x[0], (float)r.x[1], (float)r.x[2], (float)r.x[3]};
}
__device__ __forceinline__ f32x4 raw4_to_f32(const Raw4<float>& r) { return r.a; }
template <typename T, int AUX>
__device__ __forceinline__ void store4b(__amdgpu_buffer_rsrc_t rs, unsigned voff, f32x4 a) {
    if constexpr (sizeof(T) == 2) {
        const f16x4 h = f16x4{(f16)a[0], (f16)a[1], (f16)a[2], (f16)a[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), rs, voff, 0, AUX);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rs, voff, 0, AUX);
    }
}
// DPT dims of one row (DPT = 8: a0 = dims 0-3, a1 = 4-7; DPT = 4: a0 only)
template <typename T, int DPT, int AUX>
__device__ __forceinline__ void store_dims(__amdgpu_buffer_rsrc_t rs, unsigned voff, f32x4 a0, f32x4 a1) {
    if constexpr (DPT == 8) store8<T, AUX>(rs, voff, a0, a1);
    else store4b<T, AUX>(rs, voff, a0);
}
__device__ __forceinline__ void raw8_to_f32(const Raw8<f16>& r, f32x4& lo, f32x4& hi) {
    lo = f32x4{(float)r.x[0], (float)r.x[1], (float)r.x[2], (float)r.x[3]};
    hi = f32x4{(float)r.x[4], (float)r.x[5], (float)r.x[6], (float)r.x[7]};
}
__device__ __forceinline__ void raw8_to_f32(const Raw8<float>& r, f32x4& lo, f32x4& hi) {
    lo = r.a;
    hi = r.b;
}
}  // namespace
}  // namespace mha_hd64
