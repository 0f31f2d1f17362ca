// Microbenchmark (diagnostic, not shipped): the throughput kernel's steady-state step, built up one
// ingredient at a time (find where the structure loses against bare MFMA).
//
// One wave = RB query blocks of 32 rows (RB = 1: 32 rows, two workgroups per CU / two waves per
// SIMD; RB = 2: 64 rows, one wave per SIMD with K and V fragments shared by both blocks). A step is
// one 64-key tile with the deferred-PV pipeline of csrc/mha_hd64_stream.hip:
//   matrix pipe : QKᵀ of tile t+1 (8·RB v_mfma_f32_32x32x16_f16, C = −m)
//                 Oᵀ += Vᵀ·Pᵀ of tile t−1 (8·RB) + row sums (4·RB v_mfma_f32_16x16x32_f16)
//   vector pipe : exp2 + fp16 pack of tile t (32·RB v_exp_f32, 16·RB v_cvt_pk), row max of tile t+1
// Ingredients (bit flags, template parameter F):
//   1 EXP   the exponentials            2 CVT  the fp16 packs of P
//   4 MAX   the row max of tile t+1 + permlane + wave-uniform rescale check (never taken)
//   8 RSUM  the row-sum MFMAs (else: no row sums at all)
//  16 LDSK  K fragments from LDS (8 ds_read_b128 / step; else registers stand in)
//  32 LDSV  V fragments from LDS (16 ds_read_b64_tr_b16 / step)
//  64 DMA   4 LDS-DMA pieces (1 KiB) per wave and step from an L2-resident buffer, counted vmcnt
// 128 BAR   one s_barrier per step (the workgroup's 4 waves)
// 256 SCHK  with MAX off: the overflow check on the tile's row sum instead (1 v_cmp + ballot)
// 1024 BAR2 the barrier every second step only    2048 WAIT0 wait for this step's own pieces (vmcnt(0),
//           one step of DMA lead, as the round-3 streaming kernel) instead of the previous step's
// NW = waves per workgroup: 4 (two workgroups per CU) or 8 (one per CU, two waves per SIMD sharing
//           the K/V stream: 2 DMA pieces per wave and step)
// 4096 ROT  (NW = 8) waves 4..7 run each step's phase B before its phase A: the two waves of a SIMD
//           (w, w + 4) are in different phases between barriers
// 8192 VSUM  row sums on the vector pipe instead of RSUM's MFMAs: 16 v_dot2c_f32_f16 of the packed P
//           per step (four chains), two beside each P·V MFMA
// 512 POLY   half of the exponentials as a degree-3 exp2 polynomial on the
//           packed-FMA path (v_pk_fma_f32 + exponent insert) instead of v_exp_f32
// Prints per variant: µs per launch (HIP events, median of 5 launches), TFLOP/s (the step's useful
// QKᵀ + PV FLOPs), cycles per wave-step (s_memtime), the in-kernel clock (s_memtime /
// s_memrealtime) and the matrix-pipe share: MFMA cycles per SIMD-step ÷ cycles per step.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans -I<csrc> \
//         tools/mb_step.hip -o tools/mb_step && tools/mb_step [variant-substring]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "mha_hd64_device.h"

using namespace mha_hd64;

enum : int { EXP = 1, CVT = 2, MAX = 4, RSUM = 8, LDSK = 16, LDSV = 32, DMA = 64, BAR = 128, SCHK = 256, POLY = 512,
              BAR2 = 1024, WAIT0 = 2048, ROT = 4096, VSUM = 8192 };
constexpr int ITER = 1024;  // steps per wave (2 x this many tiles per loop trip)
constexpr int kSlot = 2 * kTileBytes;
constexpr int kSlots = 4;
constexpr int kLds = kSlots * kSlot;  // 64 KiB

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// exp2 of two values on the packed-FMA path: x = n + f (n = round(x), f in [-0.5, 0.5]),
// 2^f by a degree-3 minimax polynomial (rel. error ~1e-4: below the fp16 rounding of P), 2^n by
// an integer add into the exponent field. Inputs <= 0 (scores minus the running max) and > -126.
__device__ __forceinline__ f32x2 exp2_poly2(f32x2 x) {
    const f32x2 magic = {12582912.f, 12582912.f};  // 1.5 * 2^23: round to nearest integer
    f32x2 t = x + magic;
    f32x2 n = t - magic;
    f32x2 f = x - n;
    f32x2 p = f32x2{0.0555041f, 0.0555041f};
    p = p * f + f32x2{0.2402265f, 0.2402265f};
    p = p * f + f32x2{0.6931472f, 0.6931472f};
    p = p * f + f32x2{1.0f, 1.0f};
    const unsigned t0 = __builtin_bit_cast(unsigned, t[0]) << 23, t1 = __builtin_bit_cast(unsigned, t[1]) << 23;
    return f32x2{__builtin_bit_cast(float, __builtin_bit_cast(unsigned, p[0]) + t0),
                 __builtin_bit_cast(float, __builtin_bit_cast(unsigned, p[1]) + t1)};
}

template <int RB, int NW, int F>
__global__ __launch_bounds__(64 * NW, RB == 1 ? 2 : 1) void kern(const f16* src, float* out, unsigned long long* clk) {
    __shared__ __attribute__((aligned(1024))) char smem[kLds];
    lds_char* const lds = (lds_char*)smem;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;

    // LDS filled with random fp16 from the source (so the MFMAs see random operands)
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, 1u << 20);
    for (int off = tid * 16; off < kLds; off += 64 * NW * 16)
        lds_write16(lds, off, __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)off, 0, 0)));
    __syncthreads();

    unsigned k_addr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) k_addr[s] = (unsigned)k_off(r, 2 * s + hh);
    const int g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const int vb = (qq >> 1) & 1;
    const int v_lane = 128 * (4 * hh + qq) + 16 * (2 * (g16 & 1) + (pp >> 1)) + 8 * (pp & 1);
    const unsigned v_addr0 = (unsigned)(v_lane + 64 * vb + kTileBytes);
    const unsigned v_addr1 = (unsigned)(v_lane + 64 * (1 - vb) + kTileBytes);
    const unsigned dma_k = (unsigned)((lane >> 3) * 128 + (((lane & 7) ^ ((4 * (wave & 1) + (lane >> 4)) & 7)) << 4));
    const unsigned m0w = (unsigned)__builtin_amdgcn_readfirstlane(lds0 + (unsigned)wave * 1024u);
    const unsigned sow = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)wave * 1024u);
    const f16 sel = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? (f16)1.f : (f16)0.f;
    const f16x8 a_sum = f16x8{sel, sel, sel, sel, sel, sel, sel, sel};

    // Q fragments (scaled as the kernels do), per block b
    f16x8 qf[RB][4];
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            f16x8 x = lds_read16(lds, k_addr[s] + 4096u * b);
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = (f16)((float)x[i] * 0.18f);
            qf[b][s] = x;
        }
    f32x16 cm[RB];
#pragma unroll
    for (int b = 0; b < RB; ++b) cm[b] = splat16(-3.f);
    f32x16 o[RB][2] = {};
    f32x4 l[RB] = {};
    float vs[RB][4] = {};
    f32x16 sA[RB][2], sB[RB][2];
    f16x8 pA[RB][4], pB[RB][4];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
        sA[b][0] = sA[b][1] = sB[b][0] = sB[b][1] = splat16(-1.f);
#pragma unroll
        for (int k = 0; k < 4; ++k) pA[b][k] = pB[b][k] = qf[b][k];
    }
    float mrun = -1e30f;
    unsigned rescales = 0;
    int tile = 0;

    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();

    // one step; slot S: tile t+1's K (read), tile t-1's V (read), refill slot (S+2)%4
    auto step = [&](auto slot_c, f32x16 (&c)[RB][2], f32x16 (&n)[RB][2], const f16x8 (&pp_)[RB][4], f16x8 (&pn)[RB][4]) {
        constexpr int S = decltype(slot_c)::value;
        constexpr int NSL = (S + 1) % kSlots, VSL = (S + kSlots - 1) % kSlots, FSL = (S + 2) % kSlots;
        constexpr int G = 20 * RB;  // MFMA gaps per step (with the row sums; fewer without)
        // ---- vector work items, issued in a fixed order over the gaps ----
        auto exp_pair = [&](int e) {  // elements 2e, 2e+1 of tile t (e < 16 RB)
            if (!(F & EXP)) return;
            const int b = e / 16, ee = e % 16;
            f32x16& x = ee < 8 ? c[b][0] : c[b][1];
            const int u = (2 * ee) & 15;
            if ((F & POLY) && (e & 1)) {
                const f32x2 y = exp2_poly2(f32x2{x[u], x[u + 1]});
                x[u] = y[0];
                x[u + 1] = y[1];
            } else {
                x[u] = __builtin_amdgcn_exp2f(x[u]);
                x[u + 1] = __builtin_amdgcn_exp2f(x[u + 1]);
            }
            float a0 = x[u], a1 = x[u + 1];
            asm volatile("" : "+v"(a0), "+v"(a1));
            x[u] = a0;
            x[u + 1] = a1;
        };
        auto cvt = [&](int q) {  // pack q (< 16 RB): P group q/4 (block b, k-step k), word q%4
            if (!(F & CVT)) return;
            const int b = q / 16, g = (q / 4) % 4, w = q % 4;
            const int jj = g >> 1, ss = g & 1;
            const f32x16& x = jj ? c[b][1] : c[b][0];
            unsigned v = __builtin_bit_cast(unsigned, h2{(f16)x[8 * ss + 2 * w], (f16)x[8 * ss + 2 * w + 1]});
            asm volatile("" : "+v"(v));
            u32x4 pw = __builtin_bit_cast(u32x4, pn[b][g]);
            pw[w] = v;
            pn[b][g] = __builtin_bit_cast(f16x8, pw);
        };
        float mt[RB][4];
        auto maxk = [&](int m) {  // partial row max m (< 4 RB) of tile t+1
            if (!(F & MAX)) return;
            const int b = m / 4, k = m % 4;
            const f32x16& x = k < 2 ? n[b][0] : n[b][1];
            const int bb = 8 * (k & 1);
            const float u = max3f(x[bb], x[bb + 1], x[bb + 2]);
            const float v = max3f(x[bb + 3], x[bb + 4], x[bb + 5]);
            mt[b][k] = max3f(u, v, fmaxf(x[bb + 6], x[bb + 7]));
        };
        // gap g's fillers: one exp pair; one pack (of the group whose exps are done); one partial max
        auto fill = [&](int g) {
            if (g < 16 * RB) exp_pair(g);
            if (g >= 4 && g - 4 < 16 * RB) cvt(g - 4);
            const int m0 = G - 4 * RB - 2;  // maxes in the last gaps of phase B (after QKᵀ)
            if (g >= m0 && g - m0 < 4 * RB) maxk(g - m0);
        };
        f16x8 kf[8];
        auto read_k = [&](int s) {
            if (F & LDSK) {
                kf[2 * s] = lds_read16(lds, (unsigned)NSL * kSlot + k_addr[s]);
                kf[2 * s + 1] = lds_read16(lds, (unsigned)NSL * kSlot + k_addr[s] + 4096u);
            } else {  // (through an empty asm: loop-invariant operands would let the compiler hoist the MFMAs)
                kf[2 * s] = qf[0][s];
                kf[2 * s + 1] = qf[0][(s + 1) & 3];
                asm volatile("" : "+v"(kf[2 * s]), "+v"(kf[2 * s + 1]));
            }
        };
        f16x8 vfa[2][2], vfb[2][2];
        auto read_v = [&](int jj) {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                if (F & LDSV) {
                    const unsigned rowc = (unsigned)VSL * kSlot + 128u * (32 * jj + 16 * ss);
                    vfa[jj][ss] = cat8(tr_read(lds, v_addr0 + rowc), tr_read(lds, v_addr0 + rowc + 8 * 128));
                    vfb[jj][ss] = cat8(tr_read(lds, v_addr1 + rowc), tr_read(lds, v_addr1 + rowc + 8 * 128));
                } else {
                    vfa[jj][ss] = qf[0][(jj + ss) & 3];
                    vfb[jj][ss] = qf[0][(jj + ss + 1) & 3];
                    asm volatile("" : "+v"(vfa[jj][ss]), "+v"(vfb[jj][ss]));
                }
            }
        };
        auto dma = [&](int i) {  // piece i (0..4·4/NW): K w, K w+4, V w, V w+4 (NW = 8: K w, V w)
            if (!(F & DMA) || i >= 16 / NW) return;
            const int kv = NW == 8 ? i : i >> 1, hi = NW == 8 ? 0 : i & 1;
            const unsigned m = m0w + (unsigned)(FSL * kSlot + kv * kTileBytes + hi * 4096);
            const unsigned so = (unsigned)((tile & 63) * kSlot) + sow + (unsigned)(hi * 4096 + kv * kTileBytes);
            lds_dma16(m, dma_k, rs, so);
        };

        int g = 0;
        // phase A: QKᵀ(t+1)
        auto phase_a = [&](bool rv) {
        read_k(0);
        read_k(1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int b = 0; b < RB; ++b)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) {
                    n[b][kb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[2 * s + kb], qf[b][s], s == 0 ? cm[b] : n[b][kb], 0, 0, 0);
                    fill(g++);
                    if (b == 0 && kb == 0) {
                        if (s < 2) read_k(s + 2);
                        if (rv && s == 1) read_v(0);
                        if (rv && s == 2) read_v(1);
                        dma(s);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
        }
        };
        // phase B: Oᵀ += Vᵀ·Pᵀ(t−1) and row sums
        auto phase_b = [&]() {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int jj = k >> 1, ss = k & 1;
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                o[b][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfa[jj][ss], pp_[b][k], o[b][0], 0, 0, 0);
                fill(g++);
                __builtin_amdgcn_sched_barrier(0);
                if (F & VSUM) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        vs[b][k] = __builtin_amdgcn_fdot2(h2{pp_[b][k][2 * j], pp_[b][k][2 * j + 1]}, h2{(f16)1.f, (f16)1.f},
                                                          vs[b][k], false);
                }
                o[b][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vfb[jj][ss], pp_[b][k], o[b][1], 0, 0, 0);
                fill(g++);
                if (F & VSUM) {
#pragma unroll
                    for (int j = 2; j < 4; ++j)
                        vs[b][k] = __builtin_amdgcn_fdot2(h2{pp_[b][k][2 * j], pp_[b][k][2 * j + 1]}, h2{(f16)1.f, (f16)1.f},
                                                          vs[b][k], false);
                }
                __builtin_amdgcn_sched_barrier(0);
                if (F & RSUM) {
                    l[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_sum, pp_[b][k], l[b], 0, 0, 0);
                    fill(g++);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        };
        if ((F & ROT) && wave >= NW / 2) {
            read_v(0);  // (phase B first: its V fragments before it)
            read_v(1);
            phase_b();
            phase_a(false);
        } else {
            phase_a(true);
            phase_b();
        }
        while (g < G) fill(g++);  // (without RSUM: the remaining fillers after the last MFMA)
        asm volatile("" : "+v"(pn[0][0]), "+v"(pn[0][1]), "+v"(pn[0][2]), "+v"(pn[0][3]));
        if (F & MAX) {
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                const float mx = xhalf_max(fmaxf(max3f(mt[b][0], mt[b][1], mt[b][2]), mt[b][3]));
                mrun = fmaxf(mrun, mx);
            }
            if (__builtin_amdgcn_ballot_w64(mrun > 1e30f) != 0) {  // never: the rescale branch
                asm volatile("" ::: "memory");
                ++rescales;
#pragma unroll
                for (int b = 0; b < RB; ++b) {
                    o[b][0] *= 0.5f;
                    cm[b] -= 1.f;
                }
            }
        } else if (F & SCHK) {
            bool big = false;
#pragma unroll
            for (int b = 0; b < RB; ++b) big |= l[b][0] > 1e30f;
            if (__builtin_amdgcn_ballot_w64(big) != 0) {
                asm volatile("" ::: "memory");
                ++rescales;
#pragma unroll
                for (int b = 0; b < RB; ++b) {
                    o[b][0] *= 0.5f;
                    cm[b] -= 1.f;
                }
            }
        }
        if (F & DMA) {
            if ((F & WAIT0) || NW == 8) {
                if (F & WAIT0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            }
        }
        if ((F & BAR) && (!(F & BAR2) || (S & 1))) __builtin_amdgcn_s_barrier();
        ++tile;
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;
    for (int it = 0; it < ITER / 4; ++it) {
        step(C0{}, sA, sB, pB, pA);
        step(C1{}, sB, sA, pA, pB);
        step(C2{}, sA, sB, pB, pA);
        step(C3{}, sB, sA, pA, pB);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float acc = (float)rescales;
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc += o[b][0][i] + o[b][1][i] + sA[b][0][i] + sB[b][1][i];
        acc += l[b][0] + l[b][1] + vs[b][0] + vs[b][1] + vs[b][2] + vs[b][3];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += (float)pA[b][k][0] + (float)pB[b][k][1];
    }
    out[blockIdx.x * 64 * NW + tid] = acc;
    if (tid == 0) {
        clk[blockIdx.x * 2] = t1 - t0;
        clk[blockIdx.x * 2 + 1] = r1 - r0;
    }
}

struct Res {
    double us, tflops, cyc_step, ghz, pipe;
};

template <int RB, int NW, int F>
Res run(const f16* src, float* out, unsigned long long* clk, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((kern<RB, NW, F>), dim3(grid), dim3(64 * NW), 0, 0, src, out, clk);
    std::vector<float> ms(5);
    for (auto& m : ms) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((kern<RB, NW, F>), dim3(grid), dim3(64 * NW), 0, 0, src, out, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&m, e0, e1);
    }
    std::sort(ms.begin(), ms.end());
    std::vector<unsigned long long> h(2 * grid);
    hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < grid; ++i) {
        cyc += h[2 * i];
        rt += h[2 * i + 1];
    }
    Res res;
    res.ghz = cyc / (rt / 100e6) / 1e9;
    res.us = ms[2] * 1e3;
    const double flops = 524288.0 * RB * ITER * NW * grid;  // per wave-step: 2 x (32 RB x 64 x 64) x 2
    res.tflops = flops / (res.us * 1e-6) / 1e12;
    res.cyc_step = cyc / grid / ITER;
    const int wps = grid * NW / 1024;  // waves per SIMD
    const double mfma_cyc = RB * (16 * 32 + ((F & RSUM) ? 4 * 16 : 0));
    res.pipe = mfma_cyc * wps / res.cyc_step;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return res;
}

template <int RB, int NW, int F>
void row(const char* name, const char* filt, const f16* src, float* out, unsigned long long* clk) {
    if (filt && !strstr(name, filt)) return;
    const int grid = RB == 1 ? 2048 / NW : 256;
    const Res a = run<RB, NW, F>(src, out, clk, grid);
    printf("%-34s RB=%d NW=%d grid %3d: %8.1f us  %7.1f TFLOP/s (%.3f of 2.5 PF)  %6.0f cyc/wave-step  %.2f GHz  pipe %.2f\n",
           name, RB, NW, grid, a.us, a.tflops, a.tflops / 2500.0, a.cyc_step, a.ghz, a.pipe);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const char* filt = argc > 1 ? argv[1] : nullptr;
    f16* src;
    float* out;
    unsigned long long* clk;
    hipMalloc(&src, 1 << 20);
    hipMalloc(&out, 1024 * 512 * 4);
    hipMalloc(&clk, 512 * 16);
    std::vector<f16> h(1 << 19);
    unsigned s = 12345;
    for (auto& x : h) {
        s = s * 1664525u + 1013904223u;
        x = (f16)(((s >> 8) & 0xffff) / 65536.0f * 2.0f - 1.0f);
    }
    hipMemcpy(src, h.data(), 1 << 20, hipMemcpyHostToDevice);
    constexpr int ALL = EXP | CVT | MAX | RSUM | LDSK | LDSV | DMA | BAR;
    constexpr int VEC = RSUM | EXP | CVT | MAX;
    constexpr int VECS = RSUM | EXP | CVT | SCHK;
    for (int rep = 0; rep < 2; ++rep) {
        row<1, 4, 0>("a  mfma only (no row sums)", filt, src, out, clk);
        row<1, 4, RSUM>("b  mfma + row sums", filt, src, out, clk);
        row<1, 4, RSUM | EXP>("c  + exp", filt, src, out, clk);
        row<1, 4, RSUM | EXP | CVT>("d  + cvt", filt, src, out, clk);
        row<1, 4, VEC>("e  + max (all vector work)", filt, src, out, clk);
        row<1, 4, VECS>("e' sum check instead of max", filt, src, out, clk);
        row<1, 4, VEC | LDSK | LDSV>("f  + LDS fragment reads", filt, src, out, clk);
        row<1, 4, VEC | LDSK | LDSV | DMA>("g  + DMA refill", filt, src, out, clk);
        row<1, 4, VEC | LDSK | LDSV | DMA | BAR>("h  + barrier (full step)", filt, src, out, clk);
        row<1, 4, VEC | LDSK | LDSV | DMA | BAR | WAIT0>("h0 full step, 1-step DMA lead", filt, src, out, clk);
        row<1, 4, VECS | LDSK | LDSV | DMA | BAR>("h' full step, sum check", filt, src, out, clk);
        row<1, 4, VECS | LDSK | LDSV | DMA | BAR | BAR2>("h2 sum check, barrier / 2 steps", filt, src, out, clk);
        row<1, 4, VEC | LDSK | LDSV | DMA | BAR | POLY>("i  full step, half exps poly", filt, src, out, clk);
        row<1, 8, VEC | LDSK | LDSV | DMA | BAR>("j  8 waves, full step", filt, src, out, clk);
        row<1, 8, VECS | LDSK | LDSV | DMA | BAR>("j' 8 waves, sum check", filt, src, out, clk);
        row<1, 8, VECS | LDSK | LDSV | DMA | BAR | BAR2>("j2 8 waves, sum check, bar / 2", filt, src, out, clk);
        row<1, 8, VECS | LDSK | LDSV | DMA>("j3 8 waves, sum check, no bar", filt, src, out, clk);
        row<1, 8, VEC | LDSK | LDSV | DMA | BAR | BAR2>("j4 8 waves, full step, bar / 2 (the kernel's form)", filt, src, out, clk);
        row<1, 8, (VEC & ~RSUM) | VSUM | LDSK | LDSV | DMA | BAR | BAR2>("j5 8 waves, bar / 2, VALU row sums", filt, src, out, clk);
        row<1, 4, (VEC & ~RSUM) | VSUM | LDSK | LDSV | DMA | BAR>("h3 full step, VALU row sums", filt, src, out, clk);
        row<1, 4, (VEC & ~RSUM) | VSUM>("e3 all vector work, VALU row sums", filt, src, out, clk);
        row<1, 8, VEC | LDSK | LDSV | DMA | BAR | ROT>("k  8 waves, full step, rotated", filt, src, out, clk);
        row<1, 8, VECS | LDSK | LDSV | DMA | BAR | ROT>("k' 8 waves, sum check, rotated", filt, src, out, clk);
        row<1, 8, VECS | LDSK | LDSV | DMA | BAR | BAR2 | ROT>("k2 8 waves, sum check, bar / 2, rot", filt, src, out, clk);
    }
    return 0;
}
