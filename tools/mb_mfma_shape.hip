// Microbenchmark (diagnostic, not shipped): does the attention step's MFMA shape change the clock
// the chip holds? The same FLOPs and the same vector work per FLOP (2 v_exp_f32 + 1 v_cvt_pk +
// 1 v_max3 per 8192 MACs, the head_dim-64 softmax density) issued beside either
// v_mfma_f32_32x32x16_f16 (one per group) or v_mfma_f32_16x16x32_f16 (two per group), random
// fp16 operands, 2 waves per SIMD (512 threads, 2 workgroups of 256 per CU via the grid), many
// workgroups, a long loop. Prints wall time per launch (HIP events) and TFLOP/s, and the
// in-kernel clock from s_memtime / s_memrealtime.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_mfma_shape.hip -o tools/mb_mfma_shape && tools/mb_mfma_shape
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 4096;

template <int SHAPE, int FILL>  // SHAPE 32: 32x32x16, 16: 16x16x32; FILL 0: MFMA only, 1: softmax-density fillers
__global__ __launch_bounds__(256) void kern(const float* in, float* out, unsigned long long* clk) {
    const int lane = threadIdx.x & 63;
    f16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)in[(lane * 8 + i) & 4095];
        b[i] = (_Float16)in[(lane * 8 + i + 1000) & 4095];
    }
    f32x16 c0 = {}, c1 = {};
    f32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = in[(lane + 17 * i) & 4095] * 0.01f;
    unsigned pk = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (SHAPE == 8) {  // v_mfma_f32_32x32x8_f16: half the K of the 32x32x16 form (FLOPs counted as such)
                const f16x4 a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
                if (g & 1) c1 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c1, 0, 0, 0);
                else c0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, c0, 0, 0, 0);
            } else if (SHAPE == 32) {
                if (g & 1) c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
                else c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
            } else {
                if (g & 1) {
                    d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d1, 0, 0, 0);
                } else {
                    d2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d2, 0, 0, 0);
                    d3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d3, 0, 0, 0);
                }
            }
            if (FILL) {
                const int r = (2 * g) & 7;
                x[r] = __builtin_amdgcn_exp2f(x[r] - 0.5f);
                x[r + 1] = __builtin_amdgcn_exp2f(x[r + 1] - 0.5f);
                pk ^= __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(x[r], x[r + 1]));
                x[(r + 3) & 7] = fmaxf(fmaxf(x[(r + 3) & 7], x[(r + 4) & 7]), x[(r + 5) & 7]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = (float)pk;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) s += d0[i] + d1[i] + d2[i] + d3[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[blockIdx.x * 2] = t1 - t0;
        clk[blockIdx.x * 2 + 1] = r1 - r0;
    }
}

template <int SHAPE, int FILL>
void run(const char* name, float* in, float* out, unsigned long long* clk, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((kern<SHAPE, FILL>), dim3(grid), dim3(256), 0, 0, in, out, clk);
    hipEventRecord(e0);
    const int reps = 10;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((kern<SHAPE, FILL>), dim3(grid), dim3(256), 0, 0, in, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long h[4096];
    hipMemcpy(h, clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < grid; ++i) {
        cyc += h[2 * i];
        rt += h[2 * i + 1];
    }
    const double ghz = cyc / (rt / 100e6) / 1e9;
    // FLOPs: per wave per group 32x32x16 x 2 (or 2 x 16x16x32 x 2) = 32768 MACs x 2
    const double flops = 2.0 * 32 * 32 * (SHAPE == 8 ? 8 : 16) * 4.0 * ITER * 4.0 * grid;  // 4 groups, 4 waves/WG
    const double t = ms * 1e-3 / reps;
    printf("%-28s grid %4d: %8.1f us/launch  %7.1f TFLOP/s  in-kernel clock %.2f GHz\n", name, grid, t * 1e6,
           flops / t / 1e12, ghz);
}

int main() {
    float *in, *out;
    unsigned long long* clk;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, 2048 * 256 * 4);
    hipMalloc(&clk, 4096 * 8 * 2);
    static float h[4096];
    unsigned s = 12345;
    for (int i = 0; i < 4096; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = ((s >> 8) & 0xffff) / 65536.0f * 2.0f - 1.0f;
    }
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    if (getenv("MB_SHAPE8")) {  // cycles of the 32x32x8 form vs 32x32x16 (us per launch, same MFMA count)
        for (int rep = 0; rep < 2; ++rep) {
            run<32, 0>("32x32x16, MFMA only", in, out, clk, 512);
            run<8, 0>("32x32x8, MFMA only", in, out, clk, 512);
        }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run<32, 0>("32x32x16, MFMA only", in, out, clk, 512);
        run<16, 0>("16x16x32, MFMA only", in, out, clk, 512);
        run<32, 1>("32x32x16 + softmax fillers", in, out, clk, 512);
        run<16, 1>("16x16x32 + softmax fillers", in, out, clk, 512);
    }
    return 0;
}
