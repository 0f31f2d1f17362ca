// Microbenchmark (diagnostic, not shipped): cycles per v_mfma_f32_32x32x16_f16 when each MFMA gap
// carries N independent fillers of one kind (v_exp_f32, v_add_f32, v_cvt_pk_f16_f32, v_max3_f32),
// one or two waves per SIMD. Answers "how much vector work hides under the matrix pipe".
//   hipcc --offload-arch=gfx950 -O3 tools/mb_mfma_fill.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ITER = 256;

template <int KIND, int N>
__device__ __forceinline__ void fill(float (&x)[16], int g) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int r = (g * N + j) & 15;
        if (KIND == 0) x[r] = __builtin_amdgcn_exp2f(x[r]);
        if (KIND == 1) x[r] = x[r] + 1.0f;
        if (KIND == 2) {
            const auto h = __builtin_amdgcn_cvt_pkrtz(x[r], x[(r + 1) & 15]);
            x[r] = __builtin_bit_cast(float, h);
        }
        if (KIND == 3) x[r] = fmaxf(fmaxf(x[r], x[(r + 5) & 15]), x[(r + 9) & 15]);
        if (KIND == 4) asm volatile("v_exp_f16 %0, %0" : "+v"(x[r]));  // (round 4: the half-precision exp)
        if (KIND == 5) asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(x[r]));  // result to the high half (SDWA)
        if (KIND == 6) asm volatile("v_exp_f32 %0, %0" : "+v"(x[r]));
    }
}

template <int KIND, int N, int MF>  // MF = 0: no MFMA (fillers alone)
__global__ __launch_bounds__(512) void kern(const float* in, float* out, long long* cyc) {
    f16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)in[threadIdx.x % 64 + i];
        b[i] = (_Float16)in[threadIdx.x % 64 + 8 + i];
    }
    f32x16 acc0 = {}, acc1 = {};
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[i] * 0.001f;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            if (MF) {
                if (g & 1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc1, 0, 0, 0);
                else acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
            }
            fill<KIND, N>(x, g);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i] + x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) {
        cyc[(blockIdx.x * 8 + threadIdx.x / 64) * 2] = t0;
        cyc[(blockIdx.x * 8 + threadIdx.x / 64) * 2 + 1] = t1;
    }
}

template <int KIND, int N, int MF>
void run(const char* name, float* in, float* out, long long* cyc, int threads) {
    hipLaunchKernelGGL((kern<KIND, N, MF>), dim3(256), dim3(threads), 0, 0, in, out, cyc);
    hipLaunchKernelGGL((kern<KIND, N, MF>), dim3(256), dim3(threads), 0, 0, in, out, cyc);
    hipDeviceSynchronize();
    long long h[256 * 8 * 2];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double sum = 0;
    int nw = threads / 64;
    for (int b = 0; b < 256; ++b) {
        long long lo = h[(b * 8) * 2], hi = h[(b * 8) * 2 + 1];
        for (int w = 0; w < nw; ++w) {
            lo = h[(b * 8 + w) * 2] < lo ? h[(b * 8 + w) * 2] : lo;
            hi = h[(b * 8 + w) * 2 + 1] > hi ? h[(b * 8 + w) * 2 + 1] : hi;
        }
        sum += hi - lo;
    }
    // block span per gap: for 2 waves/SIMD this covers both waves' MFMAs (2 per gap per SIMD)
    const double per = sum / 256.0 / (ITER * 8.0);
    printf("%-8s N=%d mfma=%d waves/SIMD=%d : %.1f cyc per gap (block span)\n", name, N, MF, threads / 256, per);
}

#define SWEEP(KIND, NAME, TH)                            \
    run<KIND, 0, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 1, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 2, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 3, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 4, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 6, 1>(NAME, in, out, cyc, TH);             \
    run<KIND, 4, 0>(NAME, in, out, cyc, TH);

int main() {
    float *in, *out;
    long long* cyc;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&cyc, 256 * 8 * 8 * 2);
    hipMemset(in, 0, 4096 * 4);
    for (int th : {256, 512}) {
        SWEEP(0, "exp", th);
        SWEEP(1, "add", th);
        SWEEP(4, "exp_f16", th);
        SWEEP(5, "exp_f16hi", th);
        SWEEP(6, "exp_f32a", th);
    }
    return 0;
}
