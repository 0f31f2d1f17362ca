// Microbenchmark (diagnostic, not shipped): issue cost of LDS-DMA pieces (buffer_load_dwordx4 ...
// lds, 1 KiB per wave instruction) vs plain buffer_load_dwordx4 into VGPRs, under the single-call
// kernel's load pattern: 256 workgroups x 4 waves (one per SIMD), every wave streaming N 1-KiB
// pieces of a 256 KiB slice (the 16-row kernel's per-wave K/V volume is 64 pieces).
// Per wave: s_memtime before the first issue, after the last issue, and after vmcnt(0).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_dma_issue.hip -o tools/mb_dma_issue && tools/mb_dma_issue
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int N>  // MODE 0: LDS-DMA, 1: plain loads into VGPRs (4 in flight, reused)
__global__ __launch_bounds__(256) void kern(const char* buf, unsigned slice_bytes, unsigned long long* out) {
    __shared__ __attribute__((aligned(16))) char smem[4 * 16384];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char* base = buf + (size_t)(blockIdx.x % 4) * slice_bytes;  // 4 heads' worth, L2-shared
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, slice_bytes,
                                                                  0x00020000);
    const unsigned voff = (unsigned)(wave * 64 * 1024 + lane * 16);
    u32x4 acc = {0, 0, 0, 0};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(smem + wave * 16384 + 1024 * (i & 15)),
                                                     16, voff, 1024 * i, 0, 0);
    } else {
        // inline asm: no compiler-inserted waits between the loads (4 rotating destinations)
        u32x4 d[4];
#pragma unroll
        for (int i = 0; i < N; ++i)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                         : "=v"(d[i & 3])
                         : "v"(voff + 1024u * (unsigned)(i >> 2) * 4u), "s"(rs), "i"(1024 * (i & 3)));
        const unsigned long long t1p = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3])::"memory");
        const unsigned long long t2p = __builtin_amdgcn_s_memtime();
        acc = d[0] ^ d[1] ^ d[2] ^ d[3];
        if (acc[0] == 0x12345678u) out[4096] = acc[1];
        if (lane == 0) {
            out[(blockIdx.x * 4 + wave) * 2] = t1p - t0;
            out[(blockIdx.x * 4 + wave) * 2 + 1] = t2p - t0;
        }
        return;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (acc[0] == 0x12345678u) out[4096] = acc[1];
    if (lane == 0) {
        out[(blockIdx.x * 4 + wave) * 2] = t1 - t0;
        out[(blockIdx.x * 4 + wave) * 2 + 1] = t2 - t0;
    }
}

template <int MODE, int N>
void run(const char* name, const char* buf, unsigned long long* out) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((kern<MODE, N>), dim3(256), dim3(256), 0, 0, buf, 256u << 10, out);
    hipDeviceSynchronize();
    static unsigned long long h[256 * 4 * 2];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    double is = 0, tot = 0;
    for (int i = 0; i < 256 * 4; ++i) {
        is += h[2 * i];
        tot += h[2 * i + 1];
    }
    is /= 1024;
    tot /= 1024;
    printf("%-22s N=%3d: issue %7.0f cyc (%5.1f per instr), issue->all landed %7.0f cyc\n", name, N, is, is / N, tot);
}

int main() {
    char* buf;
    unsigned long long* out;
    hipMalloc(&buf, 4u << 20);
    hipMalloc(&out, 8192 * 8);
    hipMemset(buf, 1, 4u << 20);
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 8>("LDS-DMA", buf, out);
        run<0, 16>("LDS-DMA", buf, out);
        run<0, 64>("LDS-DMA", buf, out);
        run<1, 8>("buffer_load to VGPR", buf, out);
        run<1, 16>("buffer_load to VGPR", buf, out);
        run<1, 64>("buffer_load to VGPR", buf, out);
    }
    return 0;
}
