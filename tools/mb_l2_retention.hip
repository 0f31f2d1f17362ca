// Microbenchmark (diagnostic, not shipped): does an XCD's L2 keep a kernel's input lines for the
// next kernel of the same stream? One lane per workgroup (8 workgroups: one per XCD) walks a
// 64-line pointer chain twice (128-B lines, dependent loads); s_memtime around each walk. In back-
// to-back launches the first walk reads lines the previous launch read: if the L2 kept them it
// costs what the second walk costs (an L2 hit each), if the kernel boundary invalidated the L2 it
// costs what a walk after a 256 MiB scrub costs. A third walk in the same launch
// gives the L2-hit figure directly (walks 1 and 3 are agent-scope atomic loads, which skip the L1); the second (plain) walk is the L1 figure. No profiler (a tracer changes cache behaviour).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_l2_retention.hip -o tools/mb_l2_retention
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

__global__ void chase(const unsigned* __restrict__ next, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    unsigned p = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 0u * i;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) p = next[p];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i) p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 0u * i;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 4 + 0] = t1 - t0;
    out[blockIdx.x * 4 + 1] = t2 - t1;
    out[blockIdx.x * 4 + 2] = t3 - t2;
    out[blockIdx.x * 4 + 3] = p;
}

__global__ void scrub(unsigned* buf, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) buf[i] += 1;
}

int main() {
    const int lines = 64;
    std::vector<unsigned> h(lines * 32, 0), perm(lines);
    for (int i = 0; i < lines; ++i) perm[i] = i;
    srand(7);
    for (int i = lines - 1; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
    for (int i = 0; i < lines; ++i) h[perm[i] * 32] = perm[(i + 1) % lines] * 32;  // one word per 128-B line
    unsigned* next;
    unsigned* big;
    unsigned long long* out;
    const size_t big_n = (256u << 20) / 4;
    if (hipMalloc(&next, h.size() * 4) || hipMalloc(&out, 8 * 4 * 8) || hipMalloc(&big, big_n * 4)) return 1;
    (void)hipMemcpy(next, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemset(big, 0, big_n * 4);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    std::vector<unsigned long long> o(32);
    auto report = [&](const char* what) {
        (void)hipMemcpy(o.data(), out, 8 * 4 * 8, hipMemcpyDeviceToHost);
        double a = 0, b = 0, c = 0;
        for (int w = 0; w < 8; ++w) a += o[w * 4], b += o[w * 4 + 1], c += o[w * 4 + 2];
        printf("{\"case\": \"%s\", \"walk1_l2path_cyc_per_load\": %.1f, \"walk2_cached_cyc_per_load\": %.1f, "
               "\"walk3_l2path_cyc_per_load\": %.1f}\n", what, a / 8 / 64, b / 8 / 64, c / 8 / 64);
    };
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(chase, dim3(8), dim3(64), 0, s, next, out);
    (void)hipStreamSynchronize(s);
    report("back_to_back_launches");
    hipLaunchKernelGGL(scrub, dim3(2048), dim3(256), 0, s, big, big_n);
    hipLaunchKernelGGL(chase, dim3(8), dim3(64), 0, s, next, out);
    (void)hipStreamSynchronize(s);
    report("after_256MiB_scrub");
    return 0;
}
