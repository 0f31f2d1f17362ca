// Microbenchmark (diagnostic, not shipped): does FETCH_SIZE count Infinity-Cache (MALL) hits, and
// what does a second XCD's re-read of a head's K/V cost when it is served on-die?
//
// Dispatch sequence (each a separate kernel launch, so rocprofv3 --pmc reports each one):
//   scrub  : stream a 1 GiB buffer (evicts X from the 256 MiB Infinity Cache)
//   cold   : 256 workgroups read X (16 MiB) once           -> X comes from HBM
//   warm   : the same launch again                         -> X from MALL (L2 is cold per dispatch
//                                                             under counter collection)
//   halves : workgroups on even XCDs read X, then (next launch) odd XCDs read X: the direct16
//            kernel's two-XCDs-per-head pattern, the second read after the first has landed
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum`, and
// under --kernel-trace for durations.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_mall_count.hip -o /tmp/mb_mall && /tmp/mb_mall
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// parity: -1 = every workgroup, 0 / 1 = only workgroups whose blockIdx % 8 is even / odd (XCD
// round-robin placement); each participating workgroup reads a contiguous share of X.
__global__ __launch_bounds__(256) void read_kernel(const f32x4* __restrict__ x, size_t n4, int parity,
                                                   float* __restrict__ out) {
    const int xcd = blockIdx.x & 7;
    if (parity >= 0 && (xcd & 1) != parity) return;
    const int parts = parity >= 0 ? gridDim.x / 2 : gridDim.x;
    const int part = parity >= 0 ? (blockIdx.x >> 3) * 4 + (xcd >> 1) : blockIdx.x;
    const size_t per = n4 / parts;
    const f32x4* p = x + per * part;
    f32x4 acc = {0, 0, 0, 0};
    for (size_t i = threadIdx.x; i < per; i += blockDim.x) acc += p[i];
    const float s = acc[0] + acc[1] + acc[2] + acc[3];
    if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keep the loads
}

int main() {
    const size_t xbytes = 16u << 20, sbytes = 1ull << 30;
    f32x4 *x, *scrub;
    float* out;
    hipMalloc(&x, xbytes);
    hipMalloc(&scrub, sbytes);
    hipMalloc(&out, 256 * 256 * 4);
    hipMemset(x, 0, xbytes);
    hipMemset(scrub, 0, sbytes);
    hipDeviceSynchronize();
    hipEvent_t e[8];
    for (auto& ev : e) hipEventCreate(&ev);
    const size_t n4 = xbytes / 16, s4 = sbytes / 16;
    float ms[6] = {};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, scrub, s4, -1, out);  // scrub
        hipEventRecord(e[0]);
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, x, n4, -1, out);  // cold
        hipEventRecord(e[1]);
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, x, n4, -1, out);  // warm (MALL)
        hipEventRecord(e[2]);
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, scrub, s4, -1, out);  // scrub
        hipEventRecord(e[3]);
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, x, n4, 0, out);  // even XCDs, cold
        hipEventRecord(e[4]);
        hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, 0, x, n4, 1, out);  // odd XCDs, MALL
        hipEventRecord(e[5]);
        hipDeviceSynchronize();
        hipEventElapsedTime(&ms[0], e[0], e[1]);
        hipEventElapsedTime(&ms[1], e[1], e[2]);
        hipEventElapsedTime(&ms[2], e[3], e[4]);
        hipEventElapsedTime(&ms[3], e[4], e[5]);
        printf("rep %d: 16 MiB read: cold %.2f us (%.0f GB/s), warm %.2f us (%.0f GB/s); even-XCD half cold %.2f us, "
               "odd-XCD half after it %.2f us\n",
               rep, ms[0] * 1e3, xbytes / (ms[0] * 1e-3) / 1e9, ms[1] * 1e3, xbytes / (ms[1] * 1e-3) / 1e9,
               ms[2] * 1e3, ms[3] * 1e3);
    }
    return 0;
}
