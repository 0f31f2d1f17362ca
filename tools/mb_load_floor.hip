// Microbenchmark (diagnostic, not shipped): the latency floor of a single-call-shaped launch that
// only moves the bytes of a 1x4x1024x1024 head_dim-64 call: every wave streams its slice of K and
// V (fp16 rows of 128 B) from a head-local region into registers and writes 16 B per lane. Grid,
// workgroup size and keys per wave span the single-call workgroup plans (no-split 32-row blocks
// on 128 workgroups, the 2-split (1,8) plan on 256, 16-row blocks on 256 x 1024 threads).
// Per-launch time = replay time of a graph of back-to-back launches / count.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_load_floor.hip -o tools/mb_load_floor && tools/mb_load_floor
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Head h's K (and V) is 1024 rows x 128 B = 128 KiB; a workgroup of head h covers `span` keys
// starting at split * span; wave w covers KPW keys of that.
template <int NT, int KPW>
__global__ __launch_bounds__(NT) void stream_kernel(const u32x4* K, const u32x4* V, u32x4* O, int wg_per_head,
                                                     int span) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // XCD-aware: blocks on one XCD (blockIdx % 8) work on one head (2 XCDs per head at 4 heads).
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int per_xcd = gridDim.x >> 3;
    const int head = xcd >> 1;
    const int local = (xcd & 1) * per_xcd + idx;  // 0 .. wg_per_head-1
    const int split = local % (1024 / span);
    const int key0 = split * span + wave * KPW;
    constexpr int N = KPW * 8 / 64;  // 16-B chunks per lane per tensor
    u32x4 acc = {0, 0, 0, 0};
    if constexpr (KPW > 0) {
        const u32x4* kb = K + (size_t)head * 1024 * 8 + (size_t)key0 * 8;
        const u32x4* vb = V + (size_t)head * 1024 * 8 + (size_t)key0 * 8;
        u32x4 r[2 * N];
#pragma unroll
        for (int i = 0; i < N; ++i) r[i] = kb[i * 64 + lane];
#pragma unroll
        for (int i = 0; i < N; ++i) r[N + i] = vb[i * 64 + lane];
#pragma unroll
        for (int i = 0; i < 2 * N; ++i) acc ^= r[i];
    }
    O[(size_t)blockIdx.x * NT + threadIdx.x] = acc;
}

// The same volume by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per instruction) into a 16 KiB
// per-wave LDS region (overwritten in turn: only the transfer rate is of interest).
// ROT (round 6): 0 every workgroup issues its pieces in the same order; 1 rotated by the workgroup's
// index within its head (piece (i + local) % N first), so the head's workgroups start on different
// lines; 2 rotated by whole 64-key tiles ((local % 4) tiles), the order a kernel could use.
template <int KPW, int NT = 512, int ROT = 0>
__global__ __launch_bounds__(NT) void dma_kernel(const u32x4* K, const u32x4* V, u32x4* O, int span) {
    __shared__ __attribute__((aligned(16))) char lds[8 * 16384];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int per_xcd = gridDim.x >> 3;
    const int head = xcd >> 1;
    const int local = (xcd & 1) * per_xcd + idx;
    const int split = local % (1024 / span);
    const int key0 = split * span + wave * KPW;
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void*)(K + (size_t)head * 1024 * 8), (short)0, 1 << 17, 0x00020000);
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc((void*)(V + (size_t)head * 1024 * 8), (short)0, 1 << 17, 0x00020000);
    constexpr int N = KPW / 8;  // 1 KiB pieces per tensor
    const int rot = ROT == 1 ? local % N : ROT == 2 ? (local % 4) * (N / 4) : 0;
    const unsigned ko = (unsigned)(key0 * 128 + lane * 16);
#pragma unroll
    for (int i = 0; i < N; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(kr, (__attribute__((address_space(3))) void*)(lds + wave * 16384 + (i & 15) * 1024), 16,
                                                 ko + (unsigned)(((i + rot) % N) * 1024), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < N; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (__attribute__((address_space(3))) void*)(lds + wave * 16384 + ((i + N) & 15) * 1024), 16,
                                                 ko + (unsigned)(((i + rot) % N) * 1024), 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    O[(size_t)blockIdx.x * NT + threadIdx.x] = *(const u32x4*)(lds + threadIdx.x * 16);
}

// fp32 K/V (256-B rows, the Float boundary's inputs) by LDS-DMA, 16 B per lane per instruction:
// twice the pieces of dma_kernel for the same keys.
template <int KPW, int NT = 256>
__global__ __launch_bounds__(NT) void dma32_kernel(const u32x4* K, const u32x4* V, u32x4* O, int span) {
    __shared__ __attribute__((aligned(16))) char lds[4 * 32768];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int per_xcd = gridDim.x >> 3;
    const int head = xcd >> 1;
    const int local = (xcd & 1) * per_xcd + idx;
    const int split = local % (1024 / span);
    const int key0 = split * span + wave * KPW;
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc((void*)(K + (size_t)head * 1024 * 16), (short)0, 1 << 18, 0x00020000);
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc((void*)(V + (size_t)head * 1024 * 16), (short)0, 1 << 18, 0x00020000);
    constexpr int N = KPW / 4;  // 1 KiB pieces per tensor
#pragma unroll
    for (int i = 0; i < N; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(kr, (__attribute__((address_space(3))) void*)(lds + wave * 32768 + (i & 31) * 1024), 16,
                                                 (unsigned)(key0 * 256 + lane * 16), i * 1024, 0, 0);
#pragma unroll
    for (int i = 0; i < N; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (__attribute__((address_space(3))) void*)(lds + wave * 32768 + ((i + N) & 31) * 1024), 16,
                                                 (unsigned)(key0 * 256 + lane * 16), i * 1024, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    O[(size_t)blockIdx.x * NT + threadIdx.x] = *(const u32x4*)(lds + threadIdx.x * 16);
}

// fp32 K/V through VGPRs, converted to fp16 and written to LDS (what a one-launch Float boundary
// would do per workgroup): 16 rows x 1024 keys per workgroup, 4 waves x 256 keys, 8 chunk
// loads in flight per batch.
template <int KPW, int NT = 256>
__global__ __launch_bounds__(NT) void cvt32_kernel(const u32x4* K, const u32x4* V, u32x4* O, int span) {
    __shared__ __attribute__((aligned(16))) char lds[4 * 16384];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
    const int per_xcd = gridDim.x >> 3;
    const int head = xcd >> 1;
    const int local = (xcd & 1) * per_xcd + idx;
    const int split = local % (1024 / span);
    const int key0 = split * span + wave * KPW;
    constexpr int N = KPW / 8;  // 8-row pieces per tensor (one 32-B, 8-float chunk per lane each)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const u32x4* base = (t == 0 ? K : V) + (size_t)head * 1024 * 16 + (size_t)key0 * 16;
#pragma unroll 4
        for (int b = 0; b < N / 16; ++b) {
            u32x4 r[32];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                r[2 * i] = base[(b * 16 + i) * 128 + 2 * lane];
                r[2 * i + 1] = base[(b * 16 + i) * 128 + 2 * lane + 1];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float* f = reinterpret_cast<const float*>(&r[2 * i]);
                typedef _Float16 h8 __attribute__((ext_vector_type(8)));
                h8 h = {(_Float16)f[0], (_Float16)f[1], (_Float16)f[2], (_Float16)f[3],
                        (_Float16)f[4], (_Float16)f[5], (_Float16)f[6], (_Float16)f[7]};
                *reinterpret_cast<__attribute__((address_space(3))) h8*>(
                    (__attribute__((address_space(3))) char*)lds + wave * 16384 + ((b * 16 + i) & 15) * 1024 + lane * 16) = h;
            }
            asm volatile("" ::: "memory");  // the overwritten stores stay (no dead-store elimination)
        }
    }
    __syncthreads();
    O[(size_t)blockIdx.x * NT + threadIdx.x] = *(const u32x4*)(lds + threadIdx.x * 16);
}

__global__ void empty_kernel() {}

template <typename F>
static double time_graph(F launch, hipStream_t s, int count) {
    hipGraph_t g;
    hipGraphExec_t ge;
    launch();
    CK(hipStreamSynchronize(s));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < count; ++i) launch();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<double> t;
    for (int rep = 0; rep < 7; ++rep) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms * 1e3 / count);
    }
    std::sort(t.begin(), t.end());
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    u32x4 *K, *V, *O;
    CK(hipMalloc(&K, 4 << 20));
    CK(hipMalloc(&V, 4 << 20));
    CK(hipMalloc(&O, 16 << 20));
    CK(hipMemset(K, 1, 4 << 20));
    CK(hipMemset(V, 2, 4 << 20));
    const int C = 200;
    printf("{\"empty_256x512_us\": %.3f", time_graph([&] { empty_kernel<<<256, 512, 0, s>>>(); }, s, C));
#define RUN(NAME, GRID, NT, KPW, SPAN)                                                                     \
    printf(", \"%s\": %.3f", NAME,                                                                         \
           time_graph([&] { stream_kernel<NT, KPW><<<GRID, NT, 0, s>>>(K, V, O, GRID / 4, SPAN); }, s, C))
    RUN("store_only_256x512_us", 256, 512, 0, 512);
    RUN("nosplit_128x512_kpw128_us", 128, 512, 128, 1024);   // 32 rows x 1024 keys per WG: 256 KiB/CU
    RUN("split2_256x512_kpw64_us", 256, 512, 64, 512);       // (1,8) 2-split: 128 KiB/CU
    RUN("split4_256x256_kpw64_us", 256, 256, 64, 256);       // (2,4) 4-split: 64 KiB/CU (x2 q-waves)
    RUN("nosplit16_256x1024_kpw64_us", 256, 1024, 64, 1024); // 16 rows x 1024 keys: 256 KiB/CU
    RUN("nosplit_128x1024_kpw64_us", 128, 1024, 64, 1024);   // 32 rows x 1024 keys, 16 waves
    RUN("nosplit_64x512_kpw128_us", 64, 512, 128, 1024);     // 64 rows x 1024 keys per WG
    printf(", \"dma_nosplit_128x512_kpw128_us\": %.3f",
           time_graph([&] { dma_kernel<128><<<128, 512, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_split2_256x512_kpw64_us\": %.3f",
           time_graph([&] { dma_kernel<64><<<256, 512, 0, s>>>(K, V, O, 512); }, s, C));
    RUN("nosplit16_256x256_kpw256_us", 256, 256, 256, 1024); // 16 rows x 1024 keys, 4 waves
    printf(", \"dma_nosplit_128x256_kpw256_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256><<<128, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_nosplit16_256x256_kpw256_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_nosplit16_256x256_kpw256_rot_piece_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256, 1><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_nosplit16_256x256_kpw256_rot_tile_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256, 2><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_nosplit16_256x256_kpw256_again_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma_nosplit16_256x256_kpw256_rot_piece_again_us\": %.3f",
           time_graph([&] { dma_kernel<256, 256, 1><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"dma32_nosplit16_256x256_kpw256_us\": %.3f",
           time_graph([&] { dma32_kernel<256><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf(", \"cvt32_nosplit16_256x256_kpw256_us\": %.3f",
           time_graph([&] { cvt32_kernel<256><<<256, 256, 0, s>>>(K, V, O, 1024); }, s, C));
    printf("}\n");
    return 0;
}
