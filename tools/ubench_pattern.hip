// Read-rate microbenchmark: the scan's access pattern (each wave owns 64 lane
// runs of RUN bytes; one instruction reads 128 B of each of 8 runs) against a
// contiguous one (one instruction reads 1 KiB), each through three ways in:
// LDS-DMA (global_load_lds_dwordx4, the scan's), direct nontemporal loads into
// registers, and direct plain loads.  1 GiB, nothing computed; the bytes are
// folded into one word per wave so the loads stay live.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/_bin/ubench_pattern tools/ubench_pattern.hip
//   tools/_bin/ubench_pattern
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr uint32_t kWaves = 8;    // per workgroup (LDS-DMA: 4 KiB slot x 2 per wave)
constexpr uint64_t kRun = 5632;   // the scan's lane run on C1
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// instruction-piece offsets of one wave step (4 instructions x 1 KiB):
//   strided (the scan's pair staging): step s covers half s & 1 of the wave's
//   64 runs, 128 B of each at 128 B x (s / 2); instruction j covers 8 of them
//   contiguous: instruction j covers 1 KiB at 4 KiB x step + 1 KiB x j
template <bool kStrided>
__device__ __forceinline__ uint64_t piece_off(uint64_t wave_base, uint32_t step, uint32_t j, uint32_t lane)
{
    if constexpr (kStrided) {
        const uint32_t r = 8u * j + lane / 8u + 32u * (step & 1u);  // run
        return wave_base + uint64_t(r) * kRun + 128ull * (step >> 1) + 16u * (lane % 8u);
    } else {
        return wave_base + 4096ull * step + 1024u * j + 16u * lane;
    }
}

#define DMA_ASM(POL)                                                                                        \
    asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"                        \
                 "global_load_lds_dwordx4 %1, %[base]" POL "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"            \
                 "global_load_lds_dwordx4 %2, %[base]" POL "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"            \
                 "global_load_lds_dwordx4 %3, %[base]" POL "\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"            \
                 "global_load_lds_dwordx4 %4, %[base]" POL "\n\t"                                                   \
                 "s_mov_b32 m0, %[keep]\n\ts_nop 1"                                                               \
                 : [keep] "=&s"(keep)                                                                              \
                 : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), [base] "s"(p), [dst] "s"(dst)               \
                 : "memory", "scc")

// kPol: 0 default, 1 nt, 2 nt sc1, 3 sc0 sc1 nt, 4 sc1
template <bool kStrided, int kPol = 0>
__global__ __launch_bounds__(kWaves * 64) void k_dma2(const uint8_t *p, uint64_t steps, uint64_t wave_bytes, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) char lds[kWaves * 2 * 4096];
    const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = uint64_t(blockIdx.x) * kWaves + wave;
    const uint64_t wb = w * wave_bytes;
    const uint32_t slot = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wave * 8192u;
    for (uint32_t st = 0; st < steps; ++st) {
        uint32_t keep;
        const uint32_t dst = slot + (st & 1u) * 4096u;
        uint32_t off[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) off[j] = uint32_t(piece_off<kStrided>(0, st, j, lane) + wb);
        if constexpr (kPol == 0) DMA_ASM("");
        else if constexpr (kPol == 1) DMA_ASM(" nt");
        else if constexpr (kPol == 2) DMA_ASM(" sc1 nt");
        else if constexpr (kPol == 3) DMA_ASM(" sc0 sc1 nt");
        else DMA_ASM(" sc1");
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = *reinterpret_cast<const uint32_t *>(lds);
}

template <bool kStrided, bool kNt = false>
__global__ __launch_bounds__(kWaves * 64) void k_dma(const uint8_t *p, uint64_t steps, uint64_t wave_bytes, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) char lds[kWaves * 2 * 4096];
    const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = uint64_t(blockIdx.x) * kWaves + wave;
    const uint64_t wb = w * wave_bytes;
    const uint32_t slot = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wave * 8192u;
    for (uint32_t st = 0; st < steps; ++st) {
        uint32_t keep;
        const uint32_t dst = slot + (st & 1u) * 4096u;
        uint32_t off[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) off[j] = uint32_t(piece_off<kStrided>(0, st, j, lane) + wb);
        if constexpr (kNt)
            asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, %[base] nt\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %2, %[base] nt\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %3, %[base] nt\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %4, %[base] nt\n\t"
                         "s_mov_b32 m0, %[keep]\n\ts_nop 1"
                         : [keep] "=&s"(keep)
                         : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), [base] "s"(p), [dst] "s"(dst)
                         : "memory", "scc");
        else
            asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %2, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %3, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %4, %[base]\n\t"
                         "s_mov_b32 m0, %[keep]\n\ts_nop 1"
                         : [keep] "=&s"(keep)
                         : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), [base] "s"(p), [dst] "s"(dst)
                         : "memory", "scc");
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = *reinterpret_cast<const uint32_t *>(lds);
}

template <bool kStrided, bool kNt>
__global__ __launch_bounds__(kWaves * 64) void k_direct(const uint8_t *p, uint64_t steps, uint64_t wave_bytes, uint32_t *sink)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t w = uint64_t(blockIdx.x) * kWaves + wave;
    const uint64_t wb = w * wave_bytes;
    uint32_t x = 0;
    for (uint32_t st = 0; st + 1 < steps; st += 2) {  // two steps (8 loads) in flight
        u32x4 v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            const u32x4 *a = reinterpret_cast<const u32x4 *>(p + piece_off<kStrided>(wb, st + k / 4, k % 4, lane));
            v[k] = kNt ? __builtin_nontemporal_load(a) : *a;
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (int o = 32; o; o >>= 1) x ^= uint32_t(__shfl_xor(int(x), o));
    if (lane == 0) atomicXor(sink + blockIdx.x, x);
}

template <typename K>
static void run(const char *name, K kern, uint32_t wgs, const uint8_t *d, uint64_t steps, uint64_t wave_bytes,
                uint32_t *sink, uint64_t bytes)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ms;
    for (int r = 0; r < 25; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kern, dim3(wgs), dim3(kWaves * 64), 0, 0, d, steps, wave_bytes, sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, e0, e1);
        if (r >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-34s best %7.1f GB/s  median %7.1f GB/s\n", name, bytes / (ms.front() * 1e-3) / 1e9,
           bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    // strided: every wave owns 64 runs of kRun bytes (its steps walk 128 B down each run);
    // contiguous: every wave owns the same number of bytes as one stretch
    const uint32_t wgs = uint32_t(cus) * 2u;            // 2 workgroups x 8 waves per CU (LDS: 2 x 64 KiB)
    const uint64_t waves = uint64_t(wgs) * kWaves;
    const uint64_t wave_bytes = 64ull * kRun;            // 352 KiB per wave
    const uint64_t steps = 2 * kRun / 128;               // 88 steps x 4 KiB = the wave's 352 KiB
    const uint64_t bytes_strided = waves * 4096ull * steps;  // bytes read per launch (both patterns)
    uint8_t *d = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&d, waves * wave_bytes + 4096) != hipSuccess || hipMalloc(&sink, wgs * 4) != hipSuccess) return 1;
    (void)hipMemset(d, 1, waves * wave_bytes + 4096);
    printf("%d CUs, %llu waves, %.2f GiB read per launch, run %llu B\n", cus, (unsigned long long)waves,
           bytes_strided / double(1ull << 30), (unsigned long long)kRun);
    if (getenv("UB_POLICIES")) {
        for (int rep = 0; rep < 2; ++rep) {
            run("LDS-DMA strided default", k_dma2<true, 0>, wgs, d, steps, wave_bytes, sink, bytes_strided);
            run("LDS-DMA strided nt", k_dma2<true, 1>, wgs, d, steps, wave_bytes, sink, bytes_strided);
            run("LDS-DMA strided sc1 nt", k_dma2<true, 2>, wgs, d, steps, wave_bytes, sink, bytes_strided);
            run("LDS-DMA strided sc0 sc1 nt", k_dma2<true, 3>, wgs, d, steps, wave_bytes, sink, bytes_strided);
            run("LDS-DMA strided sc1", k_dma2<true, 4>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run("LDS-DMA   strided 8x128 B", k_dma<true>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("LDS-DMA   contiguous 1 KiB", k_dma<false>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("LDS-DMA nt strided 8x128 B", k_dma<true, true>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("LDS-DMA nt contiguous 1 KiB", k_dma<false, true>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("direct nt strided 8x128 B", k_direct<true, true>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("direct nt contiguous 1 KiB", k_direct<false, true>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("direct    strided 8x128 B", k_direct<true, false>, wgs, d, steps, wave_bytes, sink, bytes_strided);
        run("direct    contiguous 1 KiB", k_direct<false, false>, wgs, d, steps, wave_bytes, sink, bytes_strided);
    }
    return 0;
}
