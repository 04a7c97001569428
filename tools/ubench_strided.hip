// Load-pattern microbenchmark for the skip walk (gfx950): 8 waves per CU, each
// wave walking its own 512-KiB region in 16-KiB blocks; per block every lane
// issues 20 buffer_load_dwordx4 and folds them.
//   pattern 0: lane slices of 256 B (+64 B lead), the skip walk's layout
//              (64 distinct 128-B lines per instruction)
//   pattern 1: coalesced, lane l at 16 l + 1024 i (8 lines per instruction)
//   pattern 2: as 0, but the next block's loads issued before folding the
//              current one (double-buffered registers)
// Reports the kernel time and the achieved bytes per second.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_strided.hip -o tools/ubench_strided.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t *base, uint32_t n)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, int(n), 0x00020000);
}

template <int PAT>
__global__ __launch_bounds__(256) void kern(const uint8_t *buf, uint64_t len, uint32_t *out, int blocks)
{
    const uint32_t lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t region = uint64_t(wave) * (512u << 10);
    uint32_t acc = 0;
    uint4 d[20], e[20];
    auto issue = [&](uint4 (&dst)[20], int b) {
        const uint64_t base = region + uint64_t(b) * (17u << 10);  // 16 KiB + 1 KiB jump per block
        const __amdgpu_buffer_rsrc_t rs = rsrc(buf + base, 0x7FFFFFF0u);
#pragma unroll
        for (int i = 0; i < 20; ++i) {
            const int off = PAT == 1 ? int(16 * lane + 1024 * i) : int(256 * lane + 16 * i);
            dst[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        }
    };
    auto fold = [&](const uint4 (&src)[20]) {
#pragma unroll
        for (int i = 0; i < 20; ++i) acc = __builtin_rotateleft32(acc, 5) ^ src[i].x ^ (src[i].y + src[i].z) ^ src[i].w;
    };
    if (PAT == 2) {
        issue(d, 0);
        for (int b = 0; b < blocks; b += 2) {
            issue(e, b + 1);
            fold(d);
            if (b + 2 < blocks) issue(d, b + 2);
            fold(e);
        }
    } else {
        for (int b = 0; b < blocks; ++b) {
            issue(d, b);
            fold(d);
        }
    }
    out[wave * 64 + lane] = acc;
}

template <int PAT>
void run(const char *name, const uint8_t *buf, uint32_t *out)
{
    const int blocks = 18, nblk = 512;  // 2048 waves x 18 x 20 KiB = 720 MiB of loads
    hipLaunchKernelGGL(kern<PAT>, dim3(nblk), dim3(256), 0, 0, buf, uint64_t(1) << 30, out, blocks);
    hipError_t err = hipDeviceSynchronize();
    if (err != hipSuccess || hipGetLastError() != hipSuccess) printf("launch error %s\n", hipGetErrorString(err));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kern<PAT>, dim3(nblk), dim3(256), 0, 0, buf, uint64_t(1) << 30, out, blocks);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double bytes = double(nblk) * 4 * 64 * 20 * 16 * blocks;
    printf("%-34s %.3f ms  %.0f GB/s of loads\n", name, best, bytes / (best * 1e-3) / 1e9);
}

int main()
{
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, (size_t(1) << 30) + (1 << 20)) != hipSuccess) { printf("malloc failed\n"); return 1; }
    hipMemset(buf, 1, (size_t(1) << 30) + (1 << 20));
    hipMalloc(&out, 2048 * 64 * 4);
    run<0>("strided 256-B lane slices", buf, out);
    run<1>("coalesced", buf, out);
    run<2>("strided, next block prefetched", buf, out);
    run<0>("strided 256-B lane slices", buf, out);
    run<1>("coalesced", buf, out);
    return 0;
}
