// HBM read-pattern microbenchmark (gfx950) for the scan's staging: 1 GiB read
// once by 248 workgroups x 12 waves, each wave streaming 64 lane runs of RUN
// bytes, with LDS-DMA (global_load_lds_dwordx4, one 1-KiB wave instruction per
// piece) into a private 4-KiB slot, or plain global loads to registers.
//   PAT 0: contiguous - each DMA instruction reads 1 KiB contiguous of the
//          wave's region (the wave's 64 runs read as one stream)
//   PAT 1: the scan's pattern - DMA j reads 64-B fragments of 16 runs
//   PAT 2: 8 runs x 128 B per DMA instruction
//   PAT 3: global_load_dwordx4 to VGPRs, contiguous 1 KiB per instruction
// Reports GB/s from hipEvents (best of 5).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_mem.hip -o tools/ubench_mem.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define WAVES 12

__device__ __forceinline__ void glds(const void *g, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0\n\ts_nop 1"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

__device__ __forceinline__ void glds_s(uint32_t off, const void *base, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0\n\ts_nop 1"
                 : "=&s"(keep)
                 : "v"(off), "s"(base), "s"(lds)
                 : "memory");
}

template <int PAT>
__global__ __launch_bounds__(WAVES * 64) void kern(const uint8_t *buf, uint64_t run, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) char lds[PAT == 6 ? 160 * 1024 : WAVES * 8192];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t task = uint64_t(blockIdx.x) * WAVES + wave;
    const uint8_t *base = buf + task * 64 * run;  // the wave's 64 runs
    const uint32_t slot = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wave * 8192;
    const uint32_t T = uint32_t(run / 64);  // stages of 64 B per lane
    uint32_t acc = 0;
    for (uint32_t t = 0; t < T; ++t) {
        if constexpr (PAT == 7) {  // PAT 5 through saddr + 32-bit per-lane offsets
            if (t & 1) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t c = 8 * j + lane / 8;
                const uint32_t k = (lane % 8) ^ ((c >> 1) & 7);
                glds_s(uint32_t(c * run + uint64_t(t / 2) * 128 + k * 16), base, slot + 1024 * j);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= *reinterpret_cast<const uint32_t *>(lds + wave * 8192 + lane * 128);
        } else if constexpr (PAT == 4 || PAT == 5 || PAT == 6) {  // 8-KiB stage: 8 DMAs of 8 runs x 128 B (all 64 runs), every other t
            if (t & 1) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t c = 8 * j + lane / 8;
                const uint32_t k = PAT >= 5 ? ((lane % 8) ^ ((c >> 1) & 7)) : (lane % 8);  // 5: XOR-swizzled pieces
                glds(base + c * run + uint64_t(t / 2) * 128 + k * 16, slot + 1024 * j);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= *reinterpret_cast<const uint32_t *>(lds + wave * 8192 + lane * 128);
        } else if constexpr (PAT == 3) {
            uint4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[j] = *reinterpret_cast<const uint4 *>(base + uint64_t(t) * 4096 + j * 1024 + lane * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint8_t *g;
                if constexpr (PAT == 0) g = base + uint64_t(t) * 4096 + j * 1024 + lane * 16;
                else if constexpr (PAT == 1) g = base + (16 * j + lane / 4) * run + uint64_t(t) * 64 + (lane % 4) * 16;
                else g = base + (8 * (j + 4 * (t & 1)) + lane / 8) * run + uint64_t(t / 2) * 128 + (lane % 8) * 16;
                glds(g, slot + 1024 * j);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= *reinterpret_cast<const uint32_t *>(lds + wave * 8192 + lane * 64);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int PAT>
void run(const char *name, const uint8_t *buf, uint32_t *out, uint64_t runlen)
{
    const uint64_t total = 1ull << 30;
    const int wgs = int(total / (WAVES * 64 * runlen));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<PAT>, dim3(wgs), dim3(WAVES * 64), 0, 0, buf, runlen, out);
    (void)hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern<PAT>, dim3(wgs), dim3(WAVES * 64), 0, 0, buf, runlen, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double bytes = double(wgs) * WAVES * 64 * runlen;
    printf("%-28s run=%5llu wgs=%4d  %7.1f GB/s  (%.1f us)\n", name, (unsigned long long)runlen, wgs,
           bytes / (best * 1e-3) / 1e9, best * 1e3);
    fflush(stdout);
}

int main()
{
    uint8_t *buf;
    uint32_t *out;
    (void)hipMalloc(&buf, (1ull << 30) + (1 << 20));
    (void)hipMalloc(&out, 64);
    (void)hipMemset(buf, 1, (1ull << 30) + (1 << 20));
    for (uint64_t rl : {5632ull}) {
        run<0>("LDS-DMA contiguous", buf, out, rl);
        run<1>("LDS-DMA 16 runs x 64 B", buf, out, rl);
        run<2>("LDS-DMA 8 runs x 128 B", buf, out, rl);
        run<3>("global_load_dwordx4 contig", buf, out, rl);
        run<4>("LDS-DMA 8 KiB: 64 runs x 128 B", buf, out, rl);
        run<5>("  same, XOR-swizzled pieces", buf, out, rl);
        run<6>("  same, 160 KiB LDS", buf, out, rl);
        run<7>("  same, saddr + u32 offsets", buf, out, rl);
    }
    return 0;
}
