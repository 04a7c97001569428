// HBM read-pattern microbenchmark, second series (gfx950): how the scan's
// LDS-DMA staging rate depends on the bytes read per run per DMA piece
// (CHUNK), on the DMA groups a wave keeps in flight (DEPTH slots of 4 KiB),
// on waves per workgroup and on the grid.  No compute: each wave walks its 64
// lane runs of RUN bytes in groups of four 1-KiB DMA instructions
// (global_load_lds_dwordx4, saddr + per-lane offsets), CHUNK bytes per run
// per piece, into a ring of DEPTH slots; group g waits for group g - DEPTH.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_mem2.hip -o tools/ubench_mem2.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

__device__ __forceinline__ void glds_s(uint32_t off, const void *base, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0\n\ts_nop 1"
                 : "=&s"(keep)
                 : "v"(off), "s"(base), "s"(lds)
                 : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm()
{
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else static_assert(N < 0, "vmcnt");
}

template <int CHUNK, int DEPTH, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void kern(const uint8_t *buf, uint64_t run, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) char lds[WAVES * DEPTH * 4096];
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t task = uint64_t(blockIdx.x) * WAVES + wave;
    const uint8_t *base = buf + task * 64 * run;  // the wave's 64 runs
    const uint32_t slot0 = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wave * DEPTH * 4096;
    constexpr uint32_t kPer = 1024 / CHUNK;        // runs per DMA instruction
    constexpr uint32_t kRunsPerGroup = 4 * kPer;   // runs per group
    constexpr uint32_t kSub = 64 / kRunsPerGroup;  // groups per chunk position
    constexpr uint32_t kLanesPerRun = CHUNK / 16;
    const uint32_t npos = uint32_t(run / CHUNK);
    const uint32_t ngroups = npos * kSub;
    uint32_t acc = 0;
    for (uint32_t g = 0; g < ngroups; ++g) {
        const uint32_t pos = g / kSub, sub = g % kSub;
        const uint32_t slot = slot0 + (g % DEPTH) * 4096;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t r = sub * kRunsPerGroup + j * kPer + lane / kLanesPerRun;
            glds_s(uint32_t(r * run + uint64_t(pos) * CHUNK + (lane % kLanesPerRun) * 16), base, slot + 1024 * j);
        }
        if (g + 1 >= DEPTH) {
            wait_vm<4 * (DEPTH - 1)>();
            acc ^= *reinterpret_cast<const uint32_t *>(lds + (slot0 - uint32_t(reinterpret_cast<uintptr_t>(lds))) +
                                                       ((g + 1) % DEPTH) * 4096 + lane * 64);
        }
    }
    wait_vm<0>();
    if (acc == 0x12345678u) out[0] = acc;
}

template <int CHUNK, int DEPTH, int WAVES>
void run(const uint8_t *buf, uint32_t *out, uint64_t runlen, int wgs)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL((kern<CHUNK, DEPTH, WAVES>), dim3(wgs), dim3(WAVES * 64), 0, 0, buf, runlen, out);
    (void)hipDeviceSynchronize();
    float best = 1e9f, sum = 0;
    for (int r = 0; r < 20; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((kern<CHUNK, DEPTH, WAVES>), dim3(wgs), dim3(WAVES * 64), 0, 0, buf, runlen, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double bytes = double(wgs) * WAVES * 64 * double(runlen / CHUNK * CHUNK);
    printf("chunk %4d depth %d waves %2d wgs %4d run %6llu: best %7.1f GB/s  avg %7.1f GB/s  (%.1f us)\n", CHUNK, DEPTH,
           WAVES, wgs, (unsigned long long)runlen, bytes / (best * 1e-3) / 1e9, bytes / (sum / 20 * 1e-3) / 1e9,
           best * 1e3);
    fflush(stdout);
}

// Cold start: every launch of the first N timed on its own (the clock ramp).
template <int CHUNK, int DEPTH, int WAVES>
void cold(const uint8_t *buf, uint32_t *out, uint64_t runlen, int wgs, int n)
{
    std::vector<hipEvent_t> ev(n + 1);
    for (auto &e : ev) (void)hipEventCreate(&e);
    (void)hipEventRecord(ev[0]);
    for (int i = 0; i < n; ++i) {
        hipLaunchKernelGGL((kern<CHUNK, DEPTH, WAVES>), dim3(wgs), dim3(WAVES * 64), 0, 0, buf, runlen, out);
        (void)hipEventRecord(ev[i + 1]);
    }
    (void)hipDeviceSynchronize();
    const double bytes = double(wgs) * WAVES * 64 * double(runlen / CHUNK * CHUNK);
    double t = 0;
    for (int b = 0; b < n; b += 10) {
        double sum = 0;
        for (int i = b; i < b + 10 && i < n; ++i) {
            float ms;
            (void)hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
            sum += ms;
        }
        printf("launches %3d-%3d  t=%7.2f ms  avg %6.1f us  %7.1f GB/s\n", b, b + 9, t, sum / 10 * 1e3,
               bytes / (sum / 10 * 1e-3) / 1e9);
        t += sum;
    }
}

int main(int argc, char **argv)
{
    uint8_t *buf;
    uint32_t *out;
    (void)hipMalloc(&buf, (1ull << 30) + (4 << 20));
    (void)hipMalloc(&out, 64);
    (void)hipMemset(buf, 1, (1ull << 30) + (4 << 20));
    if (argc > 1 && strcmp(argv[1], "cold") == 0) {
        cold<128, 1, 12>(buf, out, 5632, 248, 300);
        return 0;
    }
    // one GiB: wgs * waves * 64 * run
    run<128, 1, 12>(buf, out, 5632, 248);
    run<128, 2, 12>(buf, out, 5632, 248);
    run<128, 3, 12>(buf, out, 5632, 248);
    run<256, 1, 12>(buf, out, 5632, 248);
    run<256, 2, 12>(buf, out, 5632, 248);
    run<256, 3, 12>(buf, out, 5632, 248);
    run<512, 1, 12>(buf, out, 5632, 248);
    run<512, 2, 12>(buf, out, 5632, 248);
    run<512, 3, 12>(buf, out, 5632, 248);
    run<1024, 2, 12>(buf, out, 6144, 228);
    run<128, 2, 8>(buf, out, 8448, 248);
    run<256, 2, 8>(buf, out, 8448, 248);
    run<256, 4, 8>(buf, out, 8448, 248);
    run<512, 4, 8>(buf, out, 8192, 256);
    run<128, 2, 16>(buf, out, 4096, 256);
    run<256, 2, 16>(buf, out, 4096, 256);
    run<128, 1, 12>(buf, out, 5376, 260);
    run<256, 2, 12>(buf, out, 5376, 260);
    return 0;
}
