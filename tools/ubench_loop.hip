// The byte scan's inner loop with no memory traffic (gfx950): W waves per CU
// (one workgroup per CU), each lane rolling 16-byte groups of synthetic bytes
// through the 32-copy LDS Gear table exactly as k_scan does (v_perm address,
// ds_read_b64 gather one group ahead, v_lshl_add_u64 chain, hi-dword filter
// with v_and + v_min3).  Reports shader cycles per 16-byte group per SIMD,
// i.e. the loop's compute ceiling at each occupancy.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_loop.hip -o /tmp/ubl && /tmp/ubl
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t gear_addr(uint32_t laneoff, uint32_t word, int k)
{
    return __builtin_amdgcn_perm(laneoff, word, 0x0C0C0004u | (uint32_t(k & 3) << 8));
}
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t word_of(const uint4 &d, int i) { return i == 0 ? d.x : i == 1 ? d.y : i == 2 ? d.z : d.w; }

// MODE 0: full loop (perm + gather + chain + filter); 1: no filter; 2: chain + filter, gathers replaced by
// a register table value (no LDS)
template <int W, int MODE>
__global__ __launch_bounds__(W * 64) void kern(uint32_t *out, uint64_t *cyc, int groups, uint32_t vhi)
{
    __shared__ uint64_t tab[256 * 32];
    for (uint32_t i = threadIdx.x; i < 256 * 32; i += W * 64) tab[i] = (0x9E3779B97F4A7C15ull * (i / 32 + 1)) << 14;
    __syncthreads();
    const char *t = reinterpret_cast<const char *>(tab);
    const uint32_t lane = threadIdx.x & 63, laneoff = (lane & 31) << 3;
    uint4 d = make_uint4(threadIdx.x * 0x01010101u, threadIdx.x * 0x3u + 7, blockIdx.x, 0x12345678u);
    uint64_t gv[2][16];
    for (int k = 0; k < 16; ++k) gv[0][k] = *reinterpret_cast<const uint64_t *>(t + gear_addr(laneoff, word_of(d, k >> 2), k));
    uint64_t fp = 0;
    uint32_t hits = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int g = 0; g < groups; g += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint64_t (&cg)[16] = gv[h];
            uint64_t (&ng)[16] = gv[h ^ 1];
            const uint4 nx = make_uint4(d.x + uint32_t(g) * 0x9E3779B9u, d.y ^ uint32_t(g), d.z + uint32_t(g), d.w ^ (uint32_t(g) << 7));
            uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < 16; k += 2) {
                const uint32_t a0 = gear_addr(laneoff, word_of(nx, k >> 2), k);
                fp = (fp << 1) + cg[k];
                if (MODE == 2) ng[k] = uint64_t(a0) * 0x100000001ull;
                else ng[k] = *reinterpret_cast<const uint64_t *>(t + a0);
                const uint32_t k0 = uint32_t(fp >> 32) & vhi;
                const uint32_t a1 = gear_addr(laneoff, word_of(nx, (k + 1) >> 2), k + 1);
                fp = (fp << 1) + cg[k + 1];
                if (MODE == 2) ng[k + 1] = uint64_t(a1) * 0x100000001ull;
                else ng[k + 1] = *reinterpret_cast<const uint64_t *>(t + a1);
                if (MODE != 1) acc = umin3(acc, k0, uint32_t(fp >> 32) & vhi);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (MODE != 1 && acc == 0) ++hits;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = hits ^ uint32_t(fp) ^ uint32_t(fp >> 32);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int W, int MODE>
void run(const char *name, uint32_t *out, uint64_t *cyc)
{
    const int groups = 4000, nblk = 256;
    hipLaunchKernelGGL((kern<W, MODE>), dim3(nblk), dim3(W * 64), 0, 0, out, cyc, 10, 0xD641C0D4u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((kern<W, MODE>), dim3(nblk), dim3(W * 64), 0, 0, out, cyc, groups, 0xD641C0D4u);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nblk; ++i) avg += double(h[i]);
    avg /= nblk;
    const double wps = W / 4.0;  // waves per SIMD
    const double bytes = double(nblk) * W * 64 * 16 * groups;
    printf("%-22s W=%2d  %7.1f cycles per group per SIMD  (wave %7.1f per group)  %7.1f GB/s-equivalent (%.3f ms)\n",
           name, W, avg / (groups * wps), avg / groups, bytes / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&cyc, 256 * 8);
    run<4, 0>("full", out, cyc);
    run<8, 0>("full", out, cyc);
    run<12, 0>("full", out, cyc);
    run<16, 0>("full", out, cyc);
    run<20, 0>("full", out, cyc);
    run<12, 1>("no filter", out, cyc);
    run<16, 1>("no filter", out, cyc);
    run<12, 2>("no LDS gathers", out, cyc);
    run<16, 2>("no LDS gathers", out, cyc);
    run<24, 2>("no LDS gathers", out, cyc);
    return 0;
}
