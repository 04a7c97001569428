// VALU issue-rate microbenchmark (gfx950): W waves per CU (one workgroup per
// CU), each issuing 8 independent streams of one instruction kind; reports
// shader cycles per wave-instruction per SIMD (s_memtime ticks = shader
// cycles).  hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubv
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int OP>
__device__ __forceinline__ void step(uint32_t (&x)[8], uint64_t (&y)[8], uint32_t m)
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(m));
        if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(m));
        if constexpr (OP == 2) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(y[i]) : "v"(y[(i + 1) & 7]));
        if constexpr (OP == 3) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(m));
        if constexpr (OP == 4) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 3) & 7]));
        if constexpr (OP == 5) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0xea" : "+v"(x[i]) : "v"(m));
        if constexpr (OP == 6) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(m));
        if constexpr (OP == 7) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(y[i]));
        if constexpr (OP == 8) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(x[i]), "+v"(m), "+v"(x[(i+4)&7]) :: "vcc");
        if constexpr (OP == 9) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(m));
    }
}

template <int OP>
__global__ void kern(uint32_t *out, uint64_t *cyc, int iters, uint32_t m0)
{
    uint32_t x[8];
    uint64_t y[8];
    for (int i = 0; i < 8; ++i) {
        x[i] = threadIdx.x * (i + 1);
        y[i] = x[i] * 0x9E3779B97F4A7C15ull;
    }
    uint32_t m = m0 ^ threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) step<OP>(x, y, m);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= x[i] ^ uint32_t(y[i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char *name, int W, uint32_t *out, uint64_t *cyc)
{
    const int iters = 2000, nblk = 256;
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(W * 64), 0, 0, out, cyc, 10, 1u);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(W * 64), 0, 0, out, cyc, iters, 1u);
    hipDeviceSynchronize();
    uint64_t h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nblk; ++i) avg += double(h[i]);
    avg /= nblk;
    const double ninst = double(iters) * 64 * (OP == 8 ? 2 : 1);  // per wave
    const double wps = W / 4.0;                                       // waves per SIMD
    printf("%-16s W=%2d  %.2f cycles per wave-instruction per SIMD (wave alone %.2f)\n", name, W,
           avg / (ninst * wps), avg / ninst);
}

int main()
{
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&cyc, 256 * 8);
    for (int W : {4, 12}) {
        run<0>("v_and_b32", W, out, cyc);
        run<1>("v_perm_b32", W, out, cyc);
        run<2>("v_lshl_add_u64", W, out, cyc);
        run<3>("v_min3_u32", W, out, cyc);
        run<4>("v_mov_b32", W, out, cyc);
        run<5>("v_bitop3_b32", W, out, cyc);
        run<6>("v_add_u32", W, out, cyc);
        run<7>("v_lshlrev_b64", W, out, cyc);
        run<8>("add_co+addc", W, out, cyc);
        run<9>("v_cndmask_b32", W, out, cyc);
    }
    return 0;
}
