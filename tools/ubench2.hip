// VALU issue-throughput microbenchmark (gfx950), 8 independent chains per wave
// so dependent latency is hidden: cycles per wave-instruction per SIMD, from
// s_memtime inside the kernel, at 1 and 2 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench2.hip -o tools/ubench2.bin && tools/ubench2.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 2048
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void kern(uint64_t *cyc, uint32_t seed)
{
    uint32_t a[8], b[8];
    uint64_t f[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * (i + 3) ^ seed;
        b[i] = a[i] * 7 + i;
        f[i] = (uint64_t(a[i]) << 32) | b[i];
    }
    const uint32_t s = seed | 1;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_ITER; ++it) {
#define LSHLADD64(i) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f[i]) : "v"(f[(i + 1) & 7]));
#define PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "s"(s));
#define ANDVV(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
#define ANDSV(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[i]) : "s"(s));
#define ANDOR(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(s), "v"(b[i]));
#define ANDORV(i) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[(i + 1) & 7]), "v"(b[i]));
#define MIN3(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 1) & 7]));
#define MINVV(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
#define ADDVV(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
#define BITOP3(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe0" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 1) & 7]));
#define XORVV(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
#define LSHLADD32(i) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a[i]) : "v"(b[i]));
#define ALIGNBIT(i) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(a[i]) : "v"(b[i]));
#define LSHL64(i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(f[i]));
#define ADDC(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b[i]) : "vcc");
#define MOVDPP(i) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(b[i]));
        if constexpr (OP == 0) { R8(LSHLADD64) }
        else if constexpr (OP == 1) { R8(PERM) }
        else if constexpr (OP == 2) { R8(ANDVV) }
        else if constexpr (OP == 3) { R8(ANDSV) }
        else if constexpr (OP == 4) { R8(ANDOR) }
        else if constexpr (OP == 5) { R8(ANDORV) }
        else if constexpr (OP == 6) { R8(MIN3) }
        else if constexpr (OP == 7) { R8(MINVV) }
        else if constexpr (OP == 8) { R8(ADDVV) }
        else if constexpr (OP == 9) { R8(BITOP3) }
        else if constexpr (OP == 10) { R8(XORVV) }
        else if constexpr (OP == 11) { R8(LSHLADD32) }
        else if constexpr (OP == 12) { R8(ALIGNBIT) }
        else if constexpr (OP == 13) { R8(LSHL64) }
        else if constexpr (OP == 14) { R8(ADDC) }
        else if constexpr (OP == 15) { R8(MOVDPP) }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int i = 0; i < 8; ++i) x ^= a[i] ^ uint32_t(f[i]) ^ uint32_t(f[i] >> 32);
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = (t1 - t0) | (uint64_t(x & 1) << 63);
}

static const char *names[] = {"v_lshl_add_u64", "v_perm_b32(s)", "v_and_b32 v,v", "v_and_b32 s,v", "v_and_or_b32 (s)",
                              "v_and_or_b32 (v)", "v_min3_u32", "v_min_u32 v,v", "v_add_u32 v,v", "v_bitop3_b32",
                              "v_xor_b32 v,v", "v_lshl_add_u32", "v_alignbit_b32", "v_lshlrev_b64", "v_add_co_u32",
                              "v_mov_b32_dpp"};

template <int OP>
void run(int wps)
{
    const int blocks = 256, threads = 64 * 4 * wps;  // 4 SIMDs x wps waves per CU
    uint64_t *d;
    hipMalloc(&d, blocks * threads / 64 * 8);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipDeviceSynchronize();
    const int n = blocks * threads / 64;
    uint64_t *h = new uint64_t[n];
    hipMemcpy(h, d, n * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < n; ++i) sum += double(h[i] & ~(1ull << 63));
    const double per_wave = sum / n;
    // cycles per wave-instruction per SIMD = wave cycles / (instructions per wave * waves sharing the SIMD)
    printf("%-18s waves/SIMD=%d  %.2f cyc per wave-instr per SIMD\n", names[OP], wps, per_wave / (8.0 * N_ITER * wps));
    delete[] h;
    hipFree(d);
}

template <int OP>
void runall()
{
    run<OP>(1);
    run<OP>(2);
    if constexpr (OP + 1 < 16) runall<OP + 1>();
}

int main()
{
    runall<0>();
    return 0;
}
