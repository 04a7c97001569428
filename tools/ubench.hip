// Per-instruction throughput microbenchmark (gfx950): each kernel runs a long
// unrolled chain of independent instances of one instruction; reports cycles
// per wave-instruction per SIMD from wall time.  Used to cost the scan loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N_ITER 4096

#define BODY8(X) X X X X X X X X
template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 11, a5 = a0 + 13, a6 = a0 + 17, a7 = a0 + 19;
  uint64_t f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
  const uint32_t c = seed | 1;
  for (int i = 0; i < N_ITER; ++i) {
    if constexpr (OP == 0) {  // v_lshl_add_u64
#define X asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f0) : "v"(f1)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f2) : "v"(f3)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f4) : "v"(f5)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f6) : "v"(f7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 1) {  // v_perm_b32
#define X asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a0) : "v"(a1), "s"(c)); asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a2) : "v"(a3), "s"(c)); asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a4) : "v"(a5), "s"(c)); asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a6) : "v"(a7), "s"(c));
      BODY8(X)
#undef X
    } else if constexpr (OP == 2) {  // v_and_or_b32
#define X asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a0) : "s"(c), "v"(a1)); asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a2) : "s"(c), "v"(a3)); asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a4) : "s"(c), "v"(a5)); asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a6) : "s"(c), "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 3) {  // v_add_u32 (reference full-rate op)
#define X asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(a3)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(a5)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 4) {  // v_min3_u32
#define X asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a0) : "v"(a1), "v"(a2)); asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a3) : "v"(a4), "v"(a5)); asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a6) : "v"(a7), "v"(a1)); asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a2) : "v"(a4), "v"(a5));
      BODY8(X)
#undef X
    } else if constexpr (OP == 5) {  // v_add_co_u32 + v_addc_co_u32 pair (32-bit carry chain)
#define X asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a0), "+v"(a1) : "v"(a2), "v"(a3) : "vcc"); asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a4), "+v"(a5) : "v"(a6), "v"(a7) : "vcc");
      BODY8(X)
#undef X
    } else if constexpr (OP == 6) {  // v_lshlrev_b64
#define X asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(f0)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(f2)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(f4)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(f6));
      BODY8(X)
#undef X
    } else if constexpr (OP == 7) {  // v_lshl_add_u32
#define X asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a2) : "v"(a3)); asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a4) : "v"(a5)); asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a6) : "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 8) {  // v_mad_u64_u32
#define X asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(f0) : "v"(a1), "v"(a2) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(f2) : "v"(a3), "v"(a4) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(f4) : "v"(a5), "v"(a6) : "s0", "s1"); asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(f6) : "v"(a7), "v"(a1) : "s0", "s1");
      BODY8(X)
#undef X
    } else if constexpr (OP == 10) {  // v_mov_b32_sdwa byte insert (dst BYTE_1, preserve)
#define X asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a0) : "v"(a1)); asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a2) : "v"(a3)); asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a4) : "v"(a5)); asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a6) : "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 11) {  // v_and_b32 (VOP2 with SGPR)
#define X asm volatile("v_and_b32 %0, %1, %0" : "+v"(a0) : "s"(c)); asm volatile("v_and_b32 %0, %1, %0" : "+v"(a2) : "s"(c)); asm volatile("v_and_b32 %0, %1, %0" : "+v"(a4) : "s"(c)); asm volatile("v_and_b32 %0, %1, %0" : "+v"(a6) : "s"(c));
      BODY8(X)
#undef X
    } else if constexpr (OP == 12) {  // v_min_u32 (VOP2)
#define X asm volatile("v_min_u32 %0, %0, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_min_u32 %0, %0, %1" : "+v"(a2) : "v"(a3)); asm volatile("v_min_u32 %0, %0, %1" : "+v"(a4) : "v"(a5)); asm volatile("v_min_u32 %0, %0, %1" : "+v"(a6) : "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 13) {  // v_lshl_add_u64 single dependent chain (latency)
#define X asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f0) : "v"(f1)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f0) : "v"(f1)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f0) : "v"(f1)); asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(f0) : "v"(f1));
      BODY8(X)
#undef X
    } else if constexpr (OP == 14) {  // v_add_u32 single dependent chain (latency)
#define X asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
      BODY8(X)
#undef X
    } else if constexpr (OP == 15) {  // v_lshlrev_b32_sdwa byte extract + shift
#define X asm volatile("v_lshlrev_b32_sdwa %0, 8, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(a0) : "v"(a1)); asm volatile("v_lshlrev_b32_sdwa %0, 8, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(a2) : "v"(a3)); asm volatile("v_lshlrev_b32_sdwa %0, 8, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(a4) : "v"(a5)); asm volatile("v_lshlrev_b32_sdwa %0, 8, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(a6) : "v"(a7));
      BODY8(X)
#undef X
    } else if constexpr (OP == 9) {  // v_bfi_b32
#define X asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a0) : "s"(c), "v"(a1)); asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a2) : "s"(c), "v"(a3)); asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a4) : "s"(c), "v"(a5)); asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a6) : "s"(c), "v"(a7));
      BODY8(X)
#undef X
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a2 ^ a4 ^ a6 ^ (uint32_t)(f0 ^ f2 ^ f4 ^ f6) ^ (uint32_t)((f0 ^ f2 ^ f4 ^ f6) >> 32) ^ a1 ^ a3 ^ a5 ^ a7;
}

template <int OP>
void run(const char* name, int per_iter, int wpsimd, uint32_t* d) {
  // wpsimd waves per SIMD: blocks of 256 threads = 4 waves = 1 per SIMD
  int nblk = 256 * wpsimd;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(256), 0, 0, d, 7u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<OP>, dim3(nblk), dim3(256), 0, 0, d, 7u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double instr_per_wave = double(N_ITER) * per_iter;
  double cyc = ms * 1e-3 * 2.4e9;  // nominal clock
  // per SIMD: wpsimd waves each issuing instr_per_wave instructions
  printf("%-18s waves/SIMD=%d  %.2f cycles per wave-instr per SIMD (%.2f ms)\n", name, wpsimd,
         cyc / (instr_per_wave * wpsimd), ms);
}

int main() {
  uint32_t* d; hipMalloc(&d, 256 * 256 * 16 * 4);
  for (int w : {2, 4}) {
    run<10>("v_mov_b32_sdwa", 32, w, d);
    run<15>("v_lshlrev_sdwa", 32, w, d);
    run<11>("v_and_b32(s)", 32, w, d);
    run<12>("v_min_u32", 32, w, d);
  }
  run<13>("lshl_add_u64 chain", 32, 1, d);
  run<14>("add_u32 chain", 32, 1, d);
  for (int w : {4}) {
    run<3>("v_add_u32", 32, w, d);
    run<7>("v_lshl_add_u32", 32, w, d);
    run<0>("v_lshl_add_u64", 32, w, d);
    run<6>("v_lshlrev_b64", 32, w, d);
    run<1>("v_perm_b32", 32, w, d);
    run<2>("v_and_or_b32", 32, w, d);
    run<4>("v_min3_u32", 32, w, d);
    run<5>("v_add_co+addc", 32, w, d);
    run<8>("v_mad_u64_u32", 32, w, d);
    run<9>("v_bfi_b32", 32, w, d);
  }
  return 0;
}
