// Inner-loop ceiling microbenchmark: the scan's per-byte Gear roll + MaskS
// test over register-resident data (no global traffic), at several waves per
// SIMD and with parts removed, to find what bounds the scan kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r; asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r;
}
__device__ __forceinline__ uint32_t word_of(const uint4 &d, int i) { return i == 0 ? d.x : i == 1 ? d.y : i == 2 ? d.z : d.w; }

template <int MODE, int NT>  // 0 full, 1 no gather (g = addr), 2 no perm (fixed addr), 3 gather only
__global__ __launch_bounds__(NT) void loopk(uint32_t* out, int iters, uint32_t mlo, uint32_t mhi) {
  __shared__ uint64_t tab[256 * 32];
  for (int i = threadIdx.x; i < 8192; i += NT) tab[i] = 0x9E3779B97F4A7C15ull * (i + 1);
  __syncthreads();
  const char* t = (const char*)tab;
  const uint32_t laneoff = (threadIdx.x & 31) << 3;
  uint4 d = make_uint4(threadIdx.x * 0x01010101u, threadIdx.x * 0x02030405u, threadIdx.x * 0x0a0b0c0du, blockIdx.x * 0x11223344u);
  uint64_t fp = threadIdx.x;
  uint32_t acc = 0xffffffffu;
  for (int it = 0; it < iters; ++it) {
    uint64_t g[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t a;
      if constexpr (MODE == 2) a = ((k * 37) << 8) | laneoff; else a = __builtin_amdgcn_perm(laneoff, word_of(d, k >> 2), 0x0C0C0004u | ((k & 3) << 8));
      if constexpr (MODE == 1) g[k] = a; else g[k] = *(const uint64_t*)(t + a);
    }
    if constexpr (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 16; ++k) fp ^= g[k];
    } else {
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        fp = (fp << 1) + g[k];
        uint32_t k0 = ((uint32_t)fp & mlo) | ((uint32_t)(fp >> 32) & mhi);
        fp = (fp << 1) + g[k + 1];
        acc = umin3(acc, k0, ((uint32_t)fp & mlo) | ((uint32_t)(fp >> 32) & mhi));
      }
    }
    d.x += 0x01010101u; d.y ^= d.x; d.z += d.y; d.w ^= d.z;   // new data each iteration
  }
  out[blockIdx.x * NT + threadIdx.x] = acc ^ (uint32_t)fp ^ (uint32_t)(fp >> 32);
}

template <int MODE, int NT>
void run(const char* name, int bpc, uint32_t* d) {
  int nblk = 256 * bpc;  // bpc blocks per CU, NT/256 waves per SIMD each
  int iters = 2000;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((loopk<MODE, NT>), dim3(nblk), dim3(NT), 0, 0, d, iters, 0x03530000u, 0x00035907u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL((loopk<MODE, NT>), dim3(nblk), dim3(NT), 0, 0, d, iters, 0x03530000u, 0x00035907u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double bytes = double(nblk) * NT * iters * 16;
  printf("%-12s waves/SIMD=%d  %8.1f GB/s-equivalent  (%.3f ms)\n", name, bpc * NT / 256, bytes / (ms * 1e-3) / 1e9, ms);
}

int main() {
  uint32_t* d; hipMalloc(&d, 256 * 1024 * 16 * 4);
  run<0, 256>("full", 1, d); run<0, 256>("full", 2, d); run<0, 512>("full", 2, d); run<0, 1024>("full", 1, d);
  run<1, 256>("no-gather", 2, d); run<1, 512>("no-gather", 2, d);
  run<2, 256>("no-perm", 2, d); run<2, 512>("no-perm", 2, d);
  run<3, 256>("gather-only", 2, d); run<3, 512>("gather-only", 2, d);
  return 0;
}
