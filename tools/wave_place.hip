// Where do a workgroup's waves land?  Records HW_ID (SIMD, CU, SE, XCC-local)
// of every wave for a few workgroup shapes and prints, per shape, how often
// waves w and w' of one workgroup share a SIMD.
//   hipcc --offload-arch=gfx950 -O2 -o tools/wave_place.bin tools/wave_place.hip && tools/wave_place.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int WAVES, int LDS_KIB>
__global__ __launch_bounds__(WAVES * 64) void k_place(uint32_t *out, uint32_t spin)
{
    __shared__ uint32_t s[LDS_KIB * 256];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t x = s[(threadIdx.x * 7) % (WAVES * 64)];
    for (uint32_t i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;  // keep the workgroup resident a while
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * WAVES + (threadIdx.x >> 6)] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    if (x == 0x12345678u) out[0] = x;
}

template <int WAVES, int LDS_KIB>
void run(int wgs)
{
    uint32_t *d;
    hipMalloc(&d, wgs * WAVES * 4);
    hipLaunchKernelGGL((k_place<WAVES, LDS_KIB>), dim3(wgs), dim3(WAVES * 64), 0, 0, d, 200000u);
    hipDeviceSynchronize();
    std::vector<uint32_t> h(wgs * WAVES);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    // same-SIMD matrix over wave pairs
    int same[8][8] = {};
    for (int b = 0; b < wgs; ++b)
        for (int i = 0; i < WAVES; ++i)
            for (int j = 0; j < WAVES; ++j)
                same[i][j] += ((h[b * WAVES + i] >> 4) & 3) == ((h[b * WAVES + j] >> 4) & 3);
    printf("%d waves/WG, %d KiB LDS, %d WGs: fraction of WGs where waves i, j share a SIMD\n", WAVES, LDS_KIB, wgs);
    for (int i = 0; i < WAVES; ++i) {
        printf("  w%d:", i);
        for (int j = 0; j < WAVES; ++j) printf(" %.2f", double(same[i][j]) / wgs);
        printf("\n");
    }
    printf("  first WG simd ids:");
    for (int i = 0; i < WAVES; ++i) printf(" %u", (h[i] >> 4) & 3);
    printf("\n");
}

int main()
{
    run<6, 128>(240);
    run<6, 128>(256);
    run<3, 64>(480);
    run<3, 64>(171);
    run<4, 64>(256);
    run<8, 128>(256);
    return 0;
}
