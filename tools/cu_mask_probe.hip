// Where do workgroups of a CU-masked stream land, and does such a stream
// synchronise with the legacy null stream?  The backup's digest streams are
// created the same way (cdc_backup.cpp: hipExtStreamCreateWithCUMask with
// every other CU bit set).
//   hipcc --offload-arch=gfx950 -O2 -o tools/_bin/cu_mask_probe tools/cu_mask_probe.hip && tools/_bin/cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <map>
#include <set>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(64) void k_where(uint32_t *out, uint32_t spin)
{
    __shared__ uint32_t s[16384];  // 64 KiB: at most two workgroups per CU, like a digest workgroup (66 KiB)
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t x = s[(threadIdx.x * 7) & 63];
    for (uint32_t i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));      // HW_ID
        out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11)); // XCC_ID
    }
    if (x == 0x12345678u) out[0] = x;
}

static void place(const char *name, hipStream_t st, int wgs)
{
    uint32_t *d;
    (void)hipMalloc(&d, size_t(wgs) * 8);
    hipLaunchKernelGGL(k_where, dim3(wgs), dim3(64), 0, st, d, 400000u);
    (void)hipStreamSynchronize(st);
    std::vector<uint32_t> h(size_t(wgs) * 2);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    std::set<std::tuple<int, int, int, int>> cus;  // (xcc, se, sh, cu)
    std::map<int, std::set<std::tuple<int, int, int>>> per_xcc;
    std::map<int, int> cu_ids;
    for (int b = 0; b < wgs; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 15u;
        const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cus.insert({int(xcc), se, sh, cu});
        per_xcc[int(xcc)].insert({se, sh, cu});
        cu_ids[cu]++;
    }
    printf("%s: %d workgroups on %zu distinct CUs\n", name, wgs, cus.size());
    for (auto &kv : per_xcc) {
        std::set<int> ses;
        for (auto &t : kv.second) ses.insert(std::get<0>(t));
        printf("  xcc %d: %zu CUs over %zu SEs\n", kv.first, kv.second.size(), ses.size());
    }
    printf("  workgroups per CU_ID field:");
    for (auto &kv : cu_ids) printf(" %d:%d", kv.first, kv.second);
    printf("\n");
}

static double wait_behind_null(const char *name, hipStream_t st)
{
    uint32_t *d;
    (void)hipMalloc(&d, 1 << 20);
    (void)hipDeviceSynchronize();
    // a long kernel on the legacy null stream, then a short one on `st`
    hipLaunchKernelGGL(k_where, dim3(64), dim3(64), 0, nullptr, d, 40000000u);
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_where, dim3(1), dim3(64), 0, st, d + 4096, 1u);
    (void)hipStreamSynchronize(st);
    const double ms_st = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    (void)hipDeviceSynchronize();
    const double ms_all = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    (void)hipFree(d);
    unsigned flags = 0;
    (void)hipStreamGetFlags(st, &flags);
    printf("%s: flags %u; its short kernel done after %.2f ms, the null stream's long one after %.2f ms (%s)\n",
           name, flags, ms_st, ms_all, ms_st > 0.5 * ms_all ? "waited for the null stream" : "did not wait");
    return ms_st;
}

int main()
{
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<uint32_t> m(size_t((cus + 31) / 32), 0u);
    for (int c = 0; c < cus; c += 2) m[size_t(c / 32)] |= 1u << (c % 32);
    hipStream_t masked = nullptr, plain = nullptr;
    if (hipExtStreamCreateWithCUMask(&masked, uint32_t(m.size()), m.data()) != hipSuccess) {
        printf("hipExtStreamCreateWithCUMask failed\n");
        return 1;
    }
    (void)hipStreamCreateWithFlags(&plain, hipStreamNonBlocking);
    printf("device CUs: %d; mask = every other bit (%zu words)\n", cus, m.size());
    place("unmasked (non-blocking stream)", plain, 4 * cus);
    place("masked (every other CU bit)", masked, 4 * cus);
    wait_behind_null("non-blocking stream", plain);
    wait_behind_null("CU-masked stream", masked);
    return 0;
}
