// The byte scan's inner loop (as tools/ubench_loop.hip: v_perm address,
// ds_read_b64 gather one group ahead, v_lshl_add_u64 chain, hi-dword filter)
// with the scan's memory traffic added piece by piece, to see what the real
// k_scan's per-group cycles (about 1.9x the bare loop's, compute-bound at a
// cold clock) are made of.  12 waves per CU, one workgroup per CU, each wave
// 64 runs of 5,632 B of a 1.1-GB buffer; one stage = 4 groups = 64 B per lane.
//   MODE 0: the bare loop (bytes from registers)
//   MODE 1: + LDS-DMA of the stage's 4 KiB into the wave's slot (4 x
//           global_load_lds_dwordx4, 8 runs x 128 B each), vmcnt(0) before
//           the next issue; bytes still from registers
//   MODE 2: MODE 1 + the row reads (8 ds_read_b128, half the wave), bytes
//           still from registers
//   MODE 3: the row reads only (no DMA)
//   MODE 4: bytes loaded straight into registers (4 global_load_dwordx4 per
//           lane per stage, its own run, one stage ahead), no LDS slot
//   MODE 5: MODE 4 with the loop's bytes taken from the loaded registers
// Reports shader cycles per 16-byte group per wave and the kernel's rate.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_loop2.hip -o tools/_bin/ubl2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int W = 12;
constexpr uint32_t SL = 5632;  // bytes per run

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

__device__ __forceinline__ void dma4(uint64_t base_in, uint32_t dst_in, const uint32_t (&off)[4])
{
    const uint64_t base = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in >> 32)))) << 32) |
                          uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(base_in)));
    const uint32_t dst = __builtin_amdgcn_readfirstlane(dst_in);
    uint32_t keep;
    asm volatile("s_nop 4\n\ts_mov_b32 %[keep], m0\n\ts_mov_b32 m0, %[dst]\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %2, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %3, %[base]\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %4, %[base]\n\t"
                 "s_mov_b32 m0, %[keep]\n\ts_nop 1"
                 : [keep] "=&s"(keep)
                 : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), [base] "s"(base), [dst] "s"(dst)
                 : "memory", "scc");
}

// 4x4 transpose of 16-B pieces within each lane quad: before, lane 4q+i
// register k holds piece i of run 16k+q; after, lane 4q+i register k holds
// piece k of run 16i+q.  Two butterfly stages (xor 1, xor 2 lanes), each a
// DPP quad_perm read of the partner's register and a per-lane select.
__device__ __forceinline__ uint32_t qperm1(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }  // [1,0,3,2]
__device__ __forceinline__ uint32_t qperm2(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }  // [2,3,0,1]
__device__ __forceinline__ void quad_transpose(uint4 (&r)[4], uint32_t lane)
{
    const bool b0 = lane & 1u, b1 = lane & 2u;
    auto xch = [&](uint4 &lo, uint4 &hi, bool b, auto perm) {
        // b = 0: lo keeps, hi <- partner's lo;  b = 1: lo <- partner's hi, hi keeps
        uint32_t *pl = reinterpret_cast<uint32_t *>(&lo), *ph = reinterpret_cast<uint32_t *>(&hi);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t send = b ? pl[d] : ph[d];
            const uint32_t recv = perm(send);
            const uint32_t nl = b ? recv : pl[d], nh = b ? ph[d] : recv;
            pl[d] = nl;
            ph[d] = nh;
        }
    };
    xch(r[0], r[1], b0, qperm1);
    xch(r[2], r[3], b0, qperm1);
    xch(r[0], r[2], b1, qperm2);
    xch(r[1], r[3], b1, qperm2);
}

template <int MODE>
__global__ __launch_bounds__(W * 64) void kern(const uint8_t *buf, uint32_t *out, uint64_t *cyc, int stages,
                                               uint32_t vhi)
{
    __shared__ __attribute__((aligned(16))) char s[256 * 32 * 8 + W * 4096];
    uint64_t *tab = reinterpret_cast<uint64_t *>(s);
    for (uint32_t i = threadIdx.x; i < 256 * 32; i += W * 64) tab[i] = (0x9E3779B97F4A7C15ull * (i / 32 + 1)) << 14;
    __syncthreads();
    const char *t = s;
    const uint32_t lane = threadIdx.x & 63, laneoff = (lane & 31) << 3, wave = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * W + wave;
    const uint64_t wbase = reinterpret_cast<uint64_t>(buf) + uint64_t(gw) * 64 * SL;
    const uint32_t ring = uint32_t(reinterpret_cast<uintptr_t>(s)) + 256 * 32 * 8 + wave * 4096;
    uint32_t off[4];
    for (int j = 0; j < 4; ++j) off[j] = (8 * j + lane / 8) * SL + 16 * (lane % 8);
    const char *rowp = s + 256 * 32 * 8 + wave * 4096 + (lane & 31) * 128;
    const uint8_t *myrun = buf + uint64_t(gw) * 64 * SL + uint64_t(lane) * SL;
    // MODE 6-8: quad loads (lane 4q+i: piece i of run 16k+q); 7/8: every wave reads the same 360-KiB region
    const uint8_t *wreg = (MODE == 7 || MODE == 8) ? buf : buf + uint64_t(gw) * 64 * SL;
    auto qload = [&](uint4 (&r)[4], int st) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            r[k] = *reinterpret_cast<const uint4 *>(wreg + uint64_t(16 * k + lane / 4) * SL + 64 * (st % 88) + 16 * (lane % 4));
    };
    uint4 d = make_uint4(threadIdx.x * 0x01010101u, threadIdx.x * 0x3u + 7, blockIdx.x, 0x12345678u);
    uint4 cur[4], nxt[4];
    if (MODE == 4 || MODE == 5)
        for (int j = 0; j < 4; ++j) cur[j] = *reinterpret_cast<const uint4 *>(myrun + 16 * j);
    if (MODE == 6 || MODE == 7) {
        qload(cur, 0);
        quad_transpose(cur, lane);
    }
    uint64_t gv[2][16];
    for (int k = 0; k < 16; ++k) gv[0][k] = *reinterpret_cast<const uint64_t *>(t + gear_addr(laneoff, word_of(d, k >> 2), k));
    uint64_t fp = 0;
    uint32_t hits = 0, sink = 0;
    const uint64_t dbase = MODE == 8 ? reinterpret_cast<uint64_t>(buf) : wbase;
    if (MODE == 1 || MODE == 2 || MODE == 8) dma4(dbase, ring, off);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int st = 0; st < stages; ++st) {
        if (MODE == 4 || MODE == 5) {
            const int sn = st + 1 < stages ? st + 1 : st;
#pragma unroll
            for (int j = 0; j < 4; ++j) nxt[j] = *reinterpret_cast<const uint4 *>(myrun + 64 * (sn % 88) + 16 * j);
        }
        if (MODE == 6 || MODE == 7) qload(nxt, st + 1 < stages ? st + 1 : st);
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
            uint64_t (&cg)[16] = gv[gi & 1];
            uint64_t (&ng)[16] = gv[(gi & 1) ^ 1];
            if (gi == 3 && (MODE == 6 || MODE == 7)) quad_transpose(nxt, lane);
            if (gi == 3 && (MODE == 1 || MODE == 2 || MODE == 8)) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if ((MODE == 2 || MODE == 8) && (lane >> 5) == (uint32_t(st) & 1)) {
                    uint4 r[8];
#pragma unroll
                    for (int g = 0; g < 8; ++g) r[g] = *reinterpret_cast<const uint4 *>(rowp + 16 * (g ^ ((lane >> 1) & 7)));
#pragma unroll
                    for (int g = 0; g < 8; ++g) sink ^= r[g].x ^ r[g].w;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                dma4(dbase + uint64_t(((st + 1) / 2) % 44) * 128 + uint64_t((st + 1) & 1) * 32ull * SL, ring, off);
            }
            if (gi == 3 && MODE == 3 && (lane >> 5) == (uint32_t(st) & 1)) {
                uint4 r[8];
#pragma unroll
                for (int g = 0; g < 8; ++g) r[g] = *reinterpret_cast<const uint4 *>(rowp + 16 * (g ^ ((lane >> 1) & 7)));
#pragma unroll
                for (int g = 0; g < 8; ++g) sink ^= r[g].x ^ r[g].w;
            }
            uint4 nx;
            if (MODE == 5 || MODE == 6 || MODE == 7) nx = gi < 3 ? cur[gi + 1] : nxt[0];
            else nx = make_uint4(d.x + uint32_t(st * 4 + gi) * 0x9E3779B9u, d.y ^ uint32_t(st), d.z + uint32_t(gi), d.w ^ (uint32_t(st) << 7));
            uint32_t acc = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < 16; k += 2) {
                const uint32_t a0 = gear_addr(laneoff, word_of(nx, k >> 2), k);
                fp = (fp << 1) + cg[k];
                ng[k] = *reinterpret_cast<const uint64_t *>(t + a0);
                const uint32_t k0 = uint32_t(fp >> 32) & vhi;
                const uint32_t a1 = gear_addr(laneoff, word_of(nx, (k + 1) >> 2), k + 1);
                fp = (fp << 1) + cg[k + 1];
                ng[k + 1] = *reinterpret_cast<const uint64_t *>(t + a1);
                acc = umin3(acc, k0, uint32_t(fp >> 32) & vhi);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (acc == 0) ++hits;
        }
        if (MODE >= 4 && MODE <= 7) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (MODE == 4) sink ^= cur[j].x ^ cur[j].z;
                cur[j] = nxt[j];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = hits ^ uint32_t(fp) ^ uint32_t(fp >> 32) ^ sink;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char *name, const uint8_t *buf, uint32_t *out, uint64_t *cyc)
{
    const int stages = 88, nblk = 256;  // 88 x 64 B = 5,632 B per lane
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        for (int i = 0; i < 20; ++i)
            hipLaunchKernelGGL((kern<MODE>), dim3(nblk), dim3(W * 64), 0, 0, buf, out, cyc, stages, 0xD641C0D4u);
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t h[256];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < nblk; ++i) avg += double(h[i]);
        avg /= nblk;
        const double bytes = double(nblk) * W * 64 * SL;
        printf("%-34s rep %d: %7.1f cycles per group per wave, %7.1f us per launch, %6.0f GB/s\n", name, rep,
               avg / (stages * 4), ms * 1e3 / 20, bytes / (ms * 1e-3 / 20) / 1e9);
    }
}

int main()
{
    uint8_t *buf;
    uint32_t *out;
    uint64_t *cyc;
    const size_t n = size_t(256) * W * 64 * SL + 4096;
    hipMalloc(&buf, n);
    hipMemset(buf, 0x5A, n);
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&cyc, 256 * 8);
    run<0>("0 bare loop", buf, out, cyc);
    run<1>("1 + LDS-DMA", buf, out, cyc);
    run<2>("2 + LDS-DMA + row reads", buf, out, cyc);
    run<3>("3 + row reads only", buf, out, cyc);
    run<4>("4 + direct loads (unused)", buf, out, cyc);
    run<5>("5 direct loads feed the loop", buf, out, cyc);
    run<6>("6 quad loads + DPP transpose", buf, out, cyc);
    run<7>("7 = 6, L2-resident region", buf, out, cyc);
    run<8>("8 = 2 (LDS-DMA), L2-resident region", buf, out, cyc);
    run<3>("3 row reads only (again)", buf, out, cyc);
    run<0>("0 bare loop (again)", buf, out, cyc);
    return 0;
}
