// Per-chunk digests on MI355X (gfx950): SHA-256 of every chunk and, on
// request, its byte histogram, for a device-resident buffer and its device
// cut list.  Replaces the per-chunk work of plakar's processChunk
// (snapshot/backup.go:594-629): chunkHasher.Write/Sum (backup.go:604-606,
// hashing "SHA256" = crypto/sha256, hashing/hashing.go:31-36) and the
// frequency count of entropy() (backup.go:548-557).  The float64 entropy is
// left to the caller, whose math.Log2 and summation order define it.
//
// SHA-256 is a serial chain over a message's 64-byte blocks, so the unit of
// parallelism is the chunk: one lane per chunk (FIPS 180-4, multi-buffer
// style), one wave per workgroup.  Each lane reads its chunk as aligned
// dwords and builds the big-endian message words with one v_perm_b32 per
// word (funnel shift + byte swap).  The histogram is kept per lane in LDS,
// transposed (bin b of lane l at 4 * (64 b + l)) so that every lane always
// hits its own bank: 64 KiB per wave.
//
// Roofline: VALU-bound (~1,400 VALU per 64-byte block per lane); the time is
// set by the longest chunk of the launch (blocks x dependent-chain latency),
// see DESIGN.md.
#include <hip/hip_runtime.h>

#include "cdc_internal.h"

namespace cdc {

__constant__ uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c in one VALU
}

// One SHA-256 compression of the 16 big-endian words w into h.
__device__ __forceinline__ void sha256_block(uint32_t (&h)[8], uint32_t (&w)[16])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
            w[t & 15] = wt;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);   // (e & f) | (~e & g)
        const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);   // majority
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + S0 + mj;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}

constexpr uint32_t kDigestHistBytes = 256u * 64u * 4u;  // 64 KiB: one wave's transposed histograms

// grid (ceil(max cap / 64), nbufs) workgroups of 64: lane i of workgroup
// (w, b) owns chunk 64 w + i of buffer b, so every chunk of the launch group
// hashes in parallel (a launch lasts as long as its longest chunk).
template <bool HIST>
__global__ __launch_bounds__(64) void k_chunk_digest(const DigestBatch DB)
{
    extern __shared__ uint32_t s_hist[];  // [256][64] when HIST
    const DigestBuf &B = DB.b[blockIdx.y];
    const uint8_t *data = B.data;
    const uint64_t len = B.len, cap = B.cap;
    const cdc_cut *cuts = B.cuts;
    const cdc_result *res = B.res;
    uint8_t *digests = B.digests;
    uint32_t *hist = B.hist;
    const uint32_t lane = threadIdx.x;
    uint64_t n_cuts = cap;
    if (res) n_cuts = min<uint64_t>(cap, uint64_t(res->ncuts));
    const uint64_t i = uint64_t(blockIdx.x) * 64u + lane;
    if (HIST) {
#pragma unroll 8
        for (uint32_t b = 0; b < 256; ++b) s_hist[b * 64u + lane] = 0;
    }
    if (i >= n_cuts) return;
    if (HIST && !hist) return;  // launch-wide HIST, this buffer wants digests only: not a case the API makes
    const cdc_cut cut = cuts[i];
    uint64_t n = cut.length;
    if (cut.offset > len) n = 0;
    else if (n > len - cut.offset) n = len - cut.offset;  // clipped to the buffer (a malformed list must not fault)
    const uint8_t *p = data + cut.offset;
    auto count = [&](uint32_t word_be, uint32_t nbytes) {  // histogram of the first nbytes of a big-endian word
        if (!HIST) return;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (j < nbytes) {
                const uint32_t bv = (word_be >> (24u - 8u * j)) & 0xFFu;
                __hip_atomic_fetch_add(&s_hist[bv * 64u + lane], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
    };

    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint32_t w[16];
    // full blocks: aligned dword loads, v_perm funnel shift + byte swap
    const uint64_t nfull = n / 64u;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    const uint32_t sel = (sh << 24) | ((sh + 1u) << 16) | ((sh + 2u) << 8) | (sh + 3u);
    // derived from the kernel argument (not through an integer), so the loads
    // are global_load, not flat
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p - sh);
    if (nfull) {
        // software pipeline: block b + 1's words are loaded before block b is
        // compressed (~1,400 VALU), so the load latency is not exposed
        // Block b uses dwords q[16 b .. 16 b + 16].  With sh == 0 the last one
        // holds no byte of the block (v_perm selects only `lo`), and for the
        // last block it can lie past the buffer end: it is not loaded then.
        auto load16 = [&](const uint32_t *qb, bool last, uint32_t (&x)[16]) {
#pragma unroll
            for (int k = 0; k < 15; ++k) x[k] = qb[k];
            x[15] = qb[(last && sh == 0) ? 14 : 15];  // index select: no load past the chunk
        };
        uint32_t lo = q[0];
        const uint32_t *qb = q + 1;
        uint32_t nx[16];
        load16(qb, nfull == 1, nx);
        for (uint64_t blk = 0; blk < nfull; ++blk) {
            uint32_t dw[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) dw[k] = nx[k];
            qb += 16;
            if (blk + 1 < nfull) load16(qb, blk + 2 == nfull, nx);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                w[k] = __builtin_amdgcn_perm(dw[k], lo, sel);
                lo = dw[k];
                count(w[k], 4);
            }
            sha256_block(h, w);
        }
    }
    // the last 1 or 2 blocks: the remaining r < 64 bytes, 0x80, zeros, bit length
    const uint64_t r = n - nfull * 64u;
    const uint8_t *tail = p + nfull * 64u;
    const uint32_t nfin = r <= 55u ? 1u : 2u;
    for (uint32_t fb = 0; fb < nfin; ++fb) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t word = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint64_t pos = uint64_t(fb) * 64u + uint64_t(k) * 4u + j;
                uint32_t byte = 0;
                if (pos < r) byte = tail[pos];
                else if (pos == r) byte = 0x80u;
                word |= byte << (24u - 8u * j);
            }
            const uint64_t kpos = uint64_t(fb) * 64u + uint64_t(k) * 4u;
            if (kpos < r) count(word, uint32_t(min<uint64_t>(4u, r - kpos)));
            w[k] = word;
        }
        if (fb + 1 == nfin) {
            const uint64_t bits = n * 8u;
            w[14] = uint32_t(bits >> 32);
            w[15] = uint32_t(bits);
        }
        sha256_block(h, w);
    }
    uint4 *out = reinterpret_cast<uint4 *>(digests + i * 32u);
    auto bswap = [](uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); };
    out[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
    out[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
    if (HIST) {
        uint4 *ho = reinterpret_cast<uint4 *>(hist + i * 256u);
#pragma unroll 4
        for (uint32_t b = 0; b < 256; b += 4)
            ho[b / 4] = make_uint4(s_hist[b * 64u + lane], s_hist[(b + 1) * 64u + lane], s_hist[(b + 2) * 64u + lane],
                                   s_hist[(b + 3) * 64u + lane]);
    }
}

int launch_digests(const DigestBatch &DB, void *stream)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    uint64_t cap = 0;
    bool hist = false;
    for (uint32_t i = 0; i < DB.nbufs; ++i) {
        cap = DB.b[i].cap > cap ? DB.b[i].cap : cap;
        hist |= DB.b[i].hist != nullptr;
    }
    if (cap == 0 || DB.nbufs == 0) return CDC_OK;
    if ((cap + 63) / 64 > 0x7FFFFFFFull) return CDC_E_INVALID;
    const dim3 grid(uint32_t((cap + 63) / 64), DB.nbufs), block(64);
    if (hist)
        hipLaunchKernelGGL(k_chunk_digest<true>, grid, block, kDigestHistBytes, st, DB);
    else
        hipLaunchKernelGGL(k_chunk_digest<false>, grid, block, 0, st, DB);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

}  // namespace cdc
