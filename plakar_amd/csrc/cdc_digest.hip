// Per-chunk digests on MI355X (gfx950): SHA-256 of every chunk and, on
// request, its byte histogram, for a device-resident buffer and its device
// cut list.  Replaces the per-chunk work of plakar's processChunk
// (snapshot/backup.go:594-629): chunkHasher.Write/Sum (backup.go:604-606,
// hashing "SHA256" = crypto/sha256, hashing/hashing.go:31-36) and the
// frequency count of entropy() (backup.go:548-557).  The float64 entropy is
// left to the caller, whose math.Log2 and summation order define it.
//
// SHA-256 is a serial chain over a message's 64-byte blocks, so the unit of
// parallelism is the chunk: one chunk per lane (FIPS 180-4, multi-buffer
// style), and each chunk is worked on by two lanes of two waves, a producer
// (loads, padding, histogram, message schedule) and a consumer (the rounds),
// see k_chunk_digest below.
//
// Bound: the consumer's chain, ~905 VALU per 64-byte block (14 per round,
// which is what three-input adds, bitop3 and alignbit allow), at one wave per
// SIMD; a launch lasts as long as its longest chunk.
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

// Two or three waves per workgroup of 64 chunks, one lane per chunk in each:
//   wave 1, the producer: loads block b + 1's words while it works on block b,
//     builds the big-endian words (v_perm funnel shift + byte swap), pads the
//     final block(s) and expands the message schedule W[0..63] into an LDS
//     ring stage;
//   wave 2 (histograms requested): the same words, counted;
//   wave 0, the consumer: the 64 rounds of block b - 1 from the other stage.
// One s_barrier per block.  The consumer's chain is ~14 VALU per round
// instead of ~25 when one lane did everything; the producer's ~560 VALU and
// the counter's ~160 VALU + 64 LDS atomics fit under it on other SIMDs.
constexpr uint32_t kShaRing = 2;                                   // stages
constexpr uint32_t kRingBytes = kShaRing * 64u * 64u * 4u;         // 32 KiB: [stage][word quad][lane] uint4
// The histogram: u16 halves, lanes l and l + 32 share the dword of bin b at
// 4 * (32 b + (l & 31)) (every access of a wave stays in its own bank pair),
// 32 KiB; flushed to the u32 output every kFlushBlocks blocks so that a half
// never passes 64 x 1023 < 65536 counts.
constexpr uint32_t kHistPairBytes = 256u * 32u * 4u;
constexpr uint64_t kFlushBlocks = 1023;

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), o)));
    return v;
}

template <bool HIST>
__global__ __launch_bounds__(192) void k_chunk_digest(const DigestBatch DB)
{
    extern __shared__ uint4 s_mem[];
    uint4 *ring = s_mem;                                                   // [kShaRing][16][64]
    uint32_t *s_hist = reinterpret_cast<uint32_t *>(s_mem + kShaRing * 16 * 64);  // [256][32]
    const DigestBuf &B = DB.b[blockIdx.y];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0 rounds, 1 schedule, 2 histogram
    uint64_t n_cuts = B.cap;
    if (B.res) n_cuts = min<uint64_t>(B.cap, uint64_t(B.res->ncuts));
    if (uint64_t(blockIdx.x) * 64u >= n_cuts) return;  // whole workgroup: no barrier is left waiting
    const uint64_t i = uint64_t(blockIdx.x) * 64u + lane;
    const bool valid = i < n_cuts;
    uint64_t n = 0, off = 0;
    if (valid) {
        const cdc_cut cut = B.cuts[i];
        off = cut.offset;
        n = cut.length;
        if (off > B.len) n = 0;
        else if (n > B.len - off) n = B.len - off;  // clipped to the buffer (a malformed list must not fault)
    }
    // blocks of the padded message: the full ones, then 1 or 2
    const uint64_t nb = valid ? n / 64u + ((n % 64u) <= 55u ? 1u : 2u) : 0u;
    const uint64_t NB = wave_max(uint32_t(min<uint64_t>(nb, 0xFFFFFFFFull)));  // both waves: same lanes, same bound

    if (role != 0) {
        const bool counting = HIST && role == 2;  // uniform per wave
        const uint8_t *p = B.data + (valid ? off : 0);
        const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
        const uint32_t sel = (sh << 24) | ((sh + 1u) << 16) | ((sh + 2u) << 8) | (sh + 3u);
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p - sh);
        const uint64_t lastq = n ? (sh + n - 1u) >> 2 : 0;  // last dword holding a byte of the chunk
        const uint32_t hoff = (lane & 31u) * 4u, hinc = 1u << (16u * (lane >> 5));
        if (counting) {
#pragma unroll 8
            for (uint32_t b = 0; b < 256; b += 2) s_hist[b * 32u + lane] = 0;  // 64 lanes, two bins a step
        }
        auto count1 = [&](uint32_t byte) {
            __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(s_hist) + ((byte << 7) | hoff)),
                                   hinc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        bool flushed = false;
        auto flush = [&]() {
            if (valid && B.hist) {
                uint4 *ho = reinterpret_cast<uint4 *>(B.hist + i * 256u);
                const uint32_t hs = 16u * (lane >> 5);
#pragma unroll 4
                for (uint32_t b = 0; b < 256; b += 4) {
                    uint4 v = make_uint4((s_hist[b * 32u + (lane & 31u)] >> hs) & 0xFFFFu,
                                         (s_hist[(b + 1) * 32u + (lane & 31u)] >> hs) & 0xFFFFu,
                                         (s_hist[(b + 2) * 32u + (lane & 31u)] >> hs) & 0xFFFFu,
                                         (s_hist[(b + 3) * 32u + (lane & 31u)] >> hs) & 0xFFFFu);
                    if (flushed) {
                        const uint4 o = ho[b / 4];
                        v = make_uint4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w);
                    }
                    ho[b / 4] = v;
                }
            }
#pragma unroll 8
            for (uint32_t b = 0; b < 256; b += 2) s_hist[b * 32u + lane] = 0;
            flushed = true;
        };
        // block b uses dwords q[16 b .. 16 b + 16]; the loads are clamped to
        // lastq near the end (bytes from past it are masked off below)
        auto load16 = [&](uint64_t b, uint32_t (&x)[16]) {
            const uint64_t base = 16u * b + 1u;
            if (base + 15u <= lastq) {
                const uint32_t *qb = q + base;
#pragma unroll
                for (int k = 0; k < 16; ++k) x[k] = qb[k];
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k) x[k] = q[min<uint64_t>(base + k, lastq)];
            }
        };
        uint32_t lo = 0, nx[16];
        if (n) {
            lo = q[0];
            load16(0, nx);
        }
        for (uint64_t it = 0; it < NB; ++it) {
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                w[k] = __builtin_amdgcn_perm(nx[k], lo, sel);
                lo = nx[k];
            }
            if (n && it + 1 < nb) load16(it + 1, nx);  // next block's words, in flight during this one
            const int64_t rb64 = int64_t(n) - int64_t(64u * it);  // bytes of the chunk from this block on
            const int32_t rb = int32_t(max<int64_t>(-128, min<int64_t>(128, rb64)));
            if (counting && rb >= 64) {
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    count1(w[k] >> 24);
                    count1(__builtin_amdgcn_ubfe(w[k], 16, 8));
                    count1(__builtin_amdgcn_ubfe(w[k], 8, 8));
                    count1(w[k] & 0xFFu);
                }
            }
            if (rb < 64 && rb > -64) {  // the lane's final block or two: data bytes, 0x80, zeros, bit length
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int32_t rem = rb - 4 * k;
                    const uint32_t keep = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ~(0xFFFFFFFFu >> (8 * rem));
                    const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80000000u >> (8 * rem)) : 0u;
                    w[k] = (w[k] & keep) | pad;
                    if (counting) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (j < rem) count1((w[k] >> (24 - 8 * j)) & 0xFFu);
                    }
                }
                if (rb <= 55) {
                    const uint64_t bits = n * 8u;
                    w[14] = uint32_t(bits >> 32);
                    w[15] = uint32_t(bits);
                }
            }
            if (!counting) {
                uint4 *st = ring + (it & 1u) * 1024u + lane;
#pragma unroll
                for (int k = 0; k < 16; k += 4) st[k * 16] = make_uint4(w[k], w[k + 1], w[k + 2], w[k + 3]);
                uint32_t x4[4];
#pragma unroll
                for (int t = 16; t < 64; ++t) {
                    const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
                    const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                    const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                    const uint32_t wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
                    w[t & 15] = wt;
                    x4[t & 3] = wt;
                    if ((t & 3) == 3) st[(t / 4) * 64] = make_uint4(x4[0], x4[1], x4[2], x4[3]);
                }
            }
            if (counting && (it + 1) % kFlushBlocks == 0) flush();
            __syncthreads();
        }
        __syncthreads();  // the consumer's last block
        if (counting) flush();
    } else {
        uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                         0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
        __builtin_amdgcn_s_setprio(3);  // the critical chain wins issue when waves share a SIMD
        __syncthreads();  // stage 0 filled
        for (uint64_t it = 0; it < NB; ++it) {
            const uint4 *st = ring + (it & 1u) * 1024u + lane;
            uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
            for (int q4 = 0; q4 < 16; ++q4) {
                const uint4 v = st[q4 * 64];
                const uint32_t wq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = 4 * q4 + j;
                    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
                    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
                    const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wq[j];
                    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
                    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
                    hh = g;
                    g = f;
                    f = e;
                    e = d + t1;
                    d = c;
                    c = b;
                    b = a;
                    a = t1 + S0 + mj;
                }
            }
            if (it < nb) {
                h[0] += a;
                h[1] += b;
                h[2] += c;
                h[3] += d;
                h[4] += e;
                h[5] += f;
                h[6] += g;
                h[7] += hh;
            }
            __syncthreads();
        }
        if (valid) {
            uint4 *out = reinterpret_cast<uint4 *>(B.digests + i * 32u);
            auto bswap = [](uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); };
            out[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
            out[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
        }
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
    const dim3 grid(uint32_t((cap + 63) / 64), DB.nbufs), block(hist ? 192 : 128);
    if (hist)
        hipLaunchKernelGGL(k_chunk_digest<true>, grid, block, kRingBytes + kHistPairBytes, st, DB);
    else
        hipLaunchKernelGGL(k_chunk_digest<false>, grid, block, kRingBytes, st, DB);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

}  // namespace cdc
