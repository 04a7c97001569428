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

#include <algorithm>
#include <cstring>
#include <mutex>

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

// SHA-256: two waves per group of 64 lanes; a lane hashes a run of
// consecutive chunks of the cut list, one after the other (one chunk per lane
// unless the launch holds more chunks than the device keeps lanes resident),
// taking its next chunk from its workgroup's queue, so every resident lane
// stays busy until the launch drains instead of idling once its one chunk is
// done.  Per lane:
//   the producer: loads block b + 2's words while it works on block b
//     (across chunk boundaries: the next chunk's first blocks), builds the
//     big-endian words (v_perm funnel shift + byte swap), pads each chunk's
//     final block(s) and expands the message schedule W[0..63] into an LDS
//     ring stage;
//   the consumer: the 64 rounds of block b - 1 from the other stage, the
//     digest written when a chunk's last block is done.
// One s_barrier per block.  The consumer's chain is ~14 VALU per round
// instead of ~25 when one lane did everything; the producer's ~560 VALU fit
// under it on another SIMD.
constexpr uint32_t kShaRing = 2;                                   // stages
constexpr uint32_t kRingBytes = kShaRing * 64u * 64u * 4u;         // 32 KiB: [stage][word quad][lane] uint4

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), o)));
    return v;
}

__device__ __forceinline__ uint64_t chunk_count(const DigestBuf &B)
{
    return B.res ? min<uint64_t>(B.cap, uint64_t(B.res->ncuts)) : B.cap;
}

// Cut c, clipped to the buffer (a malformed list must not fault).
__device__ __forceinline__ void cut_at(const DigestBuf &B, uint64_t c, uint64_t &off, uint64_t &n)
{
    const cdc_cut cut = B.cuts[c];
    off = cut.offset;
    n = cut.length;
    if (off > B.len) n = 0;
    else if (n > B.len - off) n = B.len - off;
}

// blocks of the padded message: the full ones, then 1 or 2
__device__ __forceinline__ uint64_t sha_blocks(uint64_t n) { return n / 64u + ((n % 64u) <= 55u ? 1u : 2u); }

// A chunk's bytes as aligned dwords: q[0] holds its first byte at byte sh,
// block b uses q[16 b .. 16 b + 16] (funnel-shifted by sel), q[lastq] holds
// its last byte.
struct ChunkWords {
    const uint32_t *q;
    uint32_t sel;
    uint64_t lastq;
};

__device__ __forceinline__ ChunkWords chunk_words(const uint8_t *data, uint64_t off, uint64_t n)
{
    const uint8_t *p = data + off;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(p) & 3u);
    return ChunkWords{reinterpret_cast<const uint32_t *>(p - sh),
                      (sh << 24) | ((sh + 1u) << 16) | ((sh + 2u) << 8) | (sh + 3u), n ? (sh + n - 1u) >> 2 : 0};
}

// block b's 16 dwords after q[16 b]; clamped to lastq near the end (bytes from
// past it are masked off by the padding)
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-B loads

__device__ __forceinline__ void load16(const ChunkWords &A, uint64_t b, uint32_t (&x)[16])
{
    const uint64_t base = 16u * b + 1u;
    if (base + 15u <= A.lastq) {  // four dwordx4 loads (a lane's own chunk: 4x fewer per-lane line lookups)
        const u32x4_a4 *qb = reinterpret_cast<const u32x4_a4 *>(A.q + base);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4_a4 v = qb[k];
            x[4 * k] = v.x;
            x[4 * k + 1] = v.y;
            x[4 * k + 2] = v.z;
            x[4 * k + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = A.q[min<uint64_t>(base + k, A.lastq)];
    }
}

// Two lane groups of 64 per workgroup (two workgroups per CU by LDS), waves
// by role so that a SIMD runs one round wave: a workgroup's waves land on
// SIMDs in the cyclic order 0 -> 2 -> 1 -> 3 (MI355X_MICROARCH.md, LDS;
// tools/wave_place.hip), so waves 0-1 (the producers) and 2-3 (the rounds)
// sit on four SIMDs.
constexpr uint32_t kDigestGroups = 2;  // one group per workgroup (four per CU): no faster at any size
constexpr uint32_t kDigestWaves = 2 * kDigestGroups;

// Per-lane block metadata beside each ring stage (written by the producer,
// read by the rounds one block behind): the chunk (relative to the
// workgroup's first) and flags.
constexpr uint32_t kMetaLive = 1u << 9, kMetaLast = 1u << 10;  // bits 0-8: rb + 128
constexpr uint32_t kSortCap = 1024;  // chunks a workgroup sorts longest first (8 KiB of LDS)

// The workgroup's buffer: from the kernel arguments (<= 32 buffers), or from
// device memory (launch_digests_many).
template <bool kInd>
__device__ __forceinline__ const DigestBuf &digest_buf(const DigestBatch &DB)
{
    return kInd ? DB.ind[blockIdx.y] : DB.b[blockIdx.y];
}

// Chunks of every buffer of the launch (the same value in every workgroup).
// Descriptors in device memory: the workgroup's threads sum them in parallel.
template <bool kInd>
__device__ __forceinline__ uint64_t launch_chunks(const DigestBatch &DB)
{
    uint64_t total = 0;
    if constexpr (!kInd) {
        for (uint32_t j = 0; j < DB.nbufs; ++j) total += chunk_count(DB.b[j]);
    } else {
        __shared__ uint64_t s_part[kDigestWaves];  // this instantiation only
        for (uint32_t j = threadIdx.x; j < DB.nbufs; j += blockDim.x) total += chunk_count(DB.ind[j]);
#pragma unroll
        for (int o = 32; o; o >>= 1) total += __shfl_xor(total, o);
        if ((threadIdx.x & 63u) == 0) s_part[threadIdx.x >> 6] = total;
        __syncthreads();
        total = 0;
        for (uint32_t w = 0; w < blockDim.x / 64u; ++w) total += s_part[w];
    }
    return total;
}

template <bool kInd>
__global__ __launch_bounds__(kDigestWaves * 64) void k_chunk_digest(const DigestBatch DB)
{
    constexpr uint32_t kLanes = 64u * kDigestGroups;
    __shared__ uint4 s_ring[kDigestGroups][kRingBytes / 16u];
    __shared__ uint32_t s_meta[kDigestGroups][kShaRing][2][64];
    __shared__ uint32_t s_any[kShaRing][kDigestGroups];  // some lane of the group holds a block in that stage
    __shared__ uint32_t s_next;                          // the workgroup's chunk queue (relative)
    __shared__ uint64_t s_order[kSortCap];               // its chunks longest first: (length << 32) | index
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t grp = wave % kDigestGroups;
    const uint32_t role = wave / kDigestGroups;  // 0 producer, 1 rounds
    uint4 *ring = s_ring[grp];                   // [kShaRing][16][64]
    const DigestBuf &B = digest_buf<kInd>(DB);
    const uint32_t lane = threadIdx.x & 63u;
    // Chunks per workgroup: kLanes while the launch fits the resident lanes,
    // else kLanes * k, k = ceil(chunks / resident lanes) (every wave of every
    // workgroup derives the same k).  The workgroup's lanes take its chunks
    // in order from an LDS queue, a lane its next one block before its
    // current one's last.
    const uint64_t total = launch_chunks<kInd>(DB);
    const uint64_t R = DB.resident_lanes ? DB.resident_lanes : 1u;
    const uint64_t k = total > R ? (total + R - 1) / R : 1u;
    const uint64_t n_cuts = chunk_count(B);
    const uint64_t C0 = uint64_t(blockIdx.x) * kLanes * k;
    if (C0 >= n_cuts) return;  // whole workgroup: no barrier is left waiting
    const uint64_t C1 = min(C0 + kLanes * k, n_cuts);
    if (threadIdx.x == 0) s_next = kLanes;
    // With more chunks than lanes, the queue hands them out longest first
    // (LPT: the short ones fill the lanes' ends), sorted in LDS by a bitonic
    // network when they fit kSortCap.
    const uint32_t nq = uint32_t(C1 - C0);
    const bool sorted = nq > kLanes && nq <= kSortCap;
    if (sorted) {
        uint32_t m = kLanes;
        while (m < nq) m <<= 1;
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
            uint64_t o = 0, len = 0;
            if (i < nq) cut_at(B, C0 + i, o, len);
            s_order[i] = i < nq ? (len << 32) | i : 0ull;  // padding sorts last
        }
        __syncthreads();
        for (uint32_t size = 2; size <= m; size <<= 1) {
            for (uint32_t stride = size >> 1; stride; stride >>= 1) {
                for (uint32_t t = threadIdx.x; t < m / 2; t += blockDim.x) {
                    const uint32_t i = 2 * stride * (t / stride) + t % stride, j = i + stride;
                    const bool desc = (i & size) == 0;  // descending runs, merged into one descending order
                    const uint64_t a = s_order[i], b = s_order[j];
                    if ((a < b) == desc) {
                        s_order[i] = b;
                        s_order[j] = a;
                    }
                }
                __syncthreads();
            }
        }
    }
    __syncthreads();
    // the workgroup's q-th chunk in queue order
    auto queued = [&](uint32_t q) -> uint64_t { return C0 + (sorted ? uint32_t(s_order[q]) : q); };

    if (role == 0) {
        // Blocks are loaded two ahead of the one being scheduled (a lane's
        // loads are uncoalesced and one block of cover left the producer
        // waiting on memory).  Every slot issues the same 17 dword loads on
        // every path (clamped to the chunk's last dword; a lane without a
        // block reads the cut list), so the compiler's vmcnt waits only for
        // the slot it consumes.
        const uint32_t *dummy = reinterpret_cast<const uint32_t *>(B.cuts);
        const uint32_t q0 = 64u * grp + lane;
        uint64_t lc = q0 < nq ? queued(q0) : C1, loff = 0, ln = 0, lnb = 0, lb = 0;  // load cursor
        // load-cursor flags in ONE variable: two bools captured by reference got a
        // pointer select and went to scratch, with a vmcnt(0) on every block
        constexpr uint32_t kHas = 1u, kResv = 2u;  // the cursor has a chunk; its next one is requested
        uint32_t lst = lc < C1 ? kHas : 0u;
        if (lst & kHas) {
            cut_at(B, lc, loff, ln);
            lnb = sha_blocks(ln);
        }
        ChunkWords LA = chunk_words(B.data, loff, ln);
        // the load cursor's next chunk, taken from the queue (and its cut
        // loaded) one block before the current one's last: late enough that
        // a lane does not hold a chunk it will only start much later (the
        // launch's tail), early enough to hide the cut's load
        uint64_t cn = ~0ull, noff = 0, nn = 0;
        auto reserve = [&]() __attribute__((always_inline)) {
            const uint32_t q = __hip_atomic_fetch_add(&s_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            cn = q < nq ? queued(q) : ~0ull;
            if (cn != ~0ull) cut_at(B, cn, noff, nn);
            lst |= kResv;
        };
        struct Blk {
            uint32_t x[17];  // q[16 b .. 16 b + 16]
            uint32_t sel, crel, n, itc;  // crel = kNoChunk: the lane has no block
        };
        constexpr uint32_t kNoChunk = 0xFFFFFFFFu;
        auto issue = [&](Blk &k) __attribute__((always_inline)) {  // the load cursor's block into k, then advance the cursor
            const bool real = (lst & kHas) && ln != 0;
            const uint32_t *q = real ? LA.q : dummy;
            const uint64_t base = real ? 16u * lb : 0u, lim = real ? LA.lastq : 0u;
#pragma unroll
            for (int j = 0; j < 17; ++j) k.x[j] = q[min<uint64_t>(base + j, lim)];
            k.sel = LA.sel;
            k.crel = (lst & kHas) ? uint32_t(lc - C0) : kNoChunk;
            k.n = uint32_t(ln);
            k.itc = uint32_t(lb);
            if (lst & kHas) {
                ++lb;
                if (!(lst & kResv) && lb + 1u >= lnb) reserve();
                if (lb == lnb) {
                    if (cn != ~0ull) {
                        lc = cn;
                        loff = noff;
                        ln = nn;
                        lnb = sha_blocks(nn);
                        lb = 0;
                        LA = chunk_words(B.data, loff, ln);
                        lst = kHas;
                    } else {
                        lst = 0u;
                    }
                }
            }
        };
        // schedule block `it` from slot k; false once no lane of the workgroup has one
        auto step = [&](uint32_t it, const Blk &k) __attribute__((always_inline)) -> bool {
            const bool live = k.crel != kNoChunk;
            const bool last = live && k.itc + 1u == sha_blocks(k.n);  // the chunk's final block
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) w[q] = __builtin_amdgcn_perm(k.x[q + 1], k.x[q], k.sel);
            const int64_t rb64 = int64_t(k.n) - int64_t(64u * k.itc);  // bytes of the chunk from this block on
            const int32_t rb = live ? int32_t(max<int64_t>(-128, min<int64_t>(128, rb64))) : 128;
            if (rb < 64 && rb > -64) {  // the chunk's final block or two: data bytes, 0x80, zeros, bit length
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int32_t rem = rb - 4 * q;
                    const uint32_t keep = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ~(0xFFFFFFFFu >> (8 * rem));
                    const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80000000u >> (8 * rem)) : 0u;
                    w[q] = (w[q] & keep) | pad;
                }
                if (rb <= 55) {
                    const uint64_t bits = uint64_t(k.n) * 8u;
                    w[14] = uint32_t(bits >> 32);
                    w[15] = uint32_t(bits);
                }
            }
            const uint32_t stg = it & 1u;
            uint4 *st = ring + stg * 1024u + lane;
#pragma unroll
            for (int q = 0; q < 16; q += 4) st[q * 16] = make_uint4(w[q], w[q + 1], w[q + 2], w[q + 3]);
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
            s_meta[grp][stg][0][lane] = k.crel;
            s_meta[grp][stg][1][lane] = uint32_t(rb + 128) | (live ? kMetaLive : 0u) | (last ? kMetaLast : 0u);
            const bool any = __ballot(live) != 0;
            if (lane == 0) s_any[stg][grp] = any ? 1u : 0u;
            __syncthreads();
            return (s_any[stg][0] | s_any[stg][kDigestGroups - 1]) != 0;  // every wave stops after the same barrier
        };
        Blk b0, b1, b2;
        issue(b0);
        issue(b1);
        for (uint32_t it = 0;; it += 3) {  // unrolled by the slot rotation
            issue(b2);
            if (!step(it, b0)) break;
            issue(b0);
            if (!step(it + 1, b1)) break;
            issue(b1);
            if (!step(it + 2, b2)) break;
        }
    } else {  // role 1: the rounds
        constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
        uint32_t h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = kIV[j];
        __builtin_amdgcn_s_setprio(3);  // the critical chain wins issue when waves share a SIMD
        for (uint32_t it = 0;; ++it) {
            __syncthreads();  // stage it filled
            const uint32_t stg = it & 1u;
            // the stop flag, the block's metadata and its first words in one round trip
            const uint32_t any = s_any[stg][0] | s_any[stg][kDigestGroups - 1];
            const uint32_t m = s_meta[grp][stg][1][lane], crel = s_meta[grp][stg][0][lane];
            const uint4 *st = ring + stg * 1024u + lane;
            const uint4 v0 = st[0];
            if (!any) break;
            uint32_t a = h[0], b = h[1], cc = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
            for (int q4 = 0; q4 < 16; ++q4) {
                const uint4 v = q4 ? st[q4 * 64] : v0;
                const uint32_t wq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = 4 * q4 + j;
                    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
                    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
                    const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wq[j];
                    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
                    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, cc, 0xE8);
                    hh = g;
                    g = f;
                    f = e;
                    e = d + t1;
                    d = cc;
                    cc = b;
                    b = a;
                    a = t1 + S0 + mj;
                }
            }
            if (m & kMetaLive) {
                h[0] += a;
                h[1] += b;
                h[2] += cc;
                h[3] += d;
                h[4] += e;
                h[5] += f;
                h[6] += g;
                h[7] += hh;
                if (m & kMetaLast) {  // the chunk's digest, then the next chunk from the IV
                    uint4 *out = reinterpret_cast<uint4 *>(B.digests + (C0 + crel) * 32u);
                    auto bswap = [](uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); };
                    out[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
                    out[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
#pragma unroll
                    for (int j = 0; j < 8; ++j) h[j] = kIV[j];
                }
            }
        }
    }
}

// Byte histograms, one wave per chunk (a wave takes chunks w, w + waves, ...):
// the frequency count of entropy() (snapshot/backup.go:548-557).  Unlike the
// SHA-256 chain a histogram has no order, so the wave reads its chunk
// coalesced, 16 bytes per lane per step, and counts into 8 LDS copies of the
// 256 bins (copy = lane & 7, bin b of copy c at dword 8 b + c: lanes of one
// copy only collide on equal bytes); then the copies are summed, one uint4
// of bins per lane, into the chunk's row.
constexpr uint32_t kHistWaves = 4, kHistCopies = 8;

template <bool kInd>
__global__ __launch_bounds__(kHistWaves * 64) void k_chunk_hist(const DigestBatch DB)
{
    __shared__ uint32_t s_h[kHistWaves][256 * kHistCopies];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const DigestBuf &B = digest_buf<kInd>(DB);
    if (!B.hist) return;
    uint32_t *h = s_h[wave];
    const uint32_t cpy = lane & (kHistCopies - 1u);
    const uint64_t n_cuts = chunk_count(B);
    const uint64_t waves = uint64_t(gridDim.x) * kHistWaves;
    for (uint64_t c = uint64_t(blockIdx.x) * kHistWaves + wave; c < n_cuts; c += waves) {
#pragma unroll
        for (uint32_t i = 0; i < 256 * kHistCopies / 64; ++i) h[i * 64 + lane] = 0;
        uint64_t off, n;
        cut_at(B, c, off, n);
        const uint8_t *p = B.data + off;
        // 16-B aligned steps covering [p, p + n); bytes outside it are skipped
        const uint64_t a0 = reinterpret_cast<uintptr_t>(p) & ~15ull, end = reinterpret_cast<uintptr_t>(p) + n;
        auto count = [&](uint32_t byte) {
            __hip_atomic_fetch_add(h + byte * kHistCopies + cpy, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        // the next step's 16 bytes in flight while this step counts; every
        // lane loads every step (from a block holding chunk bytes: the last
        // one when past the end), so the compiler waits only for the current
        const uint64_t alast = (end - 1) & ~15ull;
        auto ld = [&](uint64_t a) {  // global (not flat) loads: LDS waits do not wait for them
            typedef __attribute__((address_space(1))) const uint64_t g64;
            const g64 *q = reinterpret_cast<const g64 *>(uintptr_t(a <= alast ? a : alast));
            const uint64_t x = q[0], y = q[1];
            return make_uint4(uint32_t(x), uint32_t(x >> 32), uint32_t(y), uint32_t(y >> 32));
        };
        uint4 vn = n ? ld(a0 + 16u * lane) : make_uint4(0, 0, 0, 0);
        for (uint64_t a = a0 + 16u * lane; n && a < end; a += 1024u) {
            const uint4 v = vn;
            vn = ld(a + 1024u);
            const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
            if (a >= reinterpret_cast<uintptr_t>(p) && a + 16u <= end) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    count(wd[q] & 0xFFu);
                    count(__builtin_amdgcn_ubfe(wd[q], 8, 8));
                    count(__builtin_amdgcn_ubfe(wd[q], 16, 8));
                    count(wd[q] >> 24);
                }
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const uint64_t x = a + uint64_t(q);
                    if (x >= reinterpret_cast<uintptr_t>(p) && x < end) count((wd[q >> 2] >> (8 * (q & 3))) & 0xFFu);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        uint32_t sum[4] = {0, 0, 0, 0};
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
#pragma unroll
            for (uint32_t k = 0; k < kHistCopies; ++k) sum[j] += h[(4 * lane + j) * kHistCopies + k];
        reinterpret_cast<uint4 *>(B.hist + c * 256u)[lane] = make_uint4(sum[0], sum[1], sum[2], sum[3]);
        __builtin_amdgcn_wave_barrier();
    }
}

// entropy() of snapshot/backup.go:548-569 from a byte histogram row: e = 0;
// for b in 0..255 with f_b > 0: p = f_b / len; e -= p * Log2(p), with Go's
// math.Log2 (math/log2.go: Frexp, frac == 0.5 -> exp - 1, else
// Log(frac) * (1/Ln2) + exp) and Go's Log (math/log.go, the fdlibm e_log.c
// reduction and polynomial).  Every step is one IEEE double operation in the
// reference's order: contraction into FMAs is off for this code, division is
// the correctly rounded lowering.  Restated from plakar_amd/hashing.py
// go_log2 / entropy_from_freq, whose parity tests pin it.
#pragma clang fp contract(off)
__device__ __forceinline__ double go_log2_dev(double x)
{
    // x = p in (0, 1]: a normal double (p >= 2^-64), so Frexp is the exponent field
    const uint64_t bits = uint64_t(__double_as_longlong(x));
    const int e2 = int((bits >> 52) & 0x7FFu) - 1022;
    double frac = __longlong_as_double(int64_t((bits & 0x800FFFFFFFFFFFFFull) | (1022ull << 52)));
    if (frac == 0.5) return double(e2 - 1);
    // Log(frac): frac = f1 * 2^0, f1 in [0.5, 1)
    double f1 = frac;
    int ki = 0;
    if (f1 < 0.70710678118654757) {  // math.Sqrt2 / 2 (rounded)
        f1 *= 2.0;
        ki = -1;
    }
    const double f = f1 - 1.0;
    const double k = double(ki);
    const double s = f / (2.0 + f);
    const double s2 = s * s;
    const double s4 = s2 * s2;
    const double t1 = s2 * (6.666666666666735130e-01 + s4 * (2.857142874366239149e-01 +
                                                           s4 * (1.818357216161805012e-01 + s4 * 1.479819860511658591e-01)));
    const double t2 = s4 * (3.999999999940941908e-01 + s4 * (2.222219843214978396e-01 + s4 * 1.531383769920937332e-01));
    const double r = t1 + t2;
    const double hfsq = 0.5 * f * f;
    const double lg = k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + r) + k * 1.90821492927058770002e-10)) - f);
    return lg * 1.4426950408889634 + double(e2);  // 0x1.71547652b82fep+0: Go's 1/Ln2
}

// One wave per histogram row: lane l holds bins 4l .. 4l + 3 (one coalesced
// KiB per row), computes their terms, and the wave folds them in bin order
// (the reference's sequential e -= term: a fixed order, so bit-exact).
constexpr uint32_t kEntWaves = 4;
__global__ __launch_bounds__(kEntWaves * 64) void k_chunk_entropy(const uint32_t *__restrict__ hist, uint64_t rows,
                                                                  double *__restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = uint64_t(gridDim.x) * kEntWaves;
    for (uint64_t r = uint64_t(blockIdx.x) * kEntWaves + (threadIdx.x >> 6); r < rows; r += waves) {
        const uint4 h = reinterpret_cast<const uint4 *>(hist + r * 256u)[lane];
        uint64_t len = uint64_t(h.x) + h.y + h.z + h.w;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) len += __shfl_xor(len, o, 64);
        const double dl = double(len);
        const uint32_t hv[4] = {h.x, h.y, h.z, h.w};
        double t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double p = double(hv[j]) / dl;
            t[j] = hv[j] ? p * go_log2_dev(p) : 0.0;
        }
        double e = 0.0;
        for (int l = 0; l < 64; ++l) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double tj = __shfl(t[j], l, 64);
                const uint32_t hj = __shfl(hv[j], l, 64);
                if (hj) e -= tj;
            }
        }
        if (lane == 0) out[r] = len ? e : 0.0;
    }
}
#pragma clang fp contract(on)

int launch_entropy(const uint32_t *d_hist, uint64_t rows, double *d_out, void *stream)
{
    if (!rows) return CDC_OK;
    const uint64_t wgs = std::min<uint64_t>((rows + kEntWaves - 1) / kEntWaves, 256u * 8u);
    hipLaunchKernelGGL(k_chunk_entropy, dim3(uint32_t(wgs)), dim3(kEntWaves * 64), 0,
                       reinterpret_cast<hipStream_t>(stream), d_hist, rows, d_out);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

// A batch of files laid out in one arena (the backup pipeline's slots) as ONE
// digest buffer: file j's cut list sits at slots [cut0_j, cut0_j + cap_j) of
// `cuts` with offsets relative to the file; out[slot] is the same cut with
// the file's arena offset added, or an empty chunk at 0 for the slots past
// the file's count.  One digest launch then covers every file of the batch
// (a launch lasts as long as its longest chunk, so one launch per batch, not
// one per 32 files).  meta: (cut0, cap, arena_off) per file.
__global__ __launch_bounds__(256) void k_arena_cuts(const uint64_t *__restrict__ meta,
                                                    const cdc_result *__restrict__ res,
                                                    const cdc_cut *__restrict__ cuts, cdc_cut *__restrict__ out)
{
    const uint32_t j = blockIdx.x;
    const uint64_t c0 = meta[3 * j], cap = meta[3 * j + 1], base = meta[3 * j + 2];
    const uint64_t n = min<uint64_t>(cap, res[j].ncuts);
    for (uint64_t q = threadIdx.x; q < cap; q += blockDim.x) {
        cdc_cut c = {0, 0, 0};
        if (q < n) {
            c = cuts[c0 + q];
            c.offset += base;
        }
        out[c0 + q] = c;
    }
}

int launch_arena_cuts(const uint64_t *d_meta, uint32_t nfiles, const cdc_result *d_res, const cdc_cut *d_cuts,
                      cdc_cut *d_out, void *stream)
{
    if (!nfiles) return CDC_OK;
    hipLaunchKernelGGL(k_arena_cuts, dim3(nfiles), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_meta, d_res,
                       d_cuts, d_out);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

uint64_t g_digest_lanes = 0;  // cdc_debug_set_digest_lanes (0: from the device's CU count)
thread_local int t_scan_tpw = -1;
thread_local int t_force_abort = 0;

namespace {

uint32_t device_cus()
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
        n = 256;
    return uint32_t(n);
}

template <bool kInd>
int launch_digest_kernels(DigestBatch D, uint64_t cap, bool hist, hipStream_t st, int parts = 3)
{
    static const uint32_t cus = device_cus();
    // two SHA-256 workgroups per CU (~66 KiB of LDS each)
    D.resident_lanes = g_digest_lanes ? g_digest_lanes : uint64_t(cus) * 2u * 64u * kDigestGroups;
    const uint32_t lanes_per_wg = 64u * kDigestGroups;
    if (parts & 1)
        hipLaunchKernelGGL(k_chunk_digest<kInd>, dim3(uint32_t((cap + lanes_per_wg - 1) / lanes_per_wg), D.nbufs),
                           dim3(kDigestWaves * 64), 0, st, D);
    if (hist && (parts & 2)) {  // a wave per chunk; up to 8 workgroups per CU
        const uint64_t wgs = std::min<uint64_t>((cap + kHistWaves - 1) / kHistWaves, uint64_t(cus) * 8u);
        hipLaunchKernelGGL(k_chunk_hist<kInd>, dim3(uint32_t(wgs), D.nbufs), dim3(kHistWaves * 64), 0, st, D);
    }
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

// Per-device ring of descriptor slots: pinned staging + device copy; a slot is
// reused once the launch group that read it has finished (its event).
constexpr uint32_t kDescRing = 16, kDescMax = 8192;
struct DescRing {
    std::mutex mu;
    DigestBuf *h = nullptr, *d = nullptr;
    hipEvent_t ev[kDescRing] = {};
    bool used[kDescRing] = {};
    uint32_t next = 0;
    bool failed = false;
};

DescRing &desc_ring(int device)
{
    static DescRing rings[64];
    return rings[device & 63];
}

}  // namespace

int launch_digests(const DigestBatch &DB, void *stream, int parts)
{
    uint64_t cap = 0;
    bool hist = false;
    for (uint32_t i = 0; i < DB.nbufs; ++i) {
        cap = DB.b[i].cap > cap ? DB.b[i].cap : cap;
        hist |= DB.b[i].hist != nullptr;
    }
    if (cap == 0 || DB.nbufs == 0) return CDC_OK;
    if (cap > 0xFFFFFFFFull) return CDC_E_INVALID;  // chunk indices relative to a workgroup's first are u32
    DigestBatch D = DB;
    D.ind = nullptr;
    return launch_digest_kernels<false>(D, cap, hist, reinterpret_cast<hipStream_t>(stream), parts);
}

// ---------------------------------------------------------------------------
// Hybrid digests (cdc_chunk_digests_hybrid): the longest chunks' SHA-256 on
// host cores.  A chain costs the device ~2 us per 64-B block (one round wave,
// above) against ~35 ns on a host core with the SHA extensions, so a launch
// that lasts as long as its longest chunk ends sooner when the longest go to
// the host.  k_gather packs those chunks' bytes into a staging buffer (one
// workgroup per chunk, aligned dwords funnel-shifted, reads clamped to the
// chunk's last dword) for one copy to the host; k_scatter_digests writes the
// host's digests back into the caller's digest rows.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gather(const GatherJob *jobs, uint8_t *stage)
{
    const GatherJob J = jobs[blockIdx.x];
    if (J.len == 0) return;
    const uint64_t s = reinterpret_cast<uint64_t>(J.src);
    const uint32_t sh = uint32_t(s & 3u);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(s & ~3ull);
    const uint64_t nd = (J.len + 3) / 4;
    const uint64_t last = (s + J.len - 1 - (s & ~3ull)) / 4;  // the last dword holding a chunk byte
    uint32_t *d = reinterpret_cast<uint32_t *>(stage + J.dst);
    for (uint64_t i = threadIdx.x; i < nd; i += blockDim.x) {
        const uint32_t lo = a[min(i, last)], hi = a[min(i + 1, last)];
        d[i] = __builtin_amdgcn_alignbyte(hi, lo, sh);  // bytes sh .. sh + 3 of hi:lo
    }
}

__global__ __launch_bounds__(256) void k_scatter_digests(const ScatterJob *jobs, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 8u * n) return;
    const ScatterJob J = jobs[i / 8u];
    reinterpret_cast<uint32_t *>(J.dst)[i % 8u] = reinterpret_cast<const uint32_t *>(J.src)[i % 8u];
}

int launch_gather(const GatherJob *d_jobs, uint32_t n, uint8_t *d_stage, void *stream)
{
    if (n == 0) return CDC_OK;
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_jobs, d_stage);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

int launch_scatter_digests(const ScatterJob *d_jobs, uint32_t n, void *stream)
{
    if (n == 0) return CDC_OK;
    hipLaunchKernelGGL(k_scatter_digests, dim3((8u * n + 255u) / 256u), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_jobs, n);
    return hipGetLastError() == hipSuccess ? CDC_OK : CDC_E_DEVICE;
}

int launch_digests_many(const DigestBuf *bufs, uint32_t nbufs, void *stream)
{
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return CDC_E_DEVICE;
    DescRing &R = desc_ring(dev);
    for (uint32_t i0 = 0; i0 < nbufs; i0 += kDescMax) {
        const uint32_t n = std::min(kDescMax, nbufs - i0);
        uint64_t cap = 0;
        bool hist = false;
        for (uint32_t i = 0; i < n; ++i) {
            cap = std::max(cap, bufs[i0 + i].cap);
            hist |= bufs[i0 + i].hist != nullptr;
        }
        if (cap == 0) continue;
        if (cap > 0xFFFFFFFFull) return CDC_E_INVALID;
        std::lock_guard<std::mutex> lk(R.mu);
        if (!R.h) {
            if (R.failed) return CDC_E_DEVICE;
            const size_t bytes = size_t(kDescRing) * kDescMax * sizeof(DigestBuf);
            bool ok = hipHostMalloc(reinterpret_cast<void **>(&R.h), bytes, hipHostMallocDefault) == hipSuccess &&
                      hipMalloc(reinterpret_cast<void **>(&R.d), bytes) == hipSuccess;
            for (auto &e : R.ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            if (!ok) {
                R.failed = true;  // leave it unusable rather than half made
                return CDC_E_DEVICE;
            }
        }
        const uint32_t slot = R.next++ % kDescRing;
        if (R.used[slot] && hipEventSynchronize(R.ev[slot]) != hipSuccess) return CDC_E_DEVICE;
        DigestBuf *h = R.h + size_t(slot) * kDescMax, *d = R.d + size_t(slot) * kDescMax;
        std::memcpy(h, bufs + i0, n * sizeof(DigestBuf));
        if (hipMemcpyAsync(d, h, n * sizeof(DigestBuf), hipMemcpyHostToDevice, st) != hipSuccess) return CDC_E_DEVICE;
        DigestBatch D;
        std::memset(&D, 0, sizeof(D));
        D.nbufs = n;
        D.ind = d;
        int s2 = launch_digest_kernels<true>(D, cap, hist, st);
        if (s2 != CDC_OK) return s2;
        if (hipEventRecord(R.ev[slot], st) != hipSuccess) return CDC_E_DEVICE;
        R.used[slot] = true;
    }
    return CDC_OK;
}

}  // namespace cdc
