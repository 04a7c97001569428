// Encode on the device: plakar's (*Repository).Encode
// (repository/repository.go:212-236) of a batch of blobs: the LZ4 frame of
// compression.DeflateLZ4Stream (compression/compression.go:94-106,
// github.com/pierrec/lz4/v4 v4.1.18 NewWriter defaults: independent blocks of
// at most 4 MiB, content checksum on), then the AES-256-GCM stream of
// encryption.EncryptStream (encryption/symmetric.go:72-163): a random subkey
// sealed under the repository key, then every 64-KiB piece of the
// compressed stream sealed under the subkey with its own nonce.
//
// Kernels, in launch order (one batch = the blobs of one call):
//   k_xxh32       XXH32 of every blob (the frame's content checksum), on a
//                 side stream: four blobs per wave, a lane quad's chains each
//   k_lz4_seq     one wave per 16-KiB segment: greedy LZ4 match search, 64
//                 positions per step at LZ4's accelerating stride (hash table
//                 of 4,096 u16 in LDS, matches found by ballot, extended 64
//                 bytes per step both ways); sequences out as (match start,
//                 offset, length) records
//   k_lz4_size    one workgroup per 4-MiB LZ4 block: literal runs across
//                 segment boundaries, encoded size (raw when not smaller)
//   k_enc_plan    one workgroup: frame sizes, block offsets in the frame,
//                 GCM pieces and output offsets of every blob (scans)
//   k_lz4_emit    a workgroup per block (16 per stored block): its bytes
//   k_frame_fin   one wave per blob: frame header, end mark, checksum
//   k_blob_keys   one thread per blob: the subkey's round keys, H and its
//                 4-bit table, and the sealed subkey (header)
//   k_blob_pows   one wave per blob: H^1..H^64 (a doubling ladder over the
//                 lanes) and the 8-bit table of H^64
//   k_gcm         one wave per 64-KiB piece: AES-256-CTR (two rotated
//                 T-tables in LDS, 32 bank-conflict-free copies each; rounds
//                 1-2 partly once per piece) and GHASH (lane l hashes blocks
//                 l, l+64, ... by Horner in H^64 with an 8-bit table, reduced
//                 once per block, then multiplies by its own H^e), tag
//
// Matches stay inside their 16-KiB segment, so compression ratios are those
// of LZ4 with a 16-KiB window; any LZ4 decoder reads the frames (the tests
// decode them with the system's liblz4).  Nonces and subkeys come from the
// caller (the host fills them from the OS CSPRNG), as crypto/rand does in
// the reference; piece k of a blob uses the blob's data nonce with its last
// four bytes XOR k (big-endian), unique per subkey.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "cdc_internal.h"

namespace enc {

constexpr uint32_t kSegLZ = 8192;             // LZ4 match-search segment
constexpr uint64_t kBlockLZ = 4ull << 20;     // LZ4 block (pierrec Block4Mb)
constexpr uint32_t kPiece = 65536;            // EncryptStream chunkSize
constexpr uint32_t kHashBits = 11;
constexpr uint32_t kRecCap = kSegLZ / 4 + 2;  // records per segment (a match per 4 bytes at most)

// ---------------------------------------------------------------------------
// AES tables, built on the host (FIPS-197: S-box = affine(inverse in GF(2^8))).
// ---------------------------------------------------------------------------
__device__ uint32_t g_te0[256];
__device__ uint8_t g_sbox[256];

static void build_tables(uint32_t te0[256], uint8_t sbox[256])
{
    auto mul = [](uint8_t a, uint8_t b) {
        uint8_t p = 0;
        for (int i = 0; i < 8; ++i) {
            if (b & 1) p ^= a;
            const uint8_t hi = a & 0x80;
            a = uint8_t(a << 1);
            if (hi) a ^= 0x1B;
            b >>= 1;
        }
        return p;
    };
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x)
            for (int y = 1; y < 256; ++y)
                if (mul(uint8_t(x), uint8_t(y)) == 1) {
                    inv = uint8_t(y);
                    break;
                }
        uint8_t s = inv;
        for (int i = 1; i <= 4; ++i) s ^= uint8_t((inv << i) | (inv >> (8 - i)));
        sbox[x] = uint8_t(s ^ 0x63);
    }
    for (int x = 0; x < 256; ++x) {
        const uint8_t s = sbox[x];
        te0[x] = uint32_t(mul(s, 2)) << 24 | uint32_t(s) << 16 | uint32_t(s) << 8 | mul(s, 3);
    }
}

__device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// AES-256 key schedule (FIPS-197 §5.2), words big-endian.
__device__ void aes256_expand(const uint8_t key[32], uint32_t rk[60], const uint8_t *sbox)
{
    for (int i = 0; i < 8; ++i)
        rk[i] = uint32_t(key[4 * i]) << 24 | uint32_t(key[4 * i + 1]) << 16 | uint32_t(key[4 * i + 2]) << 8 |
                key[4 * i + 3];
    uint32_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 8 == 0) {
            t = rol32(t, 8);
            t = uint32_t(sbox[t >> 24]) << 24 | uint32_t(sbox[(t >> 16) & 255]) << 16 |
                uint32_t(sbox[(t >> 8) & 255]) << 8 | sbox[t & 255];
            t ^= rcon << 24;
            rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0);
        } else if (i % 8 == 4) {
            t = uint32_t(sbox[t >> 24]) << 24 | uint32_t(sbox[(t >> 16) & 255]) << 16 |
                uint32_t(sbox[(t >> 8) & 255]) << 8 | sbox[t & 255];
        }
        rk[i] = rk[i - 8] ^ t;
    }
}

// One block, words big-endian (T-table form; Te1..3 are rotations of Te0).
__device__ __forceinline__ void aes256_block(const uint32_t *rk, const uint32_t *te, const uint8_t *sb, uint32_t s[4])
{
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t t0 = te[s0 >> 24] ^ ror32(te[(s1 >> 16) & 255], 8) ^ ror32(te[(s2 >> 8) & 255], 16) ^
                            ror32(te[s3 & 255], 24) ^ rk[4 * r];
        const uint32_t t1 = te[s1 >> 24] ^ ror32(te[(s2 >> 16) & 255], 8) ^ ror32(te[(s3 >> 8) & 255], 16) ^
                            ror32(te[s0 & 255], 24) ^ rk[4 * r + 1];
        const uint32_t t2 = te[s2 >> 24] ^ ror32(te[(s3 >> 16) & 255], 8) ^ ror32(te[(s0 >> 8) & 255], 16) ^
                            ror32(te[s1 & 255], 24) ^ rk[4 * r + 2];
        const uint32_t t3 = te[s3 >> 24] ^ ror32(te[(s0 >> 16) & 255], 8) ^ ror32(te[(s1 >> 8) & 255], 16) ^
                            ror32(te[s2 & 255], 24) ^ rk[4 * r + 3];
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    s[0] = (uint32_t(sb[s0 >> 24]) << 24 | uint32_t(sb[(s1 >> 16) & 255]) << 16 | uint32_t(sb[(s2 >> 8) & 255]) << 8 |
            sb[s3 & 255]) ^ rk[56];
    s[1] = (uint32_t(sb[s1 >> 24]) << 24 | uint32_t(sb[(s2 >> 16) & 255]) << 16 | uint32_t(sb[(s3 >> 8) & 255]) << 8 |
            sb[s0 & 255]) ^ rk[57];
    s[2] = (uint32_t(sb[s2 >> 24]) << 24 | uint32_t(sb[(s3 >> 16) & 255]) << 16 | uint32_t(sb[(s0 >> 8) & 255]) << 8 |
            sb[s1 & 255]) ^ rk[58];
    s[3] = (uint32_t(sb[s3 >> 24]) << 24 | uint32_t(sb[(s0 >> 16) & 255]) << 16 | uint32_t(sb[(s1 >> 8) & 255]) << 8 |
            sb[s2 & 255]) ^ rk[59];
}

// ---------------------------------------------------------------------------
// GF(2^128) in GCM's bit order (SP 800-38D §6.3): an element is (hi, lo) =
// the big-endian halves of its 16 bytes.  4-bit tables: T[i] = i * V for the
// 4-bit value i read MSB-first (T[8] = V, T[4] = V x, ...).
// ---------------------------------------------------------------------------
struct G128 {
    uint64_t hi, lo;
};

__device__ __forceinline__ G128 gx(G128 a, G128 b) { return {a.hi ^ b.hi, a.lo ^ b.lo}; }

__device__ void gtable(G128 v, G128 t[16])
{
    auto half = [](G128 x) {  // x * x^1 (one right shift with reduction)
        const uint64_t r = (x.lo & 1) ? 0xE100000000000000ull : 0;
        return G128{(x.hi >> 1) ^ r, (x.lo >> 1) | (x.hi << 63)};
    };
    t[0] = {0, 0};
    t[8] = v;
    t[4] = half(t[8]);
    t[2] = half(t[4]);
    t[1] = half(t[2]);
    for (int i = 3; i < 16; ++i)
        if (i & (i - 1)) t[i] = gx(t[i & -i], t[i & (i - 1)]);
}

// rem_4bit[r]: the reduction of the 4 bits shifted out, in the top 16 bits.
__device__ __forceinline__ uint64_t rem4(uint32_t r)
{
    uint64_t x = 0;
    if (r & 1) x ^= 0x1C20;
    if (r & 2) x ^= 0x3840;
    if (r & 4) x ^= 0x7080;
    if (r & 8) x ^= 0xE100;
    return x << 48;
}

// x * V with V's 4-bit table (processed nibble by nibble from the last byte).
template <typename TAB>
__device__ __forceinline__ G128 gmul4(G128 x, const TAB &t)
{
    G128 z = {0, 0};
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        const uint64_t w = i >= 16 ? x.lo : x.hi;
        const uint32_t nib = uint32_t(w >> (4 * ((31 - i) & 15))) & 15;
        if (i != 31) {
            const uint32_t rem = uint32_t(z.lo) & 15;
            z.lo = (z.hi << 60) | (z.lo >> 4);
            z.hi = (z.hi >> 4) ^ rem4(rem);
        }
        const G128 e = t[nib];
        z.hi ^= e.hi;
        z.lo ^= e.lo;
    }
    return z;
}

// a * b bit by bit (SP 800-38D Algorithm 1), for a per-lane multiplier.
__device__ G128 gmul_bits(G128 a, G128 b)
{
    // branch-free: the bit of a as a sign mask (v_ashrrev), z ^= v & mask and
    // the reduction's 0xE1 as one v_bitop3 each, v shifted by v_alignbit
    uint32_t z[4] = {0, 0, 0, 0};
    uint32_t v[4] = {uint32_t(b.hi >> 32), uint32_t(b.hi), uint32_t(b.lo >> 32), uint32_t(b.lo)};
    const uint32_t aw[4] = {uint32_t(a.hi >> 32), uint32_t(a.hi), uint32_t(a.lo >> 32), uint32_t(a.lo)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t w = aw[k];
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const uint32_t m = uint32_t(int32_t(w) >> 31);
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = __builtin_amdgcn_bitop3_b32(z[q], v[q], m, 0x78);  // z ^ (v & m)
            w <<= 1;
            const uint32_t r = uint32_t(int32_t(v[3] << 31) >> 31);  // v's last bit as a mask
            v[3] = __builtin_amdgcn_alignbit(v[2], v[3], 1);
            v[2] = __builtin_amdgcn_alignbit(v[1], v[2], 1);
            v[1] = __builtin_amdgcn_alignbit(v[0], v[1], 1);
            v[0] = __builtin_amdgcn_bitop3_b32(v[0] >> 1, r, 0xE1000000u, 0x78);  // (v0 >> 1) ^ (r & 0xE1..)
        }
    }
    return {uint64_t(z[0]) << 32 | z[1], uint64_t(z[2]) << 32 | z[3]};
}

__device__ __forceinline__ G128 g_from_words(const uint32_t w[4])
{
    return {uint64_t(w[0]) << 32 | w[1], uint64_t(w[2]) << 32 | w[3]};
}

// Per-blob GCM state (workspace): AES round keys of the subkey, the 4-bit
// tables of H and H^64, and H^1..H^64.
struct BlobKey {
    uint32_t rk[60];
    uint32_t pad[4];
    G128 th[16];      // 4-bit table of H (the length block)
    G128 hpow[64];    // H^1 .. H^64
    G128 t64[256];    // 8-bit table of H^64 (the lanes' Horner steps)
};

struct Seg {             // a 16-KiB LZ4 search segment
    uint64_t src;        // byte offset in the input base
    uint32_t len;
    uint32_t rem;        // bytes from the segment's start to its LZ4 block's end
};

struct Blk {             // a 4-MiB LZ4 block
    uint64_t src;
    uint32_t len, blob;
    uint32_t seg0, nseg;
    uint32_t k;          // block index in its blob
    uint32_t pad;
};

struct BlobDesc {
    uint64_t src;        // byte offset in the input base
    uint64_t len;
    uint64_t slot;       // frame slot in the frame buffer (16-B aligned)
    uint32_t blk0, nblk;
};

struct Batch {
    const uint8_t *base;
    uint32_t nblobs, nsegs, nblks, npieces_max;
    uint32_t compress, encrypt;
    const BlobDesc *blobs;
    const Seg *segs;
    const Blk *blks;
    const uint8_t *rnd;       // per blob: subkey 32, subkey nonce 12, data nonce 12
    const uint8_t *key;       // repository key (32 B, device)
    uint8_t *frames;          // frame buffer
    uint8_t *out;
    uint64_t out_cap;
    // workspace
    uint2 *recs;              // kRecCap per segment
    uint32_t *nrec;           // per segment
    uint32_t *trail;          // per segment: literals after its last match (from its start when none)
    uint32_t *seg_out;        // per segment: bytes of its sequences in the block (k_lz4_size)
    uint32_t *blk_size;       // per block: encoded size, bit 31 = stored raw
    uint64_t *blk_foff;       // per block: offset of its header in the frame
    uint32_t *xxh;            // per blob
    uint64_t *frame_len;      // per blob
    uint64_t *out_off;        // nblobs + 1
    uint32_t *piece_base;     // nblobs + 1
    BlobKey *keys;            // per blob
    uint64_t *status;         // [0]: CDC_E_NOSPACE when out_cap is too small
    const uint32_t *xx_ids;   // XXH32 order of the blobs
};

// Global-memory views (global_load, counted in vmcnt only; a generic pointer
// gives flat loads, which also count in lgkmcnt).
typedef __attribute__((address_space(1))) const uint32_t gu32;
typedef __attribute__((address_space(1))) const uint8_t gu8;

__device__ __forceinline__ uint32_t ld32u(const uint8_t *p)  // unaligned
{
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// ---------------------------------------------------------------------------
// XXH32 (the frame's content checksum): lanes 0-3 run accumulators v1..v4 over
// the 16-byte stripes, lane 0 the tail.
// ---------------------------------------------------------------------------
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;

// A wave hashes kXxPerWave blobs (sorted longest first on the host: the
// longest chains start first).  Their stripes stream through LDS, a region of
// kXxRegion / kXxPerWave bytes per blob at a time, regions r + 1 and r + 2 in
// flight while lane quad g runs blob g's four accumulator chains (lane a:
// accumulator a) over region r.  The loading lanes store each word already
// multiplied by PRIME32_2, so a chain step is add, rotate, multiply.  A batch
// takes as long as its longest blob's chain (a 4-MiB blob: 262,144 steps);
// more blobs per wave (less idle VALU work) measured slower, because the chain
// latency, not VALU throughput, bounds it.
constexpr uint32_t kXxWaves = 4;
constexpr uint32_t kXxRegion = 4096;                 // bytes per wave per stage
constexpr uint32_t kXxPerWave = 1;                   // blobs per wave
constexpr uint32_t kXxBlobRegion = kXxRegion / kXxPerWave;
constexpr uint32_t kXxLoadLanes = 64 / kXxPerWave;  // lanes loading one blob's region
static_assert(kXxBlobRegion == 16 * 4 * kXxLoadLanes, "16 words per loading lane");

// The merge of the four accumulators, the tail and the avalanche.
__device__ uint32_t xxh_finish(uint32_t v1, uint32_t v2, uint32_t v3, uint32_t v4, const uint8_t *p, uint64_t n)
{
    uint32_t h = n >= 16 ? rol32(v1, 1) + rol32(v2, 7) + rol32(v3, 12) + rol32(v4, 18) : P5;
    h += uint32_t(n);
    uint64_t i = n / 16 * 16;
    for (; i + 4 <= n; i += 4) h = rol32(h + ld32u(p + i) * P3, 17) * P4;
    for (; i < n; ++i) h = rol32(h + p[i] * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(kXxWaves * 64) void k_xxh32(const Batch B)
{
    __shared__ uint32_t s_buf[kXxWaves][2][kXxRegion / 4];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t i0 = (blockIdx.x * kXxWaves + wv) * kXxPerWave;  // the wave's first blob (sorted order)
    if (i0 >= B.nblobs) return;
    // the blob this lane loads for (lg) and, for lanes < 4 kXxPerWave, chains (cg)
    const uint32_t lg = lane / kXxLoadLanes, sub = lane % kXxLoadLanes, cg = lane >> 2, a = lane & 3u;
    auto blob = [&](uint32_t g, const uint8_t *&p, uint64_t &n, uint32_t &w) {
        const bool ok = i0 + g < B.nblobs;
        w = ok ? B.xx_ids[i0 + g] : 0u;
        p = B.base + (ok ? B.blobs[w].src : 0);
        n = ok ? B.blobs[w].len : 0;
    };
    const uint8_t *lp, *cp;
    uint64_t ln, cn;
    uint32_t lw, cw;
    blob(lg, lp, ln, lw);
    blob(cg < kXxPerWave ? cg : 0u, cp, cn, cw);
    const uint64_t cstripes = cg < kXxPerWave ? cn / 16 : 0;
    // a global-address-space pointer: flat loads would also count in
    // lgkmcnt, so every LDS wait of the chains would wait for the prefetch too
    const gu32 *A = reinterpret_cast<const gu32 *>(reinterpret_cast<uintptr_t>(lp) & ~uintptr_t(3));
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(lp) & 3u) * 8u;
    // regions: the wave's longest blob (its first: sorted)
    uint64_t n0;
    {
        const uint8_t *p0;
        uint32_t w0;
        blob(0, p0, n0, w0);
    }
    const uint64_t R = (n0 / 16 * 16 + kXxBlobRegion - 1) / kXxBlobRegion;
    // regions r + 1 and r + 2 are in flight (register sets X and Y, taking
    // turns) while the chains run over region r in LDS
    uint32_t X[16], Y[16];
    // Branch-free loads (a load under a lane condition makes the compiler wait
    // for it before the branch joins, serialising the prefetch): indices are
    // clamped to the blob's last aligned word.
    // A misaligned word takes its last bytes from the next aligned word, which
    // holds some of the blob's bytes; an aligned one ignores it (shift 0).
    const uint64_t klast = ln ? ((reinterpret_cast<uintptr_t>(lp) & 3u) + ln - 1) / 4 : 0;
    auto prefetch = [&](uint32_t (&pw)[16], uint64_t r) {
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) {
            const uint64_t k = r * (kXxBlobRegion / 4) + 16 * sub + i;  // blob word
            const uint64_t k0 = min(k, klast), k1 = min(k + 1, klast);
            // the round's input product, off the chain (words past the stripes
            // are loaded from the clamped index and never consumed)
            pw[i] = __builtin_amdgcn_alignbit(A[k1], A[k0], sh) * P2;
        }
    };
    auto store = [&](const uint32_t (&pw)[16], uint64_t r) {
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) s_buf[wv][r & 1][16 * lane + i] = pw[i];
    };
    uint32_t v = a == 0 ? P1 + P2 : a == 1 ? P2 : a == 2 ? 0u : 0u - P1;
    auto chains = [&](uint64_t r) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): region r is in LDS
        __builtin_amdgcn_wave_barrier();
        const uint64_t done = r * (kXxBlobRegion / 16);
        if (cstripes > done) {
            const uint32_t *bw = s_buf[wv][r & 1] + cg * (kXxBlobRegion / 4);
            const uint32_t ns = uint32_t(min<uint64_t>(kXxBlobRegion / 16, cstripes - done));
            uint32_t s = 0;
            for (; s + 8 <= ns; s += 8) {
                uint32_t in[8];
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) in[j] = bw[4 * (s + j) + a];
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) v = rol32(v + in[j], 13) * P1;
            }
            for (; s < ns; ++s) v = rol32(v + bw[4 * s + a], 13) * P1;
        }
        __builtin_amdgcn_wave_barrier();
    };
    if (R) {
        prefetch(X, 0);
        store(X, 0);
        prefetch(X, 1);
        prefetch(Y, 2);
    }
    // step r: chains over r; region r + 1 (set of parity r) into LDS; its set loads r + 3
    for (uint64_t r = 0; r < R; r += 2) {
        chains(r);
        if (r + 1 < R) {
            store(X, r + 1);
            prefetch(X, r + 3);
            chains(r + 1);
            if (r + 2 < R) {
                store(Y, r + 2);
                prefetch(Y, r + 4);
            }
        }
    }
    const uint32_t qb = lane & ~3u;
    const uint32_t v1 = __shfl(v, int(qb)), v2 = __shfl(v, int(qb + 1)), v3 = __shfl(v, int(qb + 2)),
                   v4 = __shfl(v, int(qb + 3));
    if (a == 0 && cg < kXxPerWave && i0 + cg < B.nblobs) B.xxh[cw] = xxh_finish(v1, v2, v3, v4, cp, cn);
}

// ---------------------------------------------------------------------------
// k_lz4_seq: one wave per segment.  Record = (match start | offset << 16,
// match length), segment-relative; the literals before a match are the bytes
// since the previous match's end.
// ---------------------------------------------------------------------------
constexpr uint32_t kSeqWaves = 2;  // 24 KiB of LDS per wave: three workgroups per CU
constexpr uint32_t kSkipShift = 6;  // LZ4's skip trigger

struct alignas(16) SeqLds {
    uint32_t data[kSegLZ / 4 + 4];
    uint16_t tab[1u << kHashBits];
};

__device__ __forceinline__ uint32_t lds_rd32(const SeqLds &L, uint32_t p)  // bytes p..p+3 (any p)
{
    const uint32_t w0 = L.data[p >> 2], w1 = L.data[(p >> 2) + 1];
    return __builtin_amdgcn_alignbit(w1, w0, (p & 3u) * 8u);
}

__device__ __forceinline__ uint32_t lds_rd8(const SeqLds &L, uint32_t p)
{
    return (L.data[p >> 2] >> ((p & 3u) * 8u)) & 255u;
}

__global__ __launch_bounds__(kSeqWaves * 64) void k_lz4_seq(const Batch B)
{
    __shared__ SeqLds s_l[kSeqWaves];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t g = blockIdx.x * kSeqWaves + wv;
    if (g >= B.nsegs) return;
    SeqLds &L = s_l[wv];
    const Seg S = B.segs[g];
    const uint8_t *src = B.base + S.src;
    const uint32_t n = S.len;
    // the segment into LDS, 16 bytes per lane and load (unaligned global
    // loads, all issued before the first store); a short segment's tail is
    // zero-filled from byte loads
    if (n == kSegLZ) {
        uint4 v[kSegLZ / 1024];
#pragma unroll
        for (uint32_t j = 0; j < kSegLZ / 1024; ++j) __builtin_memcpy(&v[j], src + 1024 * j + 16 * lane, 16);
#pragma unroll
        for (uint32_t j = 0; j < kSegLZ / 1024; ++j) *reinterpret_cast<uint4 *>(&L.data[256 * j + 4 * lane]) = v[j];
    } else for (uint32_t i = lane; i < kSegLZ / 16; i += 64) {
        const uint32_t p = 16 * i;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p + 16 <= n) {
            __builtin_memcpy(&v, src + p, 16);
        } else if (p < n) {
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; p + b < n; ++b) w[b >> 2] |= uint32_t(src[p + b]) << (8 * (b & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4 *>(&L.data[4 * i]) = v;
    }
    if (lane < 4) L.data[kSegLZ / 4 + lane] = 0;
    for (uint32_t i = lane; i < (1u << kHashBits); i += 64) L.tab[i] = 0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // LZ4 block rules: a match starts >= 12 bytes before the block's end and
    // the block's last 5 bytes are literals (segments near the end of a block
    // are limited by the block's end, not their own); and a match's first 4
    // bytes lie inside the segment.
    const uint32_t start_lim = min(n >= 4 ? n - 3 : 0u, S.rem > 12 ? S.rem - 12 : 0u);
    const uint32_t end_lim = min(n, S.rem > 5 ? S.rem - 5 : 0u);
    uint2 *rec = B.recs + uint64_t(g) * kRecCap;
    uint32_t cursor = 0, anchor = 0, nrec = 0;
    while (cursor < start_lim) {
        // LZ4's acceleration: the further from the last match, the sparser the
        // positions tried (stride 1 + distance / 64), so incompressible data
        // costs a few steps per segment
        const uint32_t stride = 1u + ((cursor - anchor) >> kSkipShift);
        const uint32_t p = cursor + lane * stride;
        const bool valid = p < start_lim;
        const uint32_t v = valid ? lds_rd32(L, p) : 0u;
        const uint32_t h = (v * 2654435761u) >> (32 - kHashBits);
        const uint32_t cand = valid ? L.tab[h] : 0u;
        const uint32_t c = cand ? cand - 1 : 0u;
        const bool ok = valid && cand != 0u && c < p && lds_rd32(L, c) == v;
        const uint64_t m = __ballot(ok);
        __builtin_amdgcn_wave_barrier();
        if (!m) {
            if (valid) L.tab[h] = uint16_t(p + 1);
            cursor += 64 * stride;
            continue;
        }
        const uint32_t f = uint32_t(__ffsll((unsigned long long)m) - 1);
        uint32_t q = cursor + f * stride;
        uint32_t cq = uint32_t(__builtin_amdgcn_readlane(int(c), int(f)));
        uint32_t len = 4;
        // extend backwards over the positions the stride skipped (not past the
        // last match's end nor the candidate's segment start)
        for (;;) {
            const uint32_t room = min(q - anchor, cq);
            if (!room) break;
            const uint32_t k = lane + 1;
            const bool eq = k <= room && lds_rd8(L, q - k) == lds_rd8(L, cq - k);
            const uint64_t mm = __ballot(!eq);
            const uint32_t run = mm ? uint32_t(__ffsll((unsigned long long)mm) - 1) : 64u;
            const uint32_t back = min(run, room);
            q -= back;
            cq -= back;
            len += back;
            if (back < 64) break;
        }
        for (;;) {
            const uint32_t i = q + len + lane;
            const bool eq = i < end_lim && lds_rd8(L, i) == lds_rd8(L, cq + len + lane);
            const uint64_t mm = __ballot(!eq);
            if (!mm) {
                len += 64;
                continue;
            }
            len += uint32_t(__ffsll((unsigned long long)mm) - 1);
            break;
        }
        if (lane == 0) rec[nrec] = make_uint2(q | ((q - cq) << 16), len);
        ++nrec;
        // the window's positions before the next cursor enter the table (later
        // ones are looked up again from there and would only shadow older
        // candidates)
        if (valid && p < q + len) L.tab[h] = uint16_t(p + 1);
        __builtin_amdgcn_wave_barrier();
        anchor = cursor = q + len;
    }
    if (lane == 0) {
        B.nrec[g] = nrec;
        B.trail[g] = n - anchor;
    }
}

__device__ __forceinline__ uint32_t ext_len(uint32_t x) { return x >= 15 ? (x - 15) / 255 + 1 : 0; }

// ---------------------------------------------------------------------------
// k_lz4_size / k_lz4_emit: one workgroup per LZ4 block.  A sequence's literal
// run starts at the previous match's end (or the block start), across segment
// boundaries; the block ends with a literal-only sequence.
// ---------------------------------------------------------------------------
constexpr uint32_t kBlkThreads = 256;
constexpr uint32_t kMaxSegsPerBlk = uint32_t(kBlockLZ / kSegLZ);

struct BlkLds {
    uint32_t rbase[kMaxSegsPerBlk + 1];  // first record index (block-relative) of each segment
    uint32_t prev_end[kMaxSegsPerBlk];   // block-relative end of the last match before each segment
    uint32_t obase[kMaxSegsPerBlk + 1];  // output offset of each segment's first sequence (emit)
    uint32_t acc[kMaxSegsPerBlk];        // per-segment sequence bytes (size)
    uint32_t wsum[3][kBlkThreads / 64];
    uint64_t total;
};

// Block-relative literal start and size of record r of segment s.
__device__ __forceinline__ void rec_geom(const Batch &B, const Blk &K, const BlkLds &L, uint32_t s, uint32_t r,
                                         uint32_t &lit_start, uint32_t &lit_len, uint32_t &mpos, uint32_t &off,
                                         uint32_t &mlen)
{
    const uint2 *rec = B.recs + uint64_t(K.seg0 + s) * kRecCap;
    const uint2 x = rec[r];
    mpos = s * kSegLZ + (x.x & 0xFFFFu);
    off = x.x >> 16;
    mlen = x.y;
    if (r == 0) {
        lit_start = L.prev_end[s];
    } else {
        const uint2 y = rec[r - 1];
        lit_start = s * kSegLZ + (y.x & 0xFFFFu) + y.y;
    }
    lit_len = mpos - lit_start;
}

__device__ __forceinline__ uint32_t seq_size(uint32_t lit_len, uint32_t mlen)
{
    return 1 + ext_len(lit_len) + lit_len + 2 + ext_len(mlen - 4);
}

// Shared prologue: per-segment record bases, the match end before each
// segment and (emit) each segment's output offset: a thread per kPerThr
// consecutive segments, exclusive sum / max scans over the workgroup.
constexpr uint32_t kPerThr = (kMaxSegsPerBlk + kBlkThreads - 1) / kBlkThreads;

__device__ void blk_prologue(const Batch &B, const Blk &K, BlkLds &L, bool with_out)
{
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    uint32_t nr[kPerThr], en[kPerThr], ob[kPerThr];
    uint32_t c = 0, m = 0, o = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPerThr; ++k) {
        const uint32_t sg = t * kPerThr + k;
        nr[k] = en[k] = ob[k] = 0;
        if (sg < K.nseg) {
            nr[k] = B.nrec[K.seg0 + sg];
            if (nr[k]) {
                const uint2 y = B.recs[uint64_t(K.seg0 + sg) * kRecCap + nr[k] - 1];
                en[k] = sg * kSegLZ + (y.x & 0xFFFFu) + y.y;
            }
            if (with_out) ob[k] = B.seg_out[K.seg0 + sg];
        }
        c += nr[k];
        m = max(m, en[k]);
        o += ob[k];
    }
    // inclusive scans over the wave, then over the waves
    uint32_t ic = c, im = m, io = o;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t yc = __shfl_up(ic, d), ym = __shfl_up(im, d), yo = __shfl_up(io, d);
        if (lane >= d) {
            ic += yc;
            im = max(im, ym);
            io += yo;
        }
    }
    if (lane == 63) {
        L.wsum[0][wv] = ic;
        L.wsum[1][wv] = im;
        L.wsum[2][wv] = io;
    }
    __syncthreads();
    uint32_t bc = 0, bm = 0, bo = 0;
    for (uint32_t i = 0; i < wv; ++i) {
        bc += L.wsum[0][i];
        bm = max(bm, L.wsum[1][i]);
        bo += L.wsum[2][i];
    }
    uint32_t xc = bc + ic - c, xm = max(bm, __shfl_up(im, 1) * (lane ? 1u : 0u)), xo = bo + io - o;  // exclusive
#pragma unroll
    for (uint32_t k = 0; k < kPerThr; ++k) {
        const uint32_t sg = t * kPerThr + k;
        if (sg < K.nseg) {
            L.rbase[sg] = xc;
            L.prev_end[sg] = xm;
            L.obase[sg] = xo;
        }
        xc += nr[k];
        xm = max(xm, en[k]);
        xo += ob[k];
    }
    if (t == kBlkThreads - 1) {
        L.rbase[K.nseg] = xc;
        L.total = xm;  // the last match's end: the final literal run starts here
        L.obase[K.nseg] = xo;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t seg_of(const BlkLds &L, uint32_t nseg, uint32_t r)
{
    uint32_t lo = 0, hi = nseg;  // last s with rbase[s] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.rbase[mid] <= r) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlkThreads) void k_lz4_size(const Batch B)
{
    __shared__ BlkLds L;
    const Blk K = B.blks[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < K.nseg; i += kBlkThreads) L.acc[i] = 0;
    blk_prologue(B, K, L, false);
    const uint32_t nr = L.rbase[K.nseg];
    const uint32_t last_end = uint32_t(L.total);
    for (uint32_t r = threadIdx.x; r < nr; r += kBlkThreads) {
        const uint32_t sg = seg_of(L, K.nseg, r);
        uint32_t ls, ll, mp, off, ml;
        rec_geom(B, K, L, sg, r - L.rbase[sg], ls, ll, mp, off, ml);
        atomicAdd(&L.acc[sg], seq_size(ll, ml));
    }
    __syncthreads();
    uint32_t sum = 0;
    for (uint32_t i = threadIdx.x; i < K.nseg; i += kBlkThreads) {
        B.seg_out[K.seg0 + i] = L.acc[i];
        sum += L.acc[i];
    }
    for (int o = 32; o; o >>= 1) sum += __shfl_xor(sum, o);
    if ((threadIdx.x & 63) == 0) L.wsum[0][threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (uint32_t i = 0; i < kBlkThreads / 64; ++i) t += L.wsum[0][i];
        const uint32_t fl = K.len - last_end;
        t += 1 + ext_len(fl) + fl;
        B.blk_size[blockIdx.x] = t < K.len ? uint32_t(t) : (K.len | 0x80000000u);
    }
}

// ---------------------------------------------------------------------------
// k_enc_plan: one workgroup of 1,024 threads: per blob its frame size (and the
// offsets of its blocks in the frame), GCM pieces and output size; then
// exclusive scans over the blobs, tile by tile.
// ---------------------------------------------------------------------------
constexpr uint32_t kPlanThreads = 1024;

__global__ __launch_bounds__(kPlanThreads) void k_enc_plan(const Batch B)
{
    __shared__ uint64_t s_o[kPlanThreads / 64];
    __shared__ uint32_t s_p[kPlanThreads / 64];
    __shared__ uint64_t s_carry_o;
    __shared__ uint32_t s_carry_p;
    if (threadIdx.x == 0) B.status[1] = 0;  // k_gcm's piece counter
    if (threadIdx.x == 0) {
        s_carry_o = 0;
        s_carry_p = 0;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t t0 = 0; t0 < B.nblobs; t0 += kPlanThreads) {
        const uint32_t b = t0 + threadIdx.x;
        uint64_t O = 0;
        uint32_t P = 0;
        if (b < B.nblobs) {
            const BlobDesc D = B.blobs[b];
            uint64_t F;
            if (B.compress && D.len == 0) {
                F = 0;  // DeflateStream of empty input is an empty stream (compression/compression.go:58-62)
            } else if (B.compress) {
                uint64_t off = 7;
                for (uint32_t k = 0; k < D.nblk; ++k) {
                    B.blk_foff[D.blk0 + k] = off;
                    off += 4 + (B.blk_size[D.blk0 + k] & 0x7FFFFFFFu);
                }
                F = off + 4 + 4;  // end mark, content checksum
            } else {
                F = D.len;
            }
            B.frame_len[b] = F;
            P = B.encrypt ? uint32_t((F + kPiece - 1) / kPiece) : 0u;
            O = B.encrypt ? 12 + 48 + F + 28ull * P : F;
        }
        uint64_t xo = O;
        uint32_t xp = P;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t yo = __shfl_up(xo, d);
            const uint32_t yp = __shfl_up(xp, d);
            if (lane >= d) {
                xo += yo;
                xp += yp;
            }
        }
        if (lane == 63) {
            s_o[wv] = xo;
            s_p[wv] = xp;
        }
        __syncthreads();
        uint64_t bo = s_carry_o;
        uint32_t bp = s_carry_p;
        for (uint32_t i = 0; i < wv; ++i) {
            bo += s_o[i];
            bp += s_p[i];
        }
        if (b < B.nblobs) {
            B.out_off[b] = bo + xo - O;
            B.piece_base[b] = bp + xp - P;
        }
        __syncthreads();
        if (threadIdx.x == kPlanThreads - 1) {
            uint64_t to = 0;
            uint32_t tp = 0;
            for (uint32_t i = 0; i < kPlanThreads / 64; ++i) {
                to += s_o[i];
                tp += s_p[i];
            }
            s_carry_o += to;
            s_carry_p += tp;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        B.out_off[B.nblobs] = s_carry_o;
        B.piece_base[B.nblobs] = s_carry_p;
        B.status[0] = s_carry_o > B.out_cap ? uint64_t(uint32_t(CDC_E_NOSPACE)) : 0ull;
    }
}

// Where the LZ4 stages write blob b's frame: the frame buffer when it is
// encrypted next, else its place in the output.
__device__ __forceinline__ uint8_t *frame_ptr(const Batch &B, uint32_t b)
{
    return B.encrypt ? B.frames + B.blobs[b].slot : B.out + B.out_off[b];
}

// The plaintext the GCM stage seals: the frame, or the blob itself uncompressed.
__device__ __forceinline__ const uint8_t *plain_ptr(const Batch &B, uint32_t b)
{
    return B.compress ? B.frames + B.blobs[b].slot : B.base + B.blobs[b].src;
}

// dst[0, n) = src[0, n) by the threads [tid, nt): aligned dword stores, each
// from two aligned source dwords (v_alignbit); the source's last aligned dword
// is read whole, never past it.
__device__ void copy_span(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t tid, uint32_t nt)
{
    const uint32_t head = uint32_t(min<uint64_t>(n, (4u - (reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u));
    if (tid < head) dst[tid] = src[tid];
    dst += head;
    src += head;
    n -= head;
    const uint64_t nw = n / 4;
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst);
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(src) & 3u) * 8u;
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(src) & ~uintptr_t(3));
    if (sh) {
        for (uint64_t i = tid; i < nw; i += nt) dw[i] = __builtin_amdgcn_alignbit(sw[i + 1], sw[i], sh);
    } else {
        for (uint64_t i = tid; i < nw; i += nt) dw[i] = sw[i];
    }
    for (uint64_t i = 4 * nw + tid; i < n; i += nt) dst[i] = src[i];
}

// Neither compressed nor encrypted: the output is the blob (Encode with no
// compression and no key configured).
__global__ __launch_bounds__(256) void k_copy(const Batch B)
{
    const uint32_t b = blockIdx.x;
    if (b >= B.nblobs || B.status[0]) return;
    copy_span(B.out + B.out_off[b], B.base + B.blobs[b].src, B.blobs[b].len, threadIdx.x, blockDim.x);
}

// Grid (blocks, kEmitSplit): a stored block is copied by all its kEmitSplit
// workgroups, a compressed one written by segment ranges, one per workgroup
// (its output offset from k_lz4_size's per-segment sizes).
constexpr uint32_t kEmitSplit = 16;

__global__ __launch_bounds__(kBlkThreads) void k_lz4_emit(const Batch B)
{
    __shared__ BlkLds L;
    if (B.status[0]) return;
    const Blk K = B.blks[blockIdx.x];
    uint8_t *dst = frame_ptr(B, K.blob) + B.blk_foff[blockIdx.x];
    const uint8_t *src = B.base + K.src;
    const uint32_t bs = B.blk_size[blockIdx.x];
    if (threadIdx.x == 0 && blockIdx.y == 0) {
        dst[0] = uint8_t(bs);
        dst[1] = uint8_t(bs >> 8);
        dst[2] = uint8_t(bs >> 16);
        dst[3] = uint8_t(bs >> 24);
    }
    dst += 4;
    if (bs & 0x80000000u) {  // stored: the raw bytes, a slice per workgroup
        const uint32_t a = uint32_t(uint64_t(K.len) * blockIdx.y / kEmitSplit);
        const uint32_t e = uint32_t(uint64_t(K.len) * (blockIdx.y + 1) / kEmitSplit);
        copy_span(dst + a, src + a, e - a, threadIdx.x, kBlkThreads);
        return;
    }
    // compressed: workgroup y writes the sequences of segments [sa, sb)
    blk_prologue(B, K, L, true);
    const uint32_t sa = K.nseg * blockIdx.y / kEmitSplit, sb = K.nseg * (blockIdx.y + 1) / kEmitSplit;
    const uint32_t r0 = L.rbase[sa], r1 = L.rbase[sb];
    const uint32_t last_end = uint32_t(L.total);
    // tiles of kBlkThreads records: sizes, workgroup-wide exclusive scan, write
    __shared__ uint32_t s_part[kBlkThreads / 64];
    uint32_t carry = L.obase[sa];
    for (uint32_t t0 = r0; t0 < r1; t0 += kBlkThreads) {
        const uint32_t r = t0 + threadIdx.x;
        uint32_t ls = 0, ll = 0, mp = 0, off = 0, ml = 0, sz = 0;
        if (r < r1) {
            const uint32_t sg = seg_of(L, K.nseg, r);
            rec_geom(B, K, L, sg, r - L.rbase[sg], ls, ll, mp, off, ml);
            sz = seq_size(ll, ml);
        }
        uint32_t x = sz;
        const uint32_t lane = threadIdx.x & 63u;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_part[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t wbase = 0;
        for (uint32_t i = 0; i < (threadIdx.x >> 6); ++i) wbase += s_part[i];
        uint32_t tile_total = 0;
        for (uint32_t i = 0; i < kBlkThreads / 64; ++i) tile_total += s_part[i];
        __syncthreads();
        if (r < r1) {
            uint8_t *o = dst + carry + wbase + x - sz;
            const uint32_t lt = ll >= 15 ? 15 : ll, mt = ml - 4 >= 15 ? 15 : ml - 4;
            *o++ = uint8_t(lt << 4 | mt);
            if (ll >= 15) {
                uint32_t e = ll - 15;
                for (; e >= 255; e -= 255) *o++ = 255;
                *o++ = uint8_t(e);
            }
            for (uint32_t i = 0; i < ll; ++i) o[i] = src[ls + i];
            o += ll;
            *o++ = uint8_t(off);
            *o++ = uint8_t(off >> 8);
            if (ml - 4 >= 15) {
                uint32_t e = ml - 4 - 15;
                for (; e >= 255; e -= 255) *o++ = 255;
                *o++ = uint8_t(e);
            }
        }
        carry += tile_total;
    }
    if (threadIdx.x == 0 && sb == K.nseg) {  // the final literal-only sequence
        uint8_t *o = dst + L.obase[K.nseg];
        const uint32_t ll = K.len - last_end;
        *o++ = uint8_t((ll >= 15 ? 15 : ll) << 4);
        if (ll >= 15) {
            uint32_t e = ll - 15;
            for (; e >= 255; e -= 255) *o++ = 255;
            *o++ = uint8_t(e);
        }
        for (uint32_t i = 0; i < ll; ++i) o[i] = src[last_end + i];
    }
}

// Frame header (pierrec/lz4 v4 defaults: version 1, independent blocks,
// content checksum, 4-MiB blocks), end mark and checksum.
__device__ uint32_t xxh32_small(const uint8_t *p, uint32_t n)
{
    uint32_t h = P5 + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) h = rol32(h + ld32u(p + i) * P3, 17) * P4;
    for (; i < n; ++i) h = rol32(h + p[i] * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(64) void k_frame_fin(const Batch B)
{
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= B.nblobs || B.status[0] || B.frame_len[b] == 0) return;  // empty blob: no frame at all
    uint8_t *f = frame_ptr(B, b);
    const uint8_t hdr[6] = {0x04, 0x22, 0x4D, 0x18, 0x64, 0x70};
    for (int i = 0; i < 6; ++i) f[i] = hdr[i];
    f[6] = uint8_t(xxh32_small(hdr + 4, 2) >> 8);
    const uint64_t F = B.frame_len[b];
    uint8_t *e = f + F - 8;
    e[0] = e[1] = e[2] = e[3] = 0;
    const uint32_t x = B.xxh[b];
    e[4] = uint8_t(x);
    e[5] = uint8_t(x >> 8);
    e[6] = uint8_t(x >> 16);
    e[7] = uint8_t(x >> 24);
}

// ---------------------------------------------------------------------------
// GCM
// ---------------------------------------------------------------------------
__device__ __forceinline__ void gcm_block_words(const uint8_t *p, uint32_t w[4])
{
    for (int i = 0; i < 4; ++i)
        w[i] = uint32_t(p[4 * i]) << 24 | uint32_t(p[4 * i + 1]) << 16 | uint32_t(p[4 * i + 2]) << 8 | p[4 * i + 3];
}

// Key setup, in two kernels.  k_blob_keys: one thread per blob (the AES
// tables and the repository key's schedule, H and 4-bit table in LDS, shared
// by the workgroup): the subkey's round keys, H = AES_K(0) and its 4-bit
// table, and the stream header (subkey nonce || Seal(repository key, subkey
// nonce, subkey)).  k_blob_pows: one wave per blob: H^1..H^64 by a doubling
// ladder (round k: lanes [2^k, 2^(k+1)) multiply H^(lane + 1 - 2^k) by H^(2^k)
// with its 4-bit table, built by 16 lanes), then four entries per lane of the
// 8-bit table of H^64 from its eight halvings.
constexpr uint32_t kKeyThreads = 256;
constexpr uint32_t kPowWaves = 4;

__device__ __forceinline__ G128 ghalf(G128 x)  // x times the field's x (one right shift with reduction)
{
    const uint64_t r = (x.lo & 1) ? 0xE100000000000000ull : 0;
    return G128{(x.hi >> 1) ^ r, (x.lo >> 1) | (x.hi << 63)};
}

__global__ __launch_bounds__(kKeyThreads) void k_blob_keys(const Batch B)
{
    __shared__ uint32_t s_te[256];
    __shared__ uint8_t s_sb[256];
    __shared__ uint32_t s_mrk[60];
    __shared__ G128 s_mth[16];
    const uint32_t t = threadIdx.x;
    s_te[t] = g_te0[t];
    s_sb[t] = g_sbox[t];
    __syncthreads();
    if (t == 0) {  // the repository key: schedule, H and its table
        uint8_t key[32];
        for (int i = 0; i < 32; ++i) key[i] = B.key[i];
        uint32_t mk[60];
        aes256_expand(key, mk, s_sb);
        for (int i = 0; i < 60; ++i) s_mrk[i] = mk[i];
        uint32_t z[4] = {0, 0, 0, 0};
        aes256_block(mk, s_te, s_sb, z);
        G128 th[16];
        gtable(g_from_words(z), th);
        for (int i = 0; i < 16; ++i) s_mth[i] = th[i];
    }
    __syncthreads();
    const uint32_t b = blockIdx.x * kKeyThreads + t;
    if (b >= B.nblobs || B.status[0]) return;
    const uint8_t *r = B.rnd + 56ull * b;  // subkey 32, subkey nonce 12, data nonce 12
    BlobKey &K = B.keys[b];
    {
        uint32_t rk[60];
        aes256_expand(r, rk, s_sb);
        for (int i = 0; i < 60; ++i) K.rk[i] = rk[i];
        uint32_t z[4] = {0, 0, 0, 0};
        aes256_block(rk, s_te, s_sb, z);
        const G128 H = g_from_words(z);
        K.hpow[0] = H;
        G128 th[16];
        gtable(H, th);
        for (int i = 0; i < 16; ++i) K.th[i] = th[i];
    }
    // header: subkey nonce || Seal(repository key, subkey nonce, subkey)
    uint8_t *o = B.out + B.out_off[b];
    for (int i = 0; i < 12; ++i) o[i] = r[32 + i];
    const uint8_t *nonce = r + 32;
    uint32_t j0[3];
    j0[0] = uint32_t(nonce[0]) << 24 | uint32_t(nonce[1]) << 16 | uint32_t(nonce[2]) << 8 | nonce[3];
    j0[1] = uint32_t(nonce[4]) << 24 | uint32_t(nonce[5]) << 16 | uint32_t(nonce[6]) << 8 | nonce[7];
    j0[2] = uint32_t(nonce[8]) << 24 | uint32_t(nonce[9]) << 16 | uint32_t(nonce[10]) << 8 | nonce[11];
    G128 S = {0, 0};
    for (uint32_t i = 0; i < 2; ++i) {
        uint32_t c[4] = {j0[0], j0[1], j0[2], 2 + i};
        aes256_block(s_mrk, s_te, s_sb, c);
        uint32_t p[4];
        gcm_block_words(r + 16 * i, p);
        for (int k = 0; k < 4; ++k) {
            c[k] ^= p[k];
            o[12 + 16 * i + 4 * k] = uint8_t(c[k] >> 24);
            o[12 + 16 * i + 4 * k + 1] = uint8_t(c[k] >> 16);
            o[12 + 16 * i + 4 * k + 2] = uint8_t(c[k] >> 8);
            o[12 + 16 * i + 4 * k + 3] = uint8_t(c[k]);
        }
        S = gmul4(gx(S, g_from_words(c)), s_mth);
    }
    S = gmul4(gx(S, G128{0, 256}), s_mth);  // len(A) = 0, len(C) = 256 bits
    uint32_t tg[4] = {j0[0], j0[1], j0[2], 1};
    aes256_block(s_mrk, s_te, s_sb, tg);
    const uint64_t hi = S.hi ^ (uint64_t(tg[0]) << 32 | tg[1]), lo = S.lo ^ (uint64_t(tg[2]) << 32 | tg[3]);
    for (int k = 0; k < 8; ++k) {
        o[44 + k] = uint8_t(hi >> (56 - 8 * k));
        o[52 + k] = uint8_t(lo >> (56 - 8 * k));
    }
}

__global__ __launch_bounds__(kPowWaves * 64) void k_blob_pows(const Batch B)
{
    struct PowLds {
        G128 pw[64];
        G128 tab[16];
    };
    __shared__ PowLds S[kPowWaves];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t b = blockIdx.x * kPowWaves + wv;
    if (b >= B.nblobs || B.status[0]) return;
    PowLds &L = S[wv];
    BlobKey &K = B.keys[b];
    if (lane == 0) L.pw[0] = K.hpow[0];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t m = 1; m < 64; m <<= 1) {
        if (lane < 16) {  // 4-bit table of X = H^m: entry i = XOR of X * x^(3 - j) over the bits j of i
            G128 v = L.pw[m - 1], e = {0, 0};
#pragma unroll
            for (int j = 3; j >= 0; --j) {
                if ((lane >> j) & 1) e = gx(e, v);
                v = ghalf(v);
            }
            L.tab[lane] = e;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        if (lane >= m && lane < 2 * m) L.pw[lane] = gmul4(L.pw[lane - m], L.tab);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    K.hpow[lane] = L.pw[lane];
    // 8-bit table of V = H^64: T[i] = XOR of v_j over the bits j of i, v_7 = V,
    // v_(j-1) = v_j * x (a halving)
    G128 v[8];
    v[7] = L.pw[63];
#pragma unroll
    for (int j = 7; j > 0; --j) v[j - 1] = ghalf(v[j]);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t i = 4 * lane + q;
        G128 e = {0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((i >> j) & 1) e = gx(e, v[j]);
        K.t64[i] = e;
    }
}

// Raw buffer resource over [base, base + bytes): reads past the end return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gcm_rsrc(uint64_t base, uint64_t bytes)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(base));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(base >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(uint32_t(bytes));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>((uint64_t(hi) << 32) | lo), 0, int(n), 0x00020000);
}

// One row per step with 16 waves (12 VGPRs spilled) and one row with 12 waves
// were 1 % and 19 % slower (profiles/r04_gcm_ab.txt, call 5).
constexpr uint32_t kGcmWaves = 12;  // one workgroup per CU (LDS: the 64-KiB table), three waves per SIMD
constexpr uint32_t kGcmRows = 2;    // rows of 64 blocks per step (their AES interleaved)

// LDS of a GCM workgroup.  Two T-tables, A = Te0 and B = Te0 rotated right by
// 8 bits, 32 copies each, in one 256-byte row per entry: A's copy c at byte
// 256 e + 4 c, B's at 256 e + 128 + 4 c.  A ds_read_b32 serves its lanes in
// two groups of 32 with banks (a/4) mod 32, so lane l reading copy l & 31 is
// conflict-free whatever the state bytes, and the address is ONE v_perm of
// the state word and the lane's offset (B: the instruction's offset 128).
// With B, a column is A[a] ^ B[b] ^ ror16(A[c] ^ B[d] ^ ror16(rk)): one
// rotate instead of three (rk16 holds the round keys rotated by 16).
struct GcmLds {
    uint32_t te[256 * 64];
    struct PerWave {
        uint32_t rk[60];
        uint32_t rk16[60];
        G128 th[16];
        G128 t64[256];
        uint4 stage[64 * kGcmRows];
    } w[kGcmWaves];
};

// Address of state byte k of word w in the 64-copy table.
__device__ __forceinline__ uint32_t te_addr(uint32_t laneoff, uint32_t w, uint32_t k)
{
    return __builtin_amdgcn_perm(laneoff, w, 0x0C0C0004u | (k << 8));
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int N>
__device__ __forceinline__ void aes256_blocks_lds(const GcmLds::PerWave &PW, const char *te, uint32_t laneoff,
                                                  uint32_t (&st)[N][4])
{
    const uint32_t *rk = PW.rk, *rk16 = PW.rk16;
    auto A = [&](uint32_t w, uint32_t k) { return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k)); };
    auto B = [&](uint32_t w, uint32_t k) {
        return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k) + 128);
    };
    uint32_t s[N][4];
#pragma unroll
    for (int n = 0; n < N; ++n)
        for (int q = 0; q < 4; ++q) s[n][q] = st[n][q] ^ rk[q];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
#pragma unroll
        for (int n = 0; n < N; ++n) {
            uint32_t t[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t u = xor3(A(s[n][(q + 2) & 3], 1), B(s[n][(q + 3) & 3], 0), rk16[4 * r + q]);
                t[q] = xor3(A(s[n][q], 3), B(s[n][(q + 1) & 3], 2), ror32(u, 16));
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) s[n][q] = t[q];
        }
    }
    // last round: S-box bytes (byte 2 of A's entries) gathered by v_perm
    auto S4 = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
        const uint32_t hi = __builtin_amdgcn_perm(A(a, 3), A(b, 2), 0x0602FFFFu);  // [Sa, Sb, -, -]
        const uint32_t lo = __builtin_amdgcn_perm(A(c, 1), A(d, 0), 0xFFFF0602u);  // [-, -, Sc, Sd]
        return (hi & 0xFFFF0000u) | (lo & 0xFFFFu);
    };
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            st[n][q] = S4(s[n][q], s[n][(q + 1) & 3], s[n][(q + 2) & 3], s[n][(q + 3) & 3]) ^ rk[56 + q];
}

// Counter mode within one piece: the counter block is (J0[0..2], ctr) with
// ctr < 2^16 (at most 4,097 blocks), so after the first AddRoundKey the
// words s0..s2 and bytes 2-3 of s3 are the piece's constants.  Round 1's
// outputs t2, t3 are then constants, and t0, t1 each depend on one counter
// byte; round 2 takes 8 of its 16 lookups from t2, t3.  Those are done once
// per piece (CtrPre, wave-uniform: SGPRs), leaving 2 + 8 lookups for rounds
// 1-2 instead of 32 (counter-mode caching).
struct CtrPre {
    uint32_t p0t, p0u, p1t, p1u;  // round 1: t0 = p0t ^ ror16(p0u ^ B(s3, 0)), t1 = p1t ^ ror16(p1u ^ A(s3, 1))
    uint32_t r0, w1, v1, w2, w3, v3;  // round 2's constant terms
};

__device__ __forceinline__ CtrPre ctr_pre(const GcmLds::PerWave &PW, const char *te, uint32_t laneoff,
                                          const uint32_t (&j0)[3])
{
    const uint32_t *rk = PW.rk, *rk16 = PW.rk16;
    auto A = [&](uint32_t w, uint32_t k) { return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k)); };
    auto B = [&](uint32_t w, uint32_t k) {
        return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k) + 128);
    };
    auto u = [](uint32_t x) { return uint32_t(__builtin_amdgcn_readfirstlane(int(x))); };
    const uint32_t s0 = j0[0] ^ rk[0], s1 = j0[1] ^ rk[1], s2 = j0[2] ^ rk[2], s3 = rk[3];  // s3: bytes 2-3 only
    CtrPre c;
    c.p0t = u(A(s0, 3) ^ B(s1, 2));
    c.p0u = u(A(s2, 1) ^ rk16[4]);
    c.p1t = u(A(s1, 3) ^ B(s2, 2));
    c.p1u = u(B(s0, 0) ^ rk16[5]);
    const uint32_t t2 = xor3(A(s2, 3), B(s3, 2), ror32(xor3(A(s0, 1), B(s1, 0), rk16[6]), 16));
    const uint32_t t3 = xor3(A(s3, 3), B(s0, 2), ror32(xor3(A(s1, 1), B(s2, 0), rk16[7]), 16));
    c.r0 = u(ror32(xor3(A(t2, 1), B(t3, 0), rk16[8]), 16));
    c.w1 = u(B(t2, 2));
    c.v1 = u(A(t3, 1) ^ rk16[9]);
    c.w2 = u(A(t2, 3) ^ B(t3, 2));
    c.w3 = u(A(t3, 3));
    c.v3 = u(B(t2, 0) ^ rk16[11]);
    return c;
}

// AES-256 of N counter blocks (J0[0..2], ctr[n]) of the piece CtrPre was made for.
template <int N>
__device__ __forceinline__ void aes256_ctr_lds(const GcmLds::PerWave &PW, const char *te, uint32_t laneoff,
                                               const CtrPre &c, const uint32_t (&ctr)[N], uint32_t (&st)[N][4])
{
    const uint32_t *rk = PW.rk, *rk16 = PW.rk16;
    auto A = [&](uint32_t w, uint32_t k) { return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k)); };
    auto B = [&](uint32_t w, uint32_t k) {
        return *reinterpret_cast<const uint32_t *>(te + te_addr(laneoff, w, k) + 128);
    };
    uint32_t s[N][4];
#pragma unroll
    for (int n = 0; n < N; ++n) {
        const uint32_t s3 = ctr[n] ^ rk[3];
        const uint32_t t0 = c.p0t ^ ror32(c.p0u ^ B(s3, 0), 16);
        const uint32_t t1 = c.p1t ^ ror32(c.p1u ^ A(s3, 1), 16);
        s[n][0] = xor3(A(t0, 3), B(t1, 2), c.r0);
        s[n][1] = xor3(A(t1, 3), c.w1, ror32(c.v1 ^ B(t0, 0), 16));
        s[n][2] = c.w2 ^ ror32(xor3(A(t0, 1), B(t1, 0), rk16[10]), 16);
        s[n][3] = xor3(c.w3, B(t0, 2), ror32(A(t1, 1) ^ c.v3, 16));
    }
#pragma unroll
    for (int r = 3; r < 14; ++r) {
#pragma unroll
        for (int n = 0; n < N; ++n) {
            uint32_t t[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t v = xor3(A(s[n][(q + 2) & 3], 1), B(s[n][(q + 3) & 3], 0), rk16[4 * r + q]);
                t[q] = xor3(A(s[n][q], 3), B(s[n][(q + 1) & 3], 2), ror32(v, 16));
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) s[n][q] = t[q];
        }
    }
    auto S4 = [&](uint32_t a, uint32_t b, uint32_t cc, uint32_t d) {
        const uint32_t hi = __builtin_amdgcn_perm(A(a, 3), A(b, 2), 0x0602FFFFu);
        const uint32_t lo = __builtin_amdgcn_perm(A(cc, 1), A(d, 0), 0xFFFF0602u);
        return (hi & 0xFFFF0000u) | (lo & 0xFFFFu);
    };
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            st[n][q] = S4(s[n][q], s[n][(q + 1) & 3], s[n][(q + 2) & 3], s[n][(q + 3) & 3]) ^ rk[56 + q];
}

// x * V with V's 8-bit table, reduced once.  x = sum over its bytes b_i
// (i = 0: the top byte of hi, GCM's x^0..x^7) of b_i x^(8 i), so x V =
// sum t[b_i] x^(8 i): each entry shifted right by 8 i bits into a 256-bit
// sum D[0..7] (dwords, D[0] the most significant), then the part past x^127
// folded back once, x^128 = 1 + x + x^2 + x^7.  The entries of one byte
// offset (i = g, g + 4, g + 8, g + 12) add at whole dwords, so only four
// partial sums are shifted; no reduction per byte (Horner's byte-by-byte
// shift and reduce took twice the VALU), and no step waits on another.
__device__ __forceinline__ G128 gmul8(G128 x, const G128 *t)
{
    const uint32_t xw[4] = {uint32_t(x.hi >> 32), uint32_t(x.hi), uint32_t(x.lo >> 32), uint32_t(x.lo)};
    uint32_t D[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        uint32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const G128 e = t[(xw[j] >> (24 - 8 * g)) & 255u];
            const uint32_t ew[4] = {uint32_t(e.hi >> 32), uint32_t(e.hi), uint32_t(e.lo >> 32), uint32_t(e.lo)};
#pragma unroll
            for (int k = 0; k < 4; ++k) a[j + k] ^= ew[k];
        }
        if (g == 0) {
#pragma unroll
            for (int k = 0; k < 7; ++k) D[k] = a[k];
            D[7] = 0;
        } else {
            const uint32_t s = 8u * g;
            D[0] ^= a[0] >> s;
#pragma unroll
            for (int k = 1; k < 7; ++k) D[k] ^= __builtin_amdgcn_alignbit(a[k - 1], a[k], s);
            D[7] ^= a[6] << (32u - s);
        }
    }
    // fold: V = D[4..7] (x^128..x^247, so V (1 + x + x^2 + x^7) stays below x^127)
    uint32_t F[4];
    F[0] = xor3(D[4], D[4] >> 1, D[4] >> 2) ^ (D[4] >> 7);
#pragma unroll
    for (int k = 1; k < 4; ++k)
        F[k] = xor3(D[4 + k], __builtin_amdgcn_alignbit(D[3 + k], D[4 + k], 1),
                    __builtin_amdgcn_alignbit(D[3 + k], D[4 + k], 2)) ^
               __builtin_amdgcn_alignbit(D[3 + k], D[4 + k], 7);
    return G128{uint64_t(D[0] ^ F[0]) << 32 | (D[1] ^ F[1]), uint64_t(D[2] ^ F[2]) << 32 | (D[3] ^ F[3])};
}

__device__ __forceinline__ uint32_t be32(uint32_t x) { return __builtin_bswap32(x); }

__global__ __launch_bounds__(kGcmWaves * 64) void k_gcm(const Batch B)
{
    __shared__ GcmLds L;
    for (uint32_t i = threadIdx.x; i < 256 * 64; i += blockDim.x)
        L.te[i] = (i & 32u) ? ror32(g_te0[i >> 6], 8) : g_te0[i >> 6];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u, laneoff = (lane & 31u) << 2;
    const char *te = reinterpret_cast<const char *>(L.te);
    __syncthreads();
    // Persistent: one workgroup per CU; each wave takes pieces from a counter
    // (B.status[1], zeroed by k_enc_plan) until none is left, so the last
    // round of pieces does not leave most CUs idle.
    const uint32_t total = B.piece_base[B.nblobs];
    if (B.status[0]) return;
    for (;;) {
    // every lane in the atomic (lane 0 adds 1): no lane-0 branch before the
    // readfirstlane, which the compiler could thread apart (cdc_kernels.hip wave_ticket)
    uint32_t pc = atomicAdd(reinterpret_cast<uint32_t *>(&B.status[1]), lane == 0 ? 1u : 0u);
    pc = uint32_t(__builtin_amdgcn_readfirstlane(int(pc)));
    if (pc >= total) break;
    uint32_t b;
    {
        uint32_t lo = 0, hi = B.nblobs;  // last blob with piece_base <= pc
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (B.piece_base[mid] <= pc) lo = mid;
            else hi = mid;
        }
        b = lo;
        const BlobKey &K = B.keys[b];
        // this wave's tables (the previous piece's reads of them are done: the
        // wave barrier at the end of its loop body)
        for (uint32_t i = lane; i < 60; i += 64) L.w[wv].rk[i] = K.rk[i];
        for (uint32_t i = lane; i < 60; i += 64) L.w[wv].rk16[i] = ror32(K.rk[i], 16);
        if (lane < 16) L.w[wv].th[lane] = K.th[lane];
        for (uint32_t i = lane; i < 256; i += 64) L.w[wv].t64[i] = K.t64[i];
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }
    const BlobKey &K = B.keys[b];
    const uint32_t k = pc - B.piece_base[b];
    const uint64_t F = B.frame_len[b];
    const uint64_t p0 = uint64_t(k) * kPiece;
    const uint32_t m = uint32_t(min<uint64_t>(kPiece, F - p0));  // piece bytes
    const uint32_t nb = (m + 15) / 16;
    const gu8 *pt = reinterpret_cast<const gu8 *>(reinterpret_cast<uintptr_t>(plain_ptr(B, b) + p0));
    const uint32_t pt_sh = uint32_t(reinterpret_cast<uintptr_t>(pt) & 3u);
    uint8_t *o = B.out + B.out_off[b] + 60 + uint64_t(k) * (kPiece + 28);
    const uint8_t *dn = B.rnd + 56ull * b + 44;  // data nonce
    uint32_t j0[3];
    j0[0] = uint32_t(dn[0]) << 24 | uint32_t(dn[1]) << 16 | uint32_t(dn[2]) << 8 | dn[3];
    j0[1] = uint32_t(dn[4]) << 24 | uint32_t(dn[5]) << 16 | uint32_t(dn[6]) << 8 | dn[7];
    j0[2] = (uint32_t(dn[8]) << 24 | uint32_t(dn[9]) << 16 | uint32_t(dn[10]) << 8 | dn[11]) ^ k;
    if (lane < 12) o[lane] = uint8_t(j0[lane >> 2] >> (24 - 8 * (lane & 3)));
    uint8_t *ct = o + 12;
    const CtrPre cpre = ctr_pre(L.w[wv], te, laneoff, j0);
    const G128 *t64 = L.w[wv].t64;
    uint8_t *stage = reinterpret_cast<uint8_t *>(L.w[wv].stage);
    // The piece's plaintext as dwords from its aligned-down start (block i:
    // dwords 4 i .. 4 i + 4, funnel-shifted by its offset in a dword).  A raw
    // buffer returns 0 past its last dword, so every lane loads without a
    // lane condition and a step's loads go out before its AES, which hides
    // their latency (loads under a lane condition were waited for at once).
    const uint32_t lastq = (pt_sh + m - 1) >> 2;
    const __amdgpu_buffer_rsrc_t prs = gcm_rsrc(reinterpret_cast<uintptr_t>(pt) - pt_sh, uint64_t(lastq + 1) * 4);
    const bool pt_fast = pt_sh == 0 && (m & 15u) == 0;  // whole aligned blocks: one 16-byte load each
    // row j: blocks 64 j + lane (1 KiB of the piece), two rows per step (their
    // AES interleaved); lane: Horner in H^64 over its blocks, in order
    G128 Z = {0, 0};
    uint32_t cnt = 0;
    const uint32_t rows = (nb + 63) / 64;
    for (uint32_t j = 0; j < rows; j += kGcmRows) {
        uint32_t c[kGcmRows][4];
#pragma unroll
        for (int u = 0; u < int(kGcmRows); ++u) {
            c[u][0] = j0[0];
            c[u][1] = j0[1];
            c[u][2] = j0[2];
            c[u][3] = 2 + 64 * (j + u) + lane;
        }
        uint32_t px[kGcmRows][5];
#pragma unroll
        for (int u = 0; u < int(kGcmRows); ++u) {
            const int32_t i = int32_t(64 * (j + u) + lane);
            if (pt_fast) {
                const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(prs, 16 * i, 0, 0));
                px[u][0] = v.x;
                px[u][1] = v.y;
                px[u][2] = v.z;
                px[u][3] = v.w;
                px[u][4] = 0;
            } else {
                // dword by dword, clamped to the last one (a wide load that
                // straddles the buffer's end may read as wholly out of range)
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    px[u][q] = __builtin_amdgcn_raw_buffer_load_b32(prs, int32_t(4 * min(uint32_t(4 * i + q), lastq)), 0, 0);
            }
        }
#ifndef GCM_DIAG_NO_AES  // build-time diagnostic only: no keystream (timing only)
        {
            uint32_t ctr[kGcmRows];
#pragma unroll
            for (uint32_t u = 0; u < kGcmRows; ++u) ctr[u] = c[u][3];
            aes256_ctr_lds<kGcmRows>(L.w[wv], te, laneoff, cpre, ctr, c);
        }
#endif
#pragma unroll
        for (int u = 0; u < int(kGcmRows); ++u) {
            const uint32_t i = 64 * (j + u) + lane;
            uint4 cw = make_uint4(0, 0, 0, 0);
            if (i < nb) {
                const uint32_t bytes = min(16u, m - 16 * i);
                uint32_t pw[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) pw[q] = be32(__builtin_amdgcn_alignbit(px[u][q + 1], px[u][q], 8 * pt_sh));
                uint32_t w[4];
                for (int q = 0; q < 4; ++q) w[q] = c[u][q] ^ pw[q];
                if (bytes < 16) {  // the keystream past the piece's end is not ciphertext (nor hashed)
                    for (int q = 0; q < 4; ++q) {
                        const int keep = int(bytes) - 4 * q;
                        w[q] = keep >= 4 ? w[q] : keep <= 0 ? 0u : (w[q] & ~(0xFFFFFFFFu >> (8 * keep)));
                    }
                }
                cw = make_uint4(be32(w[0]), be32(w[1]), be32(w[2]), be32(w[3]));
#ifdef GCM_DIAG_NO_GHASH  // build-time diagnostic only: no multiply by H^64 (timing only)
                Z = gx(Z, G128{uint64_t(w[0]) << 32 | w[1], uint64_t(w[2]) << 32 | w[3]});
#else
                Z = gx(gmul8(Z, t64), G128{uint64_t(w[0]) << 32 | w[1], uint64_t(w[2]) << 32 | w[3]});
#endif
                ++cnt;
            }
            L.w[wv].stage[64 * u + lane] = cw;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t row_bytes = min(1024u * kGcmRows, m - 1024 * j);
        // the rows' ciphertext through LDS: the bytes up to the first aligned
        // dword of the destination, then 8 coalesced dword stores (each dword
        // funnel-shifted from two of the stage's), then the last 0-3 bytes
        {
            uint8_t *dst = ct + 1024 * j;
            const uint32_t hb = min((4u - uint32_t(reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u, row_bytes);
            const uint32_t nd = (row_bytes - hb) >> 2, tb = row_bytes - hb - 4 * nd;
            const uint32_t *sw = reinterpret_cast<const uint32_t *>(stage);
            uint32_t *dw = reinterpret_cast<uint32_t *>(dst + hb);
#pragma unroll
            for (uint32_t q = 0; q < 4 * kGcmRows; ++q) {
                const uint32_t d = 64 * q + lane;
                if (d < nd) dw[d] = __builtin_amdgcn_alignbit(sw[min(d + 1, 256u * kGcmRows - 1)], sw[d], 8 * hb);
            }
            if (lane < hb) dst[lane] = stage[lane];
            if (lane < tb) dst[hb + 4 * nd + lane] = stage[hb + 4 * nd + lane];
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (cnt) {
        const uint32_t e = nb - lane - 64 * (cnt - 1);  // 1..64
        Z = gmul_bits(Z, K.hpow[e - 1]);
    }
    for (int off = 32; off; off >>= 1) {
        Z.hi ^= __shfl_xor(Z.hi, off);
        Z.lo ^= __shfl_xor(Z.lo, off);
    }
    if (lane == 0) {
        G128 S = gmul4(gx(Z, G128{0, uint64_t(m) * 8}), L.w[wv].th);
        uint32_t t[1][4] = {{j0[0], j0[1], j0[2], 1}};
        aes256_blocks_lds<1>(L.w[wv], te, laneoff, t);
        const uint64_t hi = S.hi ^ (uint64_t(t[0][0]) << 32 | t[0][1]), lo = S.lo ^ (uint64_t(t[0][2]) << 32 | t[0][3]);
        uint8_t *tag = ct + m;
        for (int q = 0; q < 8; ++q) {
            tag[q] = uint8_t(hi >> (56 - 8 * q));
            tag[8 + q] = uint8_t(lo >> (56 - 8 * q));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
static std::once_flag g_tab_once;
static int g_tab_status = CDC_OK;

static int ensure_tables()
{
    std::call_once(g_tab_once, [] {
        uint32_t te0[256];
        uint8_t sbox[256];
        build_tables(te0, sbox);
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            g_tab_status = CDC_E_DEVICE;
            return;
        }
        int cur = 0;
        (void)hipGetDevice(&cur);
        for (int d = 0; d < n; ++d) {
            if (hipSetDevice(d) != hipSuccess || hipMemcpyToSymbol(HIP_SYMBOL(g_te0), te0, sizeof(te0)) != hipSuccess ||
                hipMemcpyToSymbol(HIP_SYMBOL(g_sbox), sbox, sizeof(sbox)) != hipSuccess)
                g_tab_status = CDC_E_DEVICE;
        }
        (void)hipSetDevice(cur);
    });
    return g_tab_status;
}

static uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

// k_gcm's persistent grid: one workgroup per CU (its LDS holds one).
static uint64_t gcm_wgs()
{
    static const uint64_t n = [] {
        int c = 0, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return uint64_t(c);
    }();
    return n;
}

// Workspace kept per device between calls (grow-only); a call holds its
// device's lock while it runs (the entry point is synchronous).
struct WsCache {
    std::mutex mu;
    uint8_t *p = nullptr;
    size_t cap = 0;
    uint8_t *hp = nullptr;  // pinned staging of the host plan (one DMA instead of pageable copies)
    size_t hcap = 0;
    hipStream_t aux = nullptr;  // k_xxh32 runs here, beside the LZ4 and GCM kernels
    hipEvent_t fork = nullptr, join = nullptr;
};
// Two per device: a caller that runs two Encode calls at once (the backup
// pipeline's two encoder threads) picks the second with cdc::t_encode_ws = 1,
// so one call's kernels run beside the other's copy-back.
static WsCache g_ws[64][2];

}  // namespace enc

namespace cdc {
thread_local int t_encode_ws = 0;
}

using namespace enc;

// Device-resident encode of n blobs (see include/plakar_cdc.h).
extern "C" int cdc_encode_device(int device, const void *d_base, const uint64_t *offsets, const uint64_t *lens,
                                 uint32_t n, int compress, const uint8_t *key, const uint8_t *random, uint8_t *d_out,
                                 uint64_t out_cap, uint64_t *out_offsets, void *stream)
{
    if ((n && (!d_base || !offsets || !lens || !out_offsets)) || (key && !random) || !d_out) return CDC_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    int st = ensure_tables();
    if (st != CDC_OK) return st;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool encrypt = key != nullptr;
    // plan on the host: blobs, 4-MiB blocks, 8-KiB segments, frame slots.
    // Counted first, then written straight into the pinned staging at their
    // workspace offsets (no vectors, no copy).
    size_t nk = 0, ng = 0;
    uint64_t slot = 0, pieces_max = 0;
    for (uint32_t b = 0; b < n; ++b) {
        const uint64_t nblk = compress ? (lens[b] + kBlockLZ - 1) / kBlockLZ : 0;
        nk += nblk;
        if (nblk) ng += (nblk - 1) * ((kBlockLZ + kSegLZ - 1) / kSegLZ) +
                        (lens[b] - (nblk - 1) * kBlockLZ + kSegLZ - 1) / kSegLZ;
        const uint64_t fmax = compress ? 7 + 4ull * nblk + lens[b] + 8 : lens[b];
        slot += align16(fmax);
        pieces_max += encrypt ? (fmax + kPiece - 1) / kPiece : 0;
    }
    // one device allocation for the plan and the workspace
    const size_t nb = n;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = align16(off + bytes);
        return o;
    };
    const size_t o_blobs = take(nb * sizeof(BlobDesc)), o_blks = take(nk * sizeof(Blk)), o_segs = take(ng * sizeof(Seg));
    const size_t o_rnd = take(encrypt ? nb * 56 : 0), o_key = take(32);
    const size_t o_recs = take(ng * kRecCap * sizeof(uint2)), o_nrec = take(ng * 4), o_trail = take(ng * 4),
                 o_sout = take(ng * 4);
    const size_t o_bsz = take(nk * 4), o_bfo = take(nk * 8), o_xxh = take(nb * 4), o_flen = take(nb * 8);
    const size_t o_oo = take((nb + 1) * 8), o_pb = take((nb + 1) * 4), o_keys = take(encrypt ? nb * sizeof(BlobKey) : 0);
    const size_t o_status = take(16), o_frames = take(encrypt ? slot : 0), o_xx = take(compress ? nb * 4 : 0);
    if (device < 0 || device >= 64) return CDC_E_INVALID;
    WsCache &C = g_ws[device][cdc::t_encode_ws & 1];
    std::lock_guard<std::mutex> lk(C.mu);
    if (C.cap < off) {
        if (C.p) (void)hipFree(C.p);
        C.p = nullptr;
        C.cap = 0;
        if (hipMalloc(&C.p, off) != hipSuccess) return CDC_E_DEVICE;
        C.cap = off;
    }
    uint8_t *ws = C.p;
    if (!C.aux && (hipStreamCreateWithFlags(&C.aux, hipStreamNonBlocking) != hipSuccess ||
                   hipEventCreateWithFlags(&C.fork, hipEventDisableTiming) != hipSuccess ||
                   hipEventCreateWithFlags(&C.join, hipEventDisableTiming) != hipSuccess))
        return CDC_E_DEVICE;
    // The plan's tables at their workspace offsets [0, o_key + 32) in pinned
    // staging, XXH32 order after them: two DMAs.  (The call ends with a
    // stream sync under C.mu, so the staging is free again on return.)
    const size_t h_prefix = o_key + 32, h_xx = align16(h_prefix), h_need = h_xx + (compress ? nb * 4 : 0);
    if (C.hcap < h_need) {
        if (C.hp) (void)hipHostFree(C.hp);
        C.hp = nullptr;
        C.hcap = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&C.hp), h_need, hipHostMallocDefault) != hipSuccess)
            return CDC_E_NOMEM;
        C.hcap = h_need;
    }
    {
        BlobDesc *blobs = reinterpret_cast<BlobDesc *>(C.hp + o_blobs);
        Blk *blks = reinterpret_cast<Blk *>(C.hp + o_blks);
        Seg *segs = reinterpret_cast<Seg *>(C.hp + o_segs);
        uint32_t kb = 0, kg = 0;
        uint64_t sl = 0;
        for (uint32_t b = 0; b < n; ++b) {
            BlobDesc D{};
            D.src = offsets[b];
            D.len = lens[b];
            D.blk0 = kb;
            D.nblk = compress ? uint32_t((lens[b] + kBlockLZ - 1) / kBlockLZ) : 0u;
            for (uint32_t k = 0; k < D.nblk; ++k) {
                Blk K{};
                K.src = offsets[b] + k * kBlockLZ;
                K.len = uint32_t(std::min<uint64_t>(kBlockLZ, lens[b] - k * kBlockLZ));
                K.blob = b;
                K.k = k;
                K.seg0 = kg;
                K.nseg = (K.len + kSegLZ - 1) / kSegLZ;
                for (uint32_t g = 0; g < K.nseg; ++g) {
                    Seg S{};
                    S.src = K.src + uint64_t(g) * kSegLZ;
                    S.len = std::min<uint32_t>(kSegLZ, K.len - g * kSegLZ);
                    S.rem = K.len - g * kSegLZ;
                    segs[kg++] = S;
                }
                blks[kb++] = K;
            }
            const uint64_t fmax = compress ? 7 + 4ull * D.nblk + lens[b] + 8 : lens[b];
            D.slot = sl;
            sl += align16(fmax);
            blobs[b] = D;
        }
        if (kb != nk || kg != ng) return CDC_E_INVALID;  // the counting pass and the plan disagree (a bug)
        if (encrypt) {
            std::memcpy(C.hp + o_rnd, random, nb * 56);
            std::memcpy(C.hp + o_key, key, 32);
        }
        if (compress && nb) {
            // XXH32 order: longest first (a wave's blobs end together); ties by
            // index, so the order is the stable one.  Keys (~len, index) sort
            // without an indirection per comparison.
            thread_local std::vector<uint64_t> xk;
            xk.resize(nb);
            for (uint32_t b = 0; b < n; ++b)
                xk[b] = (uint64_t(0xFFFFFFFFu - uint32_t(std::min<uint64_t>(lens[b], 0xFFFFFFFFu))) << 32) | b;
            std::sort(xk.begin(), xk.end());
            uint32_t *xx = reinterpret_cast<uint32_t *>(C.hp + h_xx);
            for (size_t i = 0; i < nb; ++i) xx[i] = uint32_t(xk[i]);
        }
    }
    Batch Bt{};
    Bt.base = static_cast<const uint8_t *>(d_base);
    Bt.nblobs = n;
    Bt.nsegs = uint32_t(ng);
    Bt.nblks = uint32_t(nk);
    Bt.npieces_max = uint32_t(pieces_max);
    Bt.compress = compress ? 1u : 0u;
    Bt.encrypt = encrypt ? 1u : 0u;
    Bt.blobs = reinterpret_cast<BlobDesc *>(ws + o_blobs);
    Bt.blks = reinterpret_cast<Blk *>(ws + o_blks);
    Bt.segs = reinterpret_cast<Seg *>(ws + o_segs);
    Bt.rnd = ws + o_rnd;
    Bt.key = ws + o_key;
    Bt.frames = ws + o_frames;
    Bt.out = d_out;
    Bt.out_cap = out_cap;
    Bt.recs = reinterpret_cast<uint2 *>(ws + o_recs);
    Bt.nrec = reinterpret_cast<uint32_t *>(ws + o_nrec);
    Bt.trail = reinterpret_cast<uint32_t *>(ws + o_trail);
    Bt.seg_out = reinterpret_cast<uint32_t *>(ws + o_sout);
    Bt.blk_size = reinterpret_cast<uint32_t *>(ws + o_bsz);
    Bt.blk_foff = reinterpret_cast<uint64_t *>(ws + o_bfo);
    Bt.xxh = reinterpret_cast<uint32_t *>(ws + o_xxh);
    Bt.frame_len = reinterpret_cast<uint64_t *>(ws + o_flen);
    Bt.out_off = reinterpret_cast<uint64_t *>(ws + o_oo);
    Bt.piece_base = reinterpret_cast<uint32_t *>(ws + o_pb);
    Bt.keys = reinterpret_cast<BlobKey *>(ws + o_keys);
    Bt.status = reinterpret_cast<uint64_t *>(ws + o_status);
    Bt.xx_ids = reinterpret_cast<uint32_t *>(ws + o_xx);
    const uint32_t xx_wgs = (n + kXxWaves * kXxPerWave - 1) / (kXxWaves * kXxPerWave);
    bool ok = hipMemcpyAsync(ws, C.hp, h_prefix, hipMemcpyHostToDevice, s) == hipSuccess;
    if (compress && nb)
        ok = ok && hipMemcpyAsync(ws + o_xx, C.hp + h_xx, nb * 4, hipMemcpyHostToDevice, s) == hipSuccess;
    if (ok && n) {
        if (compress) {
            ok = hipEventRecord(C.fork, s) == hipSuccess && hipStreamWaitEvent(C.aux, C.fork, 0) == hipSuccess;
            hipLaunchKernelGGL(k_xxh32, dim3(xx_wgs), dim3(kXxWaves * 64), 0, C.aux, Bt);
            ok = ok && hipEventRecord(C.join, C.aux) == hipSuccess;
            if (ng) hipLaunchKernelGGL(k_lz4_seq, dim3(uint32_t((ng + kSeqWaves - 1) / kSeqWaves)), dim3(kSeqWaves * 64), 0, s, Bt);
            if (nk) hipLaunchKernelGGL(k_lz4_size, dim3(uint32_t(nk)), dim3(kBlkThreads), 0, s, Bt);
        }
        hipLaunchKernelGGL(k_enc_plan, dim3(1), dim3(kPlanThreads), 0, s, Bt);
        if (encrypt) {
            hipLaunchKernelGGL(k_blob_keys, dim3((n + kKeyThreads - 1) / kKeyThreads), dim3(kKeyThreads), 0, s, Bt);
            hipLaunchKernelGGL(k_blob_pows, dim3((n + kPowWaves - 1) / kPowWaves), dim3(kPowWaves * 64), 0, s, Bt);
        }
        if (compress) {
            if (nk) hipLaunchKernelGGL(k_lz4_emit, dim3(uint32_t(nk), kEmitSplit), dim3(kBlkThreads), 0, s, Bt);
            ok = ok && hipStreamWaitEvent(s, C.join, 0) == hipSuccess;  // the content checksums
            hipLaunchKernelGGL(k_frame_fin, dim3((n + 63) / 64), dim3(64), 0, s, Bt);
        } else if (!encrypt) {
            hipLaunchKernelGGL(k_copy, dim3(n), dim3(256), 0, s, Bt);
        }
        if (encrypt && pieces_max)
            hipLaunchKernelGGL(k_gcm, dim3(uint32_t(std::min<uint64_t>((pieces_max + kGcmWaves - 1) / kGcmWaves, gcm_wgs()))),
                               dim3(kGcmWaves * 64), 0, s, Bt);
        ok = hipGetLastError() == hipSuccess;
    }
    uint64_t status = 0;
    if (ok) {
        if (n) {
            ok = hipMemcpyAsync(out_offsets, ws + o_oo, (nb + 1) * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                 hipMemcpyAsync(&status, ws + o_status, 8, hipMemcpyDeviceToHost, s) == hipSuccess;
        } else if (out_offsets) {
            out_offsets[0] = 0;
        }
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
    }
    if (!ok) return CDC_E_DEVICE;
    return status ? int(int32_t(uint32_t(status))) : CDC_OK;
}

extern "C" uint64_t cdc_encode_bound(uint64_t len, int compress, int encrypt)
{
    const uint64_t f = compress ? 7 + 4 * ((len + kBlockLZ - 1) / kBlockLZ) + len + 8 : len;
    return encrypt ? 60 + f + 28 * ((f + kPiece - 1) / kPiece) : f;
}
