// Host SHA-256 (FIPS 180-4) for the library's host-side consumers: the
// packfile index checksum (packfile/packfile.go:247-275) and the per-object
// checksum of the backup pipeline (objectHasher over the whole file,
// snapshot/backup.go:583-609, hashing/hashing.go:31-36).  Both are one serial
// chain per message, so they run on host cores: x86 SHA extensions when the
// CPU has them (runtime dispatch), a portable scalar block function otherwise.
#include <cstdint>
#include <cstring>

// hipcc also parses this file for the device; the SHA-extension path is
// host x86 code only.
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#define CDC_SHA_NI 1
#include <immintrin.h>
#else
#define CDC_SHA_NI 0
#endif

#include "cdc_internal.h"

namespace cdc {
namespace {

alignas(16) const uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void blocks_scalar(uint32_t h[8], const uint8_t *p, size_t nblocks)
{
    for (; nblocks; --nblocks, p += 64) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = uint32_t(p[4 * i]) << 24 | uint32_t(p[4 * i + 1]) << 16 | uint32_t(p[4 * i + 2]) << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
            const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g;
            g = f;
            f = e;
            e = d + t1;
            d = c;
            c = b;
            b = a;
            a = t1 + t2;
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
}

#if CDC_SHA_NI
// SHA extensions: the state as (A,B,E,F) and (C,D,G,H) lanes, four rounds
// per message group (two SHA256RNDS2), the schedule by SHA256MSG1/MSG2.
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_ni(uint32_t h[8], const uint8_t *p, size_t nblocks)
{
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i *>(h));        // h3 h2 h1 h0
    __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(h + 4));   // h7 h6 h5 h4
    t = _mm_shuffle_epi32(t, 0xB1);                                            // CDAB
    s1 = _mm_shuffle_epi32(s1, 0x1B);                                          // EFGH
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                    // ABEF
    s1 = _mm_blend_epi16(s1, t, 0xF0);                                         // CDGH
    for (; nblocks; --nblocks, p += 64) {
        const __m128i save0 = s0, save1 = s1;
        __m128i m[4];
        for (int g = 0; g < 16; ++g) {
            __m128i msg;
            if (g < 4) {
                msg = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * g)), bswap);
            } else {
                const __m128i a = _mm_sha256msg1_epu32(m[(g - 4) & 3], m[(g - 3) & 3]);
                const __m128i b = _mm_add_epi32(a, _mm_alignr_epi8(m[(g - 1) & 3], m[(g - 2) & 3], 4));
                msg = _mm_sha256msg2_epu32(b, m[(g - 1) & 3]);
            }
            m[g & 3] = msg;
            __m128i wk = _mm_add_epi32(msg, _mm_load_si128(reinterpret_cast<const __m128i *>(kK + 4 * g)));
            s1 = _mm_sha256rnds2_epu32(s1, s0, wk);
            wk = _mm_shuffle_epi32(wk, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, wk);
        }
        s0 = _mm_add_epi32(s0, save0);
        s1 = _mm_add_epi32(s1, save1);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);         // FEBA
    s1 = _mm_shuffle_epi32(s1, 0xB1);        // DCHG
    s0 = _mm_blend_epi16(t, s1, 0xF0);       // DCBA
    s1 = _mm_alignr_epi8(s1, t, 8);          // HGFE
    _mm_storeu_si128(reinterpret_cast<__m128i *>(h), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i *>(h + 4), s1);
}

bool have_sha_ni()
{
    static const bool ok = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("ssse3");
    }();
    return ok;
}
#else
bool have_sha_ni() { return false; }
void blocks_ni(uint32_t *, const uint8_t *, size_t) {}
#endif

}  // namespace

void Sha256::blocks(const uint8_t *p, size_t nblocks)
{
    if (!nblocks) return;
    if (have_sha_ni() && !force_scalar) blocks_ni(h, p, nblocks);
    else blocks_scalar(h, p, nblocks);
}

void Sha256::update(const uint8_t *p, size_t n)
{
    total += n;
    if (fill) {
        const size_t k = n < 64 - fill ? n : 64 - fill;
        std::memcpy(buf + fill, p, k);
        fill += k;
        p += k;
        n -= k;
        if (fill < 64) return;
        blocks(buf, 1);
        fill = 0;
    }
    blocks(p, n / 64);
    p += n / 64 * 64;
    n %= 64;
    if (n) std::memcpy(buf, p, n);
    fill = n;
}

void Sha256::final(uint8_t out[32])
{
    const uint64_t bits = total * 8;
    buf[fill++] = 0x80;
    if (fill > 56) {
        std::memset(buf + fill, 0, 64 - fill);
        blocks(buf, 1);
        fill = 0;
    }
    std::memset(buf + fill, 0, 56 - fill);
    for (int i = 0; i < 8; ++i) buf[56 + i] = uint8_t(bits >> (56 - 8 * i));
    blocks(buf, 1);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = uint8_t(h[i] >> (24 - 8 * j));
}

void sha256(const void *data, size_t n, uint8_t out[32], bool force_scalar)
{
    Sha256 s;
    s.force_scalar = force_scalar;
    s.update(static_cast<const uint8_t *>(data), n);
    s.final(out);
}

bool sha256_accelerated() { return have_sha_ni(); }

}  // namespace cdc

extern "C" int cdc_sha256(const void *data, uint64_t len, int force_scalar, uint8_t out[32])
{
    if ((!data && len) || !out) return CDC_E_INVALID;
    cdc::sha256(data, size_t(len), out, force_scalar != 0);
    return CDC_OK;
}

extern "C" int cdc_sha256_accelerated(void) { return cdc::sha256_accelerated() ? 1 : 0; }
