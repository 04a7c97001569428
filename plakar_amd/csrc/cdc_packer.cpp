// Packfile builder: the consumer of the cut lists (plakar snapshot/packer.go,
// packfile/packfile.go).  Host-side, native: chunk bytes are appended to the
// packfile's data section, the index and footer are serialised exactly as
// packfile.go writes them (little-endian binary.Write of each field), and the
// index checksum is SHA-256 over the index bytes (packfile.go:247-275).
//
//   packfile.New / AddBlob        packfile/packfile.go:140-150, 389-394
//   (*PackFile).Serialize         packfile/packfile.go:241-294
//   SerializeData/Index/Footer    packfile/packfile.go:296-387
//   Packer.AddBlob / Size         snapshot/packer.go:21-31
//   PutPackfile layout            snapshot/snapshot.go:232-267 (data, Encode(index),
//                                 Encode(footer), version u32, u8 footer length)
//   packerJob flush rule          snapshot/snapshot.go:71 (Size() > MaxSize)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "cdc_internal.h"

namespace {

// ---- SHA-256 (FIPS 180-4), for the index checksum -------------------------
struct Sha256 {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint8_t buf[64];
    uint64_t total = 0;
    size_t fill = 0;

    static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

    void block(const uint8_t *p)
    {
        static const uint32_t K[64] = {
            0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
            0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
            0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
            0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
            0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
            0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
            0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
            0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
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
            const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
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

    void update(const uint8_t *p, size_t n)
    {
        total += n;
        while (n) {
            const size_t k = std::min(n, size_t(64) - fill);
            std::memcpy(buf + fill, p, k);
            fill += k;
            p += k;
            n -= k;
            if (fill == 64) {
                block(buf);
                fill = 0;
            }
        }
    }

    void final(uint8_t out[32])
    {
        const uint64_t bits = total * 8;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while (fill != 56) update(&zero, 1);
        uint8_t len[8];
        for (int i = 0; i < 8; ++i) len[i] = uint8_t(bits >> (56 - 8 * i));
        update(len, 8);
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 4; ++j) out[4 * i + j] = uint8_t(h[i] >> (24 - 8 * j));
    }
};

template <typename T>
void put_le(std::vector<uint8_t> &v, T x)
{
    for (size_t i = 0; i < sizeof(T); ++i) v.push_back(uint8_t(uint64_t(x) >> (8 * i)));
}

constexpr uint32_t kPackVersion = 100;        // packfile.VERSION (packfile/packfile.go:12)
constexpr size_t kIndexEntry = 1 + 32 + 4 + 4;  // Type, Checksum, Offset, Length
constexpr size_t kFooterBytes = 4 + 8 + 4 + 4 + 32;

}  // namespace

struct cdc_packer {
    uint32_t max_size = 0;
    std::vector<uint8_t> blobs;  // PackFile.Blobs
    std::vector<uint8_t> index;  // PackFile.Index, already in its serialised form (41 B per blob)
    uint32_t count = 0;          // Footer.Count
};

static void serialize_footer(const cdc_packer *p, int64_t timestamp, std::vector<uint8_t> &out)
{
    Sha256 h;
    h.update(p->index.data(), p->index.size());
    uint8_t sum[32];
    h.final(sum);
    put_le<uint32_t>(out, kPackVersion);
    put_le<int64_t>(out, timestamp);
    put_le<uint32_t>(out, p->count);
    put_le<uint32_t>(out, uint32_t(p->blobs.size()));  // Footer.IndexOffset = len(Blobs)
    out.insert(out.end(), sum, sum + 32);
}

extern "C" {

int cdc_packer_new(uint32_t max_size, cdc_packer **out)
{
    if (!out) return CDC_E_INVALID;
    auto *p = new cdc_packer();
    p->max_size = max_size ? max_size : (20u << 20);  // packfile.DefaultConfiguration().MaxSize
    *out = p;
    return CDC_OK;
}

// Packer.AddBlob: returns 1 when Size() > MaxSize (the caller flushes, as
// packerJob does), 0 otherwise.
int cdc_packer_add_blob(cdc_packer *p, uint8_t type, const uint8_t checksum[32], const uint8_t *data, uint64_t len)
{
    if (!p || !checksum || (len && !data) || len > 0xFFFFFFFFull || p->blobs.size() + len > 0xFFFFFFFFull)
        return CDC_E_INVALID;
    const uint32_t off = uint32_t(p->blobs.size());
    p->index.push_back(type);
    p->index.insert(p->index.end(), checksum, checksum + 32);
    put_le<uint32_t>(p->index, off);
    put_le<uint32_t>(p->index, uint32_t(len));
    p->blobs.insert(p->blobs.end(), data, data + len);
    ++p->count;
    return p->blobs.size() > p->max_size ? 1 : 0;
}

// Chunk blobs of one buffer from its cut list: cuts[i] of `base` with digest
// digests[32 i], skipping rows whose `skip` byte is non-zero (already stored:
// BlobExists, snapshot/backup.go:625).  Stops after the blob that makes the
// packfile exceed MaxSize; returns the number of cut rows consumed (skipped
// ones included), or a negative status.
int64_t cdc_packer_add_chunks(cdc_packer *p, const uint8_t *base, const cdc_cut *cuts, uint64_t n,
                              const uint8_t *digests, const uint8_t *skip)
{
    if (!p || (n && (!cuts || !digests))) return CDC_E_INVALID;
    for (uint64_t i = 0; i < n; ++i) {
        if (skip && skip[i]) continue;
        const int st = cdc_packer_add_blob(p, 1 /* TYPE_CHUNK */, digests + 32 * i, base + cuts[i].offset,
                                           cuts[i].length);
        if (st < 0) return st;
        if (st == 1) return int64_t(i + 1);
    }
    return int64_t(n);
}

uint64_t cdc_packer_size(const cdc_packer *p) { return p ? p->blobs.size() : 0; }
uint32_t cdc_packer_count(const cdc_packer *p) { return p ? p->count : 0; }

// (*PackFile).Serialize: Blobs, index, footer (timestamp = Footer.Timestamp,
// time.Now().UnixNano() in packfile.New).  Returns CDC_E_NOSPACE with *len
// set when cap is too small.
int cdc_packer_serialize(const cdc_packer *p, int64_t timestamp, uint8_t *out, uint64_t cap, uint64_t *len)
{
    if (!p || !len) return CDC_E_INVALID;
    std::vector<uint8_t> footer;
    serialize_footer(p, timestamp, footer);
    const uint64_t n = p->blobs.size() + p->index.size() + footer.size();
    *len = n;
    if (n > cap || !out) return CDC_E_NOSPACE;
    std::memcpy(out, p->blobs.data(), p->blobs.size());
    std::memcpy(out + p->blobs.size(), p->index.data(), p->index.size());
    std::memcpy(out + p->blobs.size() + p->index.size(), footer.data(), footer.size());
    return CDC_OK;
}

// SerializeData / SerializeIndex / SerializeFooter, for PutPackfile's layout
// (the index and footer are then Encode'd by the caller).  part: 0 data,
// 1 index, 2 footer.
int cdc_packer_serialize_part(const cdc_packer *p, int part, int64_t timestamp, uint8_t *out, uint64_t cap,
                              uint64_t *len)
{
    if (!p || !len || part < 0 || part > 2) return CDC_E_INVALID;
    std::vector<uint8_t> footer;
    const uint8_t *src = nullptr;
    if (part == 0) {
        src = p->blobs.data();
        *len = p->blobs.size();
    } else if (part == 1) {
        src = p->index.data();
        *len = p->index.size();
    } else {
        serialize_footer(p, timestamp, footer);
        src = footer.data();
        *len = footer.size();
    }
    if (*len > cap || (*len && !out)) return CDC_E_NOSPACE;
    if (*len) std::memcpy(out, src, *len);
    return CDC_OK;
}

void cdc_packer_reset(cdc_packer *p)
{
    if (!p) return;
    p->blobs.clear();
    p->index.clear();
    p->count = 0;
}

void cdc_packer_free(cdc_packer *p) { delete p; }

}  // extern "C"

static_assert(kIndexEntry == 41 && kFooterBytes == 52, "packfile.go record sizes");
