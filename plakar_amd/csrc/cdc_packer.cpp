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

using cdc::Sha256;  // cdc_sha256.cpp

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

}  // extern "C"

namespace cdc {

// Serialize in place for a packfile sink: the index and footer are appended
// to the data section's own buffer (no copy of the blobs), *data / *len then
// hold the packfile until cdc_packer_reset.  The buffer is reserved at MaxSize
// plus one maximal blob so that AddBlob does not reallocate.
int packer_seal(cdc_packer *p, int64_t timestamp, const uint8_t **data, uint64_t *len)
{
    if (!p || !data || !len) return CDC_E_INVALID;
    std::vector<uint8_t> footer;
    serialize_footer(p, timestamp, footer);  // IndexOffset = len(Blobs), before the append
    p->blobs.insert(p->blobs.end(), p->index.begin(), p->index.end());
    p->blobs.insert(p->blobs.end(), footer.begin(), footer.end());
    *data = p->blobs.data();
    *len = p->blobs.size();
    return CDC_OK;
}

void packer_reserve(cdc_packer *p, uint64_t max_blob)
{
    if (!p) return;
    p->blobs.reserve(size_t(p->max_size) + size_t(max_blob) + (1u << 20));
    p->index.reserve(1u << 20);
}

}  // namespace cdc

extern "C" {

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
