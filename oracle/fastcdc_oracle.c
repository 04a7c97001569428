/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libplakar_cdc.so).  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg may use it, and only as
 * the checker / the CPU baseline.
 *
 * Plain-C scalar restatement of plakar's content-defined chunking path:
 *
 *   plakar  snapshot/backup.go:631-666   chunkify routing (empty / < MinSize / CDC)
 *   plakar  repository/repository.go:283-294  (*Repository).Chunker -> NewChunker("fastcdc", ...)
 *   plakar  chunking/chunking.go:10-17   DefaultConfiguration {FASTCDC, 64Ki, 1Mi, 4Mi}
 *   ext     github.com/PlakarKorp/go-cdc-chunkers v0.0.8 (go.mod:37, go.sum:2)
 *             chunker.go        (*Chunker).Next : Peek(MaxSize) -> Algorithm -> Discard(cut)
 *             chunkers/fastcdc  (*FastCDC).Algorithm, Validate, Gear table G
 *
 * PARITY UNPINNED.  The go-cdc-chunkers module is a third-party dependency that
 * is NOT present under /root/reference (no vendor/, no module cache, no Go
 * toolchain in the build container: SURVEY.md §8c).  Its algorithm is restated
 * here from the published FastCDC algorithm (Xia et al., USENIX ATC'16, Alg. 1
 * with normalised chunking) as go-cdc-chunkers v0.0.8 implements it:
 *
 *   if n <= Min: return n ; elif n >= Max: n = Max ; elif n <= Normal: Normal = n
 *   fp = 0 ; i = Min
 *   for ; i < Normal ; i++ { fp = (fp << 1) + G[data[i]] ; if fp & MaskS == 0 { return i } }
 *   for ; i < n      ; i++ { fp = (fp << 1) + G[data[i]] ; if fp & MaskL == 0 { return i } }
 *   return i
 *
 * Items that could not be verified against the v0.0.8 source are RUNTIME
 * PARAMETERS here (and in the product), so the exact constants can be dropped
 * in without touching code: the 256-entry Gear table, MaskS / MaskL (default
 * the paper's 0x0003590703530000 / 0x0000d90003530000) and the cut convention
 * (return i, cut_adj = 0; or i + 1, cut_adj = 1).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct oracle_params {
    const uint64_t *gear; /* 256 entries */
    uint64_t mask_s;
    uint64_t mask_l;
    uint64_t min_size;
    uint64_t normal_size;
    uint64_t max_size;
    uint32_t cut_adj; /* 0: cut at i (chunk = data[:i]); 1: cut at i + 1 */
} oracle_params;

/* go-cdc-chunkers chunkers/fastcdc (*FastCDC).Validate (expected bounds:
 * 64 B <= sizes <= 1 GiB, Min < Normal < Max).  0 = ok, -1/-2/-3 = which
 * size is invalid (Normal, Min, Max in the order the module checks them). */
int oracle_fastcdc_validate(uint64_t min_size, uint64_t normal_size, uint64_t max_size)
{
    const uint64_t lo = 64, hi = 1024ull * 1024ull * 1024ull;
    if (normal_size < lo || normal_size > hi) return -1;
    if (min_size < lo || min_size > hi || min_size >= normal_size) return -2;
    if (max_size < lo || max_size > hi || max_size <= normal_size) return -3;
    return 0;
}

/* (*FastCDC).Algorithm(opts, data, n) -> cut point (chunk length). */
uint64_t oracle_fastcdc_algorithm(const oracle_params *P, const uint8_t *data, uint64_t n)
{
    uint64_t min_size = P->min_size, max_size = P->max_size, normal_size = P->normal_size;
    if (n <= min_size)
        return n;
    else if (n >= max_size)
        n = max_size;
    else if (n <= normal_size)
        normal_size = n;

    uint64_t fp = 0;
    uint64_t i = min_size;
    for (; i < normal_size; i++) {
        fp = (fp << 1) + P->gear[data[i]];
        if ((fp & P->mask_s) == 0) return i + P->cut_adj;
    }
    for (; i < n; i++) {
        fp = (fp << 1) + P->gear[data[i]];
        if ((fp & P->mask_l) == 0) return i + P->cut_adj;
    }
    return i;
}

/* Drain (*Chunker).Next() over an in-memory stream: each call peeks
 * min(remaining, MaxSize) bytes, cuts, discards.  Writes up to `cap` chunk
 * records and returns the total number of chunks. */
uint64_t oracle_chunk(const oracle_params *P, const uint8_t *data, uint64_t len,
                      uint64_t *offsets, uint32_t *lengths, uint64_t cap)
{
    uint64_t p = 0, k = 0;
    while (p < len) {
        uint64_t n = len - p;
        if (n > P->max_size) n = P->max_size; /* bufio.Reader.Peek(MaxSize) */
        uint64_t cut = oracle_fastcdc_algorithm(P, data + p, n);
        if (k < cap) {
            if (offsets) offsets[k] = p;
            if (lengths) lengths[k] = (uint32_t)cut;
        }
        k++;
        p += cut; /* bufio.Reader.Discard(cut) */
    }
    return k;
}

/* snapshot/backup.go:631-666 chunkify routing: an empty file yields one empty
 * chunk, a file smaller than MinSize one whole-file chunk (no CDC), anything
 * else goes through the chunker. */
uint64_t oracle_chunkify(const oracle_params *P, const uint8_t *data, uint64_t len,
                         uint64_t *offsets, uint32_t *lengths, uint64_t cap)
{
    if (len == 0 || len < P->min_size) {
        if (cap > 0) {
            if (offsets) offsets[0] = 0;
            if (lengths) lengths[0] = (uint32_t)len;
        }
        return 1;
    }
    return oracle_chunk(P, data, len, offsets, lengths, cap);
}

/* Number of bytes the sequential algorithm actually hashes (Σ over chunks of
 * the positions [start+Min, cut) it visits).  Used to report the work the CPU
 * reference does, next to the input size. */
uint64_t oracle_hashed_bytes(const oracle_params *P, const uint32_t *lengths, uint64_t nchunks)
{
    uint64_t s = 0;
    for (uint64_t k = 0; k < nchunks; k++) {
        uint64_t L = lengths[k];
        if (L > P->min_size) s += L - P->min_size;
    }
    return s;
}
