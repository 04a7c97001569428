/*
 * C-level test of the boundary the cgo binding uses, called
 * the way Go would call it.  Test infrastructure: links the CPU oracle
 * (oracle/fastcdc_oracle.c) as the checker.  Built by __graft_entry__.build()
 * (plakar_amd/build.py build_ctests) and run by tests/test_abi_c.py on a GPU.
 *
 *   1. cdc_chunker_new with a read callback that hands out ragged pieces
 *      (the (*Chunker).Next contract over an io.Reader), drained with
 *      cdc_chunker_next: plakar's per-file loop, snapshot/backup.go:647-665.
 *   2. cdc_chunk from 8 threads at once, each with its own buffers: the
 *      scanner goroutines of snapshot/backup.go:216-225 calling in parallel.
 *   3. cdc_batch_add_files: files read by the library into its pinned arena,
 *      then one cdc_batch_chunk (the importer, snapshot/importer/fs/fs.go:69-71).
 *   4. cdc_collector_chunk from 8 threads: per-file calls batched for the
 *      device (the scanner fan-out of snapshot/backup.go:216-225).
 *
 * Every result is compared with the oracle; exit status 0 = all identical.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "plakar_cdc.h"

typedef struct oracle_params {
    const uint64_t *gear;
    uint64_t mask_s, mask_l, min_size, normal_size, max_size;
    uint32_t cut_adj;
} oracle_params;
uint64_t oracle_chunk(const oracle_params *P, const uint8_t *data, uint64_t len, uint64_t *offsets,
                      uint32_t *lengths, uint64_t cap);

static uint64_t g_gear[256];
static const cdc_opts g_opts = {65536, 1u << 20, 4u << 20, 0};

static void fill(uint8_t *p, uint64_t n, uint64_t seed)
{
    uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
    for (uint64_t i = 0; i < n; ++i) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        p[i] = (uint8_t)(s >> 24);
    }
    /* a low-entropy stretch in every other buffer: long chunks, MaskL cuts */
    if (seed & 1)
        for (uint64_t i = n / 3; i < n / 3 + n / 4 && i < n; ++i)
            if ((i * 2654435761u) % 97) p[i] = 0;
}

/* oracle cut list of one buffer; returns the count, *off / *len malloc'd */
static uint64_t ref_cuts(const uint8_t *p, uint64_t n, uint64_t **off, uint32_t **len)
{
    oracle_params P = {g_gear, cdc_default_mask_s(), cdc_default_mask_l(), g_opts.min_size, g_opts.normal_size,
                       g_opts.max_size, 0};
    const uint64_t cap = n / g_opts.min_size + 2;
    *off = malloc(cap * 8);
    *len = malloc(cap * 4);
    return oracle_chunk(&P, p, n, *off, *len, cap);
}

/* ---- 1. read callback --------------------------------------------------- */
typedef struct {
    const uint8_t *p;
    uint64_t n, pos, rng;
} reader;

static int64_t read_cb(void *ctx, void *buf, uint64_t cap)
{
    reader *r = ctx;
    if (r->pos >= r->n) return 0;
    r->rng = r->rng * 6364136223846793005ull + 1442695040888963407ull;
    uint64_t k = 1 + (r->rng >> 33) % (3u << 20); /* ragged reads up to 3 MiB */
    if (k > cap) k = cap;
    if (k > r->n - r->pos) k = r->n - r->pos;
    memcpy(buf, r->p + r->pos, k);
    r->pos += k;
    return (int64_t)k;
}

static int test_read_callback(void)
{
    const uint64_t n = (96u << 20) + 12345;
    uint8_t *p = malloc(n);
    fill(p, n, 7);
    reader r = {p, n, 0, 99};
    cdc_chunker *c = NULL;
    int st = cdc_chunker_new("FastCDC", read_cb, &r, &g_opts, &c);
    if (st) {
        fprintf(stderr, "cdc_chunker_new: %s\n", cdc_strerror(st));
        return 1;
    }
    uint64_t *roff;
    uint32_t *rlen;
    const uint64_t nref = ref_cuts(p, n, &roff, &rlen);
    uint64_t k = 0, pos = 0;
    int bad = 0;
    for (;;) {
        const uint8_t *ch;
        uint64_t ln;
        st = cdc_chunker_next(c, &ch, &ln);
        if (st == CDC_EOF) break;
        if (st) {
            fprintf(stderr, "cdc_chunker_next: %s\n", cdc_strerror(st));
            bad = 1;
            break;
        }
        if (k >= nref || roff[k] != pos || rlen[k] != ln || memcmp(ch, p + pos, ln) != 0) {
            fprintf(stderr, "read-callback chunk %llu differs\n", (unsigned long long)k);
            bad = 1;
            break;
        }
        pos += ln;
        ++k;
    }
    if (!bad && (k != nref || pos != n)) {
        fprintf(stderr, "read-callback: %llu chunks vs %llu\n", (unsigned long long)k, (unsigned long long)nref);
        bad = 1;
    }
    cdc_chunker_free(c);
    free(roff);
    free(rlen);
    free(p);
    printf("read callback: %llu chunks over %llu bytes %s\n", (unsigned long long)k, (unsigned long long)n,
           bad ? "MISMATCH" : "identical");
    return bad;
}

/* ---- 2. concurrent cdc_chunk ---------------------------------------------- */
enum { kThreads = 8, kPerThread = 3 };
typedef struct {
    int id, bad;
    uint64_t chunks;
} job;

static void *thread_main(void *arg)
{
    job *j = arg;
    uint64_t lens[kPerThread];
    uint8_t *bufs[kPerThread];
    cdc_buf cb[kPerThread];
    uint64_t cap = 0;
    for (int i = 0; i < kPerThread; ++i) {
        lens[i] = ((uint64_t)(j->id * kPerThread + i) * 7919u % 40u + 1u) << 20;
        lens[i] += (uint64_t)(j->id * 131 + i * 17);
        bufs[i] = malloc(lens[i]);
        fill(bufs[i], lens[i], 1000 + (uint64_t)(j->id * kPerThread + i));
        cb[i].data = bufs[i];
        cb[i].len = lens[i];
        cap += lens[i] / g_opts.min_size + 2;
    }
    cdc_cut *out = malloc(cap * sizeof(cdc_cut));
    uint64_t counts[kPerThread], needed = 0;
    for (int rep = 0; rep < 3 && !j->bad; ++rep) {
        const int st = cdc_chunk(cb, kPerThread, &g_opts, out, cap, counts, &needed);
        if (st) {
            fprintf(stderr, "thread %d: cdc_chunk: %s\n", j->id, cdc_strerror(st));
            j->bad = 1;
            break;
        }
        uint64_t k = 0;
        for (int i = 0; i < kPerThread; ++i) {
            uint64_t *roff;
            uint32_t *rlen;
            const uint64_t nref = ref_cuts(bufs[i], lens[i], &roff, &rlen);
            if (nref != counts[i]) j->bad = 1;
            for (uint64_t q = 0; q < nref && !j->bad; ++q)
                if (out[k + q].offset != roff[q] || out[k + q].length != rlen[q]) j->bad = 1;
            if (j->bad) fprintf(stderr, "thread %d buffer %d differs (rep %d)\n", j->id, i, rep);
            k += counts[i];
            if (rep == 0) j->chunks += counts[i];
            free(roff);
            free(rlen);
        }
    }
    free(out);
    for (int i = 0; i < kPerThread; ++i) free(bufs[i]);
    return NULL;
}

static int test_threads(void)
{
    pthread_t th[kThreads];
    job jobs[kThreads];
    for (int t = 0; t < kThreads; ++t) {
        jobs[t] = (job){t, 0, 0};
        pthread_create(&th[t], NULL, thread_main, &jobs[t]);
    }
    int bad = 0;
    uint64_t chunks = 0;
    for (int t = 0; t < kThreads; ++t) {
        pthread_join(th[t], NULL);
        bad |= jobs[t].bad;
        chunks += jobs[t].chunks;
    }
    printf("%d threads x %d buffers x 3 calls: %llu chunks per pass %s\n", kThreads, kPerThread,
           (unsigned long long)chunks, bad ? "MISMATCH" : "identical");
    return bad;
}

/* ---- 4. collector: per-file calls from 8 threads, batched ------------------- */
static cdc_collector *g_col;

static void *collector_main(void *arg)
{
    job *j = arg;
    for (int i = 0; i < 4 && !j->bad; ++i) {
        const uint64_t n = ((uint64_t)(j->id * 4 + i) * 104729u % 23u) << 20 | (uint64_t)(j->id * 977 + i);
        uint8_t *p = malloc(n + 1);
        fill(p, n, 3000 + (uint64_t)(j->id * 4 + i));
        const uint64_t cap = n / g_opts.min_size + 2;
        cdc_cut *out = malloc(cap * sizeof(cdc_cut));
        uint64_t cnt = 0, *roff;
        uint32_t *rlen;
        const int st = cdc_collector_chunk(g_col, p, n, out, cap, &cnt);
        const uint64_t nref = ref_cuts(p, n, &roff, &rlen);
        j->bad |= st != CDC_OK || cnt != nref;
        for (uint64_t q = 0; q < nref && !j->bad; ++q) j->bad |= out[q].offset != roff[q] || out[q].length != rlen[q];
        if (j->bad) fprintf(stderr, "collector thread %d file %d differs (status %d)\n", j->id, i, st);
        j->chunks += cnt;
        free(out);
        free(roff);
        free(rlen);
        free(p);
    }
    return NULL;
}

static int test_collector(void)
{
    if (cdc_collector_new(&g_opts, 32u << 20, 2000, &g_col) != CDC_OK) return 1;
    pthread_t th[kThreads];
    job jobs[kThreads];
    for (int t = 0; t < kThreads; ++t) {
        jobs[t] = (job){t, 0, 0};
        pthread_create(&th[t], NULL, collector_main, &jobs[t]);
    }
    int bad = 0;
    uint64_t chunks = 0, req = 0, batches = 0;
    for (int t = 0; t < kThreads; ++t) {
        pthread_join(th[t], NULL);
        bad |= jobs[t].bad;
        chunks += jobs[t].chunks;
    }
    cdc_collector_stats(g_col, &req, &batches);
    cdc_collector_free(g_col);
    bad |= req != kThreads * 4 || batches >= req;
    printf("collector: %llu files from %d threads in %llu batches, %llu chunks %s\n", (unsigned long long)req, kThreads,
           (unsigned long long)batches, (unsigned long long)chunks, bad ? "MISMATCH" : "identical");
    return bad;
}

/* ---- 5. collector freed while its callers are still blocked ---------------- */
static void *collector_one(void *arg)
{
    job *j = arg;
    const uint64_t n = ((uint64_t)(j->id % 3 + 1) << 20) + (uint64_t)j->id * 7919u;
    uint8_t *p = malloc(n + 1);
    fill(p, n, 7000 + (uint64_t)j->id);
    const uint64_t cap = n / g_opts.min_size + 2;
    cdc_cut *out = malloc(cap * sizeof(cdc_cut));
    uint64_t cnt = 0, *roff;
    uint32_t *rlen;
    const int st = cdc_collector_chunk(g_col, p, n, out, cap, &cnt);
    const uint64_t nref = ref_cuts(p, n, &roff, &rlen);
    j->bad |= st != CDC_OK || cnt != nref;
    for (uint64_t q = 0; q < nref && !j->bad; ++q) j->bad |= out[q].offset != roff[q] || out[q].length != rlen[q];
    j->chunks = cnt;
    free(out);
    free(roff);
    free(rlen);
    free(p);
    return NULL;
}

static int test_collector_free_while_blocked(void)
{
    enum { kCallers = 6 };
    /* batches close only at 1 GiB, 32 files or after 3 s: the callers stay
     * blocked until cdc_collector_free closes the batch */
    if (cdc_collector_new(&g_opts, 1ull << 30, 3000000u, &g_col) != CDC_OK) return 1;
    pthread_t th[kCallers];
    job jobs[kCallers];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < kCallers; ++t) {
        jobs[t] = (job){t, 0, 0};
        pthread_create(&th[t], NULL, collector_one, &jobs[t]);
    }
    uint64_t req = 0, batches = 0;
    for (int spin = 0; spin < 2000 && req < kCallers; ++spin) {  /* every caller queued (<= 2 s) */
        usleep(1000);
        cdc_collector_stats(g_col, &req, &batches);
    }
    cdc_collector_free(g_col); /* callers still blocked: free drains them, then waits until they left */
    g_col = NULL;
    int bad = req != kCallers;
    for (int t = 0; t < kCallers; ++t) {
        pthread_join(th[t], NULL);
        bad |= jobs[t].bad;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    bad |= el > 2.9; /* free closed the batch instead of waiting out max_wait */
    printf("collector freed with %d blocked callers: %.2f s, %s\n", kCallers, el, bad ? "MISMATCH" : "identical");
    return bad;
}

/* ---- 3. pinned file arena -------------------------------------------------- */
static int test_files(void)
{
    enum { kFiles = 12 };
    char dir[] = "/tmp/cdc_abi_XXXXXX";
    if (!mkdtemp(dir)) return 1;
    char paths[kFiles][64];
    const char *pp[kFiles];
    uint8_t *data[kFiles];
    uint64_t lens[kFiles], total = 0, cap = 0;
    for (int i = 0; i < kFiles; ++i) {
        lens[i] = i == 0 ? 0 : ((uint64_t)(i * 37 % 23) << 20) + (uint64_t)i * 4099u;
        data[i] = malloc(lens[i] + 1);
        fill(data[i], lens[i], 500 + (uint64_t)i);
        snprintf(paths[i], sizeof paths[i], "%s/f%02d", dir, i);
        pp[i] = paths[i];
        FILE *f = fopen(paths[i], "wb");
        if (!f || fwrite(data[i], 1, lens[i], f) != lens[i]) return 1;
        fclose(f);
        total += (lens[i] + 4095) & ~4095ull;
        cap += lens[i] / g_opts.min_size + 2;
    }
    cdc_batch *b = NULL;
    int st = cdc_batch_new(total, &b);
    uint64_t sizes[kFiles];
    if (!st) st = cdc_batch_add_files(b, pp, kFiles, 4, sizes);
    cdc_cut *out = malloc(cap * sizeof(cdc_cut));
    uint64_t counts[kFiles], needed = 0;
    if (!st) st = cdc_batch_chunk(b, &g_opts, out, cap, counts, &needed);
    int bad = st != 0;
    if (st) fprintf(stderr, "cdc_batch: %s\n", cdc_strerror(st));
    uint64_t k = 0, chunks = 0;
    for (int i = 0; i < kFiles && !bad; ++i) {
        uint64_t *roff;
        uint32_t *rlen;
        const uint64_t nref = ref_cuts(data[i], lens[i], &roff, &rlen);
        bad |= sizes[i] != lens[i] || nref != counts[i];
        for (uint64_t q = 0; q < nref && !bad; ++q)
            bad |= out[k + q].offset != roff[q] || out[k + q].length != rlen[q];
        k += counts[i];
        chunks += counts[i];
        free(roff);
        free(rlen);
    }
    /* an arena too small fails cleanly and keeps its earlier buffers */
    cdc_batch *small = NULL;
    if (!bad && cdc_batch_new(1u << 20, &small) == CDC_OK) {
        bad |= cdc_batch_add_files(small, pp + 1, kFiles - 1, 2, NULL) != CDC_E_NOSPACE || cdc_batch_count(small) != 0;
        cdc_batch_free(small);
    }
    cdc_batch_free(b);
    free(out);
    for (int i = 0; i < kFiles; ++i) {
        unlink(paths[i]);
        free(data[i]);
    }
    rmdir(dir);
    printf("file arena: %d files, %llu chunks %s\n", kFiles, (unsigned long long)chunks, bad ? "MISMATCH" : "identical");
    return bad;
}

int main(void)
{
    cdc_default_gear(g_gear);
    int st = cdc_init(0, NULL, 0, 0, 0);
    if (st) {
        fprintf(stderr, "cdc_init: %s\n", cdc_strerror(st));
        return 2;
    }
    if (!cdc_gear_is_placeholder()) return 3;
    int bad = test_read_callback();
    bad |= test_threads();
    bad |= test_files();
    bad |= test_collector();
    bad |= test_collector_free_while_blocked();
    /* re-init with the same device set is accepted; another set is refused */
    bad |= cdc_init(0, NULL, 0, 0, 0) != CDC_OK;
    bad |= cdc_init(1u << 31, NULL, 0, 0, 0) != CDC_E_NO_DEVICE && cdc_device_count() < 32;
    cdc_shutdown();
    printf("%s\n", bad ? "FAIL" : "OK");
    return bad;
}
