/*
 * ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded
 * by, or called from the product library (libplakar_cdc.so).  Only bench.py's
 * cpu_baseline leg of the `c4b` workload (and tests/) load it.
 *
 * The whole backup leg on host cores, the work the reference does per file
 * (one goroutine per file, snapshot/backup.go:216-225) restated in C with the
 * same libraries' algorithms:
 *
 *   snapshot/importer/fs/fs.go:69-71   the file's bytes (pread)
 *   snapshot/backup.go:583, 668-681    object SHA-256 over the whole file
 *   snapshot/backup.go:631-666         chunkify routing + the chunker's Next()
 *                                      loop (oracle_chunkify, fastcdc_oracle.c)
 *   snapshot/backup.go:594-629         processChunk: chunk SHA-256, the byte
 *                                      histogram and entropy() (548-569),
 *                                      BlobExists (the run's own set)
 *   snapshot/blobs.go:9-24,            PutBlob -> Encode: LZ4 frame
 *   repository/repository.go:212-236   (compression/compression.go:94-106:
 *                                      4-MiB independent blocks, content
 *                                      checksum) then the AES-256-GCM stream
 *                                      (encryption/symmetric.go:72-163: a
 *                                      sealed 32-byte subkey, then 64-KiB
 *                                      pieces, each nonce || Seal)
 *   snapshot/snapshot.go:51-92,        packerJob: the blob appended to the
 *   packfile/packfile.go:241-294       worker's packfile with its 41-byte index
 *                                      entry; at Size() > MaxSize the footer
 *                                      (SHA-256 of the index) and a flush
 *
 * Libraries: OpenSSL libcrypto (SHA-256, AES-256-GCM; the reference uses Go's
 * crypto/sha256 and crypto/aes + cipher.GCM) and the system liblz4 frame API
 * (the reference uses github.com/pierrec/lz4/v4).  Each worker thread takes the
 * next file and does all of its work (the reference's NumCPU packer
 * goroutines are folded into the file workers: the same per-blob work).
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <math.h>
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

typedef struct oracle_params {
    const uint64_t *gear;
    uint64_t mask_s, mask_l, min_size, normal_size, max_size;
    uint32_t cut_adj;
} oracle_params;
uint64_t oracle_chunkify(const oracle_params *P, const uint8_t *data, uint64_t len, uint64_t *offsets,
                         uint32_t *lengths, uint64_t cap);

/* liblz4 frame API (lz4frame.h, v1.9: the header is not installed in this
 * image; the structure layout below is the library's stable public one). */
typedef struct {
    int blockSizeID, blockMode, contentChecksumFlag, frameType;
    unsigned long long contentSize;
    unsigned dictID;
    int blockChecksumFlag;
} lz4f_frame_info;
typedef struct {
    lz4f_frame_info frameInfo;
    int compressionLevel;
    unsigned autoFlush, favorDecSpeed, reserved[3];
} lz4f_prefs;
size_t LZ4F_compressFrameBound(size_t srcSize, const lz4f_prefs *prefs);
size_t LZ4F_compressFrame(void *dst, size_t cap, const void *src, size_t n, const lz4f_prefs *prefs);
unsigned LZ4F_isError(size_t code);

typedef struct backup_cpu_stats {
    uint64_t files, bytes, chunks, new_blobs, encoded_bytes, packfiles, packed_bytes, failed_files;
    double wall_s;
} backup_cpu_stats;

/* The run's dedup set (BlobExists): open addressing on the first 8 digest bytes. */
typedef struct {
    uint8_t *keys; /* 32 B per slot, all-zero = empty */
    uint8_t *used;
    uint64_t cap;
    pthread_mutex_t mu;
} digest_set;

static int set_insert(digest_set *S, const uint8_t d[32])
{
    uint64_t h;
    memcpy(&h, d, 8);
    pthread_mutex_lock(&S->mu);
    for (uint64_t i = h & (S->cap - 1);; i = (i + 1) & (S->cap - 1)) {
        if (!S->used[i]) {
            S->used[i] = 1;
            memcpy(S->keys + 32 * i, d, 32);
            pthread_mutex_unlock(&S->mu);
            return 1;
        }
        if (memcmp(S->keys + 32 * i, d, 32) == 0) {
            pthread_mutex_unlock(&S->mu);
            return 0;
        }
    }
}

typedef struct {
    const char *const *paths;
    int n;
    const oracle_params *P;
    const uint8_t *key;
    int compress;
    uint64_t packfile_max;
    digest_set set;
    int next;
    pthread_mutex_t mu;
    backup_cpu_stats st;
} job;

typedef struct {
    uint8_t *data, *index;
    uint64_t dlen, dcap, ilen, icap;
    uint32_t count;
} packfile;

static void grow(uint8_t **p, uint64_t *cap, uint64_t need)
{
    if (need <= *cap) return;
    uint64_t c = *cap ? *cap : 1 << 20;
    while (c < need) c *= 2;
    *p = (uint8_t *)realloc(*p, c);
    *cap = c;
}

/* (*PackFile).Serialize's footer + PutPackfile, minus the storage write. */
static uint64_t pack_flush(packfile *pk)
{
    uint8_t sum[32];
    SHA256(pk->index, pk->ilen, sum);
    const uint64_t total = pk->dlen + pk->ilen + 52;
    pk->dlen = pk->ilen = 0;
    pk->count = 0;
    (void)sum;
    return total;
}

/* Go's entropy() (snapshot/backup.go:548-569) over a 256-bin histogram. */
static double entropy(const uint32_t *h, uint64_t n)
{
    if (!n) return 0.0;
    double e = 0.0;
    for (int b = 0; b < 256; b++)
        if (h[b]) {
            const double p = (double)h[b] / (double)n;
            e -= p * log2(p);
        }
    return e;
}

/* GCM Seal of one piece: ciphertext || tag into out. */
static int seal(EVP_CIPHER_CTX *c, const uint8_t *key, const uint8_t *nonce, const uint8_t *in, int n, uint8_t *out)
{
    int ol = 0, fl = 0;
    if (EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, key, nonce) != 1) return -1;
    if (EVP_EncryptUpdate(c, out, &ol, in, n) != 1) return -1;
    if (EVP_EncryptFinal_ex(c, out + ol, &fl) != 1) return -1;
    return EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out + ol + fl) == 1 ? 0 : -1;
}

static void *worker(void *arg)
{
    job *J = (job *)arg;
    const oracle_params *P = J->P;
    EVP_CIPHER_CTX *cx = EVP_CIPHER_CTX_new();
    lz4f_prefs pr;
    memset(&pr, 0, sizeof(pr));
    pr.frameInfo.blockSizeID = 7;         /* LZ4F_max4MB */
    pr.frameInfo.blockMode = 1;           /* LZ4F_blockIndependent */
    pr.frameInfo.contentChecksumFlag = 1; /* LZ4F_contentChecksumEnabled */
    const size_t fb = LZ4F_compressFrameBound(P->max_size, &pr);
    uint8_t *frame = (uint8_t *)malloc(fb + 64);
    uint8_t *enc = (uint8_t *)malloc(fb + 64 + (fb / 65536 + 2) * 28 + 60);
    uint8_t *buf = NULL;
    uint64_t bcap = 0;
    uint64_t *offs = NULL;
    uint32_t *lens = NULL;
    uint64_t ccap = 0;
    packfile pk;
    memset(&pk, 0, sizeof(pk));
    backup_cpu_stats st;
    memset(&st, 0, sizeof(st));
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const int i = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (i >= J->n) break;
        st.files++;
        struct stat sb;
        const int fd = open(J->paths[i], O_RDONLY | O_CLOEXEC);
        if (fd < 0 || fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
            if (fd >= 0) close(fd);
            st.failed_files++;
            continue;
        }
        const uint64_t len = (uint64_t)sb.st_size;
        grow(&buf, &bcap, len + 1);
        uint64_t got = 0;
        while (got < len) {
            const ssize_t k = pread(fd, buf + got, len - got, (off_t)got);
            if (k <= 0) break;
            got += (uint64_t)k;
        }
        close(fd);
        if (got != len) {
            st.failed_files++;
            continue;
        }
        uint8_t obj[32];
        SHA256(buf, len, obj); /* the object checksum */
        const uint64_t need = len / P->min_size + 2;
        if (need > ccap) {
            ccap = need;
            offs = (uint64_t *)realloc(offs, ccap * 8);
            lens = (uint32_t *)realloc(lens, ccap * 4);
        }
        const uint64_t nc = oracle_chunkify(P, buf, len, offs, lens, ccap);
        st.chunks += nc;
        st.bytes += len;
        for (uint64_t q = 0; q < nc; q++) {
            const uint8_t *c = buf + offs[q];
            const uint64_t n = lens[q];
            uint8_t d[32];
            SHA256(c, n, d);
            uint32_t h[256];
            memset(h, 0, sizeof(h));
            for (uint64_t x = 0; x < n; x++) h[c[x]]++;
            volatile double e = entropy(h, n);
            (void)e;
            if (!set_insert(&J->set, d)) continue; /* BlobExists */
            st.new_blobs++;
            const uint8_t *src = c;
            uint64_t m = n;
            if (J->compress && n) {
                const size_t r = LZ4F_compressFrame(frame, fb + 64, c, n, &pr);
                if (LZ4F_isError(r)) continue;
                src = frame;
                m = r;
            }
            uint64_t elen = m;
            const uint8_t *blob = src;
            if (J->key) { /* subkey header, then 64-KiB pieces */
                uint8_t sub[32], sn[12], dn[12];
                RAND_bytes(sub, 32);
                RAND_bytes(sn, 12);
                RAND_bytes(dn, 12);
                memcpy(enc, sn, 12);
                seal(cx, J->key, sn, sub, 32, enc + 12);
                uint64_t o = 60;
                for (uint64_t p0 = 0, k = 0; p0 < m; p0 += 65536, k++) {
                    uint8_t nn[12];
                    memcpy(nn, dn, 12);
                    nn[8] ^= (uint8_t)(k >> 24);
                    nn[9] ^= (uint8_t)(k >> 16);
                    nn[10] ^= (uint8_t)(k >> 8);
                    nn[11] ^= (uint8_t)k;
                    const int pn = (int)(m - p0 < 65536 ? m - p0 : 65536);
                    memcpy(enc + o, nn, 12);
                    seal(cx, sub, nn, src + p0, pn, enc + o + 12);
                    o += 12 + (uint64_t)pn + 16;
                }
                elen = o;
                blob = enc;
            }
            st.encoded_bytes += elen;
            /* Packer.AddBlob: data, then {type, checksum, offset, length} */
            grow(&pk.data, &pk.dcap, pk.dlen + elen);
            memcpy(pk.data + pk.dlen, blob, elen);
            grow(&pk.index, &pk.icap, pk.ilen + 41);
            uint8_t *ix = pk.index + pk.ilen;
            ix[0] = 1;
            memcpy(ix + 1, d, 32);
            const uint32_t off32 = (uint32_t)pk.dlen, len32 = (uint32_t)elen;
            memcpy(ix + 33, &off32, 4);
            memcpy(ix + 37, &len32, 4);
            pk.ilen += 41;
            pk.dlen += elen;
            pk.count++;
            if (pk.dlen + pk.ilen + 52 > J->packfile_max) { /* Size() > MaxSize: flush */
                st.packed_bytes += pack_flush(&pk);
                st.packfiles++;
            }
        }
    }
    if (pk.count) {
        st.packed_bytes += pack_flush(&pk);
        st.packfiles++;
    }
    pthread_mutex_lock(&J->mu);
    J->st.files += st.files;
    J->st.bytes += st.bytes;
    J->st.chunks += st.chunks;
    J->st.new_blobs += st.new_blobs;
    J->st.encoded_bytes += st.encoded_bytes;
    J->st.packfiles += st.packfiles;
    J->st.packed_bytes += st.packed_bytes;
    J->st.failed_files += st.failed_files;
    pthread_mutex_unlock(&J->mu);
    EVP_CIPHER_CTX_free(cx);
    free(frame);
    free(enc);
    free(buf);
    free(offs);
    free(lens);
    free(pk.data);
    free(pk.index);
    return NULL;
}

/* One backup of `n` files with `threads` workers.  key: 32 bytes or NULL. */
int backup_cpu_run(const char *const *paths, int n, int threads, const oracle_params *P, const uint8_t *key,
                   int compress, uint64_t packfile_max, backup_cpu_stats *out)
{
    job J;
    memset(&J, 0, sizeof(J));
    J.paths = paths;
    J.n = n;
    J.P = P;
    J.key = key;
    J.compress = compress;
    J.packfile_max = packfile_max ? packfile_max : (20u << 20);
    uint64_t cap = 1 << 16;
    for (int i = 0; i < n; i++) {
        struct stat sb;
        if (stat(paths[i], &sb) == 0) cap += (uint64_t)sb.st_size / (P->min_size ? P->min_size : 1) + 2;
    }
    uint64_t c2 = 1;
    while (c2 < 2 * cap) c2 <<= 1;
    J.set.cap = c2;
    J.set.keys = (uint8_t *)malloc(32 * c2);
    J.set.used = (uint8_t *)calloc(c2, 1);
    if (!J.set.keys || !J.set.used) return -1;
    pthread_mutex_init(&J.set.mu, NULL);
    pthread_mutex_init(&J.mu, NULL);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    J.st.wall_s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    free(th);
    free(J.set.keys);
    free(J.set.used);
    if (out) *out = J.st;
    return 0;
}
