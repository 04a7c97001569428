/*
 * plakar_cdc.h — C ABI of the MI355X content-defined chunker (libplakar_cdc.so).
 *
 * Drop-in boundary for plakar's chunking path.  Every entry point below names
 * the reference interface it replaces.  Reference paths are relative to the
 * plakar tree; "ext" marks the third-party Go module
 * github.com/PlakarKorp/go-cdc-chunkers v0.0.8 (go.mod:37), whose source is not
 * vendored in the reference.
 *
 * Plain C types only: no HIP or torch types appear in any signature.  Device
 * pointers are `void *`, and HIP streams are passed as `void *` (a hipStream_t,
 * or NULL for the null stream).  No call throws.  Every call returns an int
 * status: CDC_OK / CDC_EOF / CDC_NEED_DATA (>= 0) or a negative CDC_E_* code.
 * cdc_strerror() turns a status into text.
 *
 * The product never falls back to the CPU.  If no GPU is present, or the HIP
 * runtime fails, calls return CDC_E_DEVICE / CDC_E_NO_DEVICE.
 */
#ifndef PLAKAR_CDC_H
#define PLAKAR_CDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CDC_ABI_VERSION 1

/* ---- status codes --------------------------------------------------------- */
#define CDC_OK 0
#define CDC_EOF 1           /* io.EOF: the stream is drained (Next() returned its last chunk) */
#define CDC_NEED_DATA 2     /* streaming: append more bytes (or mark EOF) before the next chunk */
#define CDC_E_INVALID (-1)  /* bad argument (NULL pointer, bad length, misaligned, ...) */
#define CDC_E_UNSUPPORTED (-2) /* algorithm not implemented here (e.g. "ultracdc") */
#define CDC_E_NOSPACE (-3)  /* output array too small; the needed count is reported */
#define CDC_E_DEVICE (-4)   /* HIP runtime / kernel failure */
#define CDC_E_NOMEM (-5)    /* host or device allocation failed */
#define CDC_E_NORMAL_SIZE (-6) /* ext fastcdc ErrNormalSize */
#define CDC_E_MIN_SIZE (-7)    /* ext fastcdc ErrMinSize */
#define CDC_E_MAX_SIZE (-8)    /* ext fastcdc ErrMaxSize */
#define CDC_E_IO (-9)       /* a reader callback reported an error */
#define CDC_E_NOT_INIT (-10) /* cdc_init() has not been called */
#define CDC_E_NO_DEVICE (-11) /* no HIP device visible */

/* ---- data types -------------------------------------------------------------- */

/* chunkers.ChunkerOpts (ext chunker.go; used at repository/repository.go:288-292,
 * chunking/chunking_test.go:19-23).  Sizes in bytes. */
typedef struct cdc_opts {
    uint32_t min_size;
    uint32_t normal_size;
    uint32_t max_size;
    uint32_t reserved; /* must be 0 */
} cdc_opts;

/* One chunk: [offset, offset + length) of its buffer.  plakar stores only the
 * length (objects.Chunk.Length, objects/objects.go:73-79); the offsets are the
 * prefix sums the VFS walks (snapshot/vfs/vfilep.go:30-49). */
typedef struct cdc_cut {
    uint64_t offset;
    uint32_t length;
    uint32_t reserved;
} cdc_cut;

/* An independent input buffer (one file, or a window of one). */
typedef struct cdc_buf {
    const void *data;
    uint64_t len;
} cdc_buf;

/* Device-side result block, written by the device path.  Read it after the
 * stream has been synchronised. */
typedef struct cdc_result {
    uint64_t ncuts;    /* chunks written (final chunk included when final != 0) */
    uint64_t consumed; /* bytes covered by the written chunks (== len when final) */
    int64_t status;    /* CDC_OK, or CDC_E_NOSPACE */
    uint64_t needed;   /* chunks needed when status == CDC_E_NOSPACE */
} cdc_result;

/* ---- library setup ------------------------------------------------------------ */

/* Initialise the library on the devices in dev_mask (bit i = HIP device i;
 * 0 = every visible device).  gear = 256-entry Gear table of
 * ext chunkers/fastcdc (the package-level G), or NULL for the built-in
 * placeholder table (see cdc_default_gear).  mask_s / mask_l = the FastCDC
 * small/large masks (0 selects the defaults 0x0003590703530000 /
 * 0x0000d90003530000).  cut_convention: 0 = Algorithm returns i (the chunk
 * excludes the byte whose fingerprint matched), 1 = returns i + 1.
 * May be called again to change the parameters: it waits for the devices to
 * go idle first, and must not race with other calls.  A different device set
 * returns CDC_E_INVALID (call cdc_shutdown() first).  A failure leaves the
 * library uninitialised with nothing allocated. */
int cdc_init(uint32_t dev_mask, const uint64_t gear[256], uint64_t mask_s, uint64_t mask_l,
             int cut_convention);
/* 1 while the table in use is the built-in placeholder (cdc_init with gear ==
 * NULL): cut points then differ from plakar's; pass the real fastcdc.G. */
int cdc_gear_is_placeholder(void);
void cdc_shutdown(void);
const char *cdc_strerror(int status);
int cdc_abi_version(void);
int cdc_device_count(void);

/* The built-in Gear table: a PLACEHOLDER (splitmix64 from a fixed seed).  The
 * v0.0.8 table of ext chunkers/fastcdc is not available in this build (see
 * DESIGN.md, "Oracle").  Pass the real table to cdc_init() once it is. */
void cdc_default_gear(uint64_t out[256]);
uint64_t cdc_default_mask_s(void);
uint64_t cdc_default_mask_l(void);

/* ext fastcdc (*FastCDC).Validate + chunkers.NewChunker's registry lookup
 * (algorithm names are matched after lower-casing, as
 * repository/repository.go:288 does).  Returns CDC_OK, CDC_E_UNSUPPORTED or
 * CDC_E_{NORMAL,MIN,MAX}_SIZE. */
int cdc_validate(const char *algorithm, const cdc_opts *opts);

/* chunking.DefaultConfiguration() (chunking/chunking.go:10-17). */
void cdc_default_opts(cdc_opts *out);

/* ---- batch path: host buffers in, host cut lists out ---------------------------
 * Replaces the per-file loop `chk := repo.Chunker(rd); for { chk.Next() }`
 * (snapshot/backup.go:647-665) for a batch of whole files already in host
 * memory.  Each buffer is chunked independently, as one complete stream.
 * out receives the cuts of buffer 0, then buffer 1, ...; out_counts[i] = the
 * number of cuts of buffer i.  If out_cap is too small, returns CDC_E_NOSPACE
 * with *out_needed set (out_needed may be NULL).  Synchronous. */
int cdc_chunk(const cdc_buf *bufs, int nbufs, const cdc_opts *opts, cdc_cut *out,
              uint64_t out_cap, uint64_t *out_counts, uint64_t *out_needed);

/* ---- collector: concurrent per-file callers -> device batches -------------------
 * plakar chunks each file in its own goroutine (snapshot/backup.go:216-225,
 * each running the Next() loop of backup.go:647-665).  A collector takes such
 * per-file calls from any number of threads and submits them to the devices
 * as batches: a batch closes at batch_bytes (0: 256 MiB), at 32 files, or
 * max_wait_us after its first file arrived; each device runs its batches
 * through a two-slot pipeline (batch k + 1 staged while batch k is chunked).
 * cdc_collector_chunk blocks until the caller's own cut list is back and has
 * cdc_chunk's contract for one buffer (CDC_E_NOSPACE with *count set when cap
 * is too small).  cdc_collector_free drains pending calls, then stops. */
typedef struct cdc_collector cdc_collector;
int cdc_collector_new(const cdc_opts *opts, uint64_t batch_bytes, uint32_t max_wait_us, cdc_collector **out);
int cdc_collector_chunk(cdc_collector *c, const void *data, uint64_t len, cdc_cut *out, uint64_t cap,
                        uint64_t *count);
int cdc_collector_stats(cdc_collector *c, uint64_t *requests, uint64_t *batches);
void cdc_collector_free(cdc_collector *c);

/* ---- Encode: LZ4 frame, then the AES-256-GCM stream ----------------------------
 * (*Repository).Encode (repository/repository.go:212-236) of n blobs that sit
 * in device memory at d_base + offsets[i], lens[i] bytes each:
 *   compress != 0: the LZ4 frame of compression.DeflateLZ4Stream
 *     (compression/compression.go:94-106; pierrec/lz4/v4 writer defaults:
 *     4-MiB independent blocks, content checksum; a block that does not
 *     shrink is stored);
 *   key != NULL (32 bytes, host memory): then encryption.EncryptStream
 *     (encryption/symmetric.go:72-163): subkey nonce (12) || Seal(key,
 *     subkey nonce, subkey) (48) || per 64-KiB piece k of the stream: nonce
 *     (12) || Seal(subkey, nonce, piece).  random (host, 56 bytes per blob:
 *     subkey 32, subkey nonce 12, data nonce 12) supplies what crypto/rand
 *     supplies in the reference; piece k's nonce is the data nonce with its
 *     last four bytes XOR k (big-endian).
 * Blob i's encoding lands at d_out + out_offsets[i] (device memory; host
 * array of n + 1 offsets, out_offsets[n] = total).  Returns CDC_E_NOSPACE
 * when out_cap is smaller than out_offsets[n].  Synchronous on `stream`. */
int cdc_encode_device(int device, const void *d_base, const uint64_t *offsets, const uint64_t *lens, uint32_t n,
                      int compress, const uint8_t *key, const uint8_t *random, uint8_t *d_out, uint64_t out_cap,
                      uint64_t *out_offsets, void *stream);

/* Upper bound of one blob's encoding (for out_cap). */
uint64_t cdc_encode_bound(uint64_t len, int compress, int encrypt);

/* ---- packfile builder: the consumer of the cut lists ---------------------------
 * snapshot/packer.go + packfile/packfile.go: blobs are appended to a
 * packfile whose bytes are those of (*PackFile).Serialize (packfile.go:241-294):
 * Blobs, then per blob {u8 type, 32-B checksum, u32 offset, u32 length}, then
 * the footer {u32 version 100, i64 timestamp, u32 count, u32 index offset,
 * 32-B SHA-256 of the index}, all little-endian.
 *   cdc_packer_add_blob    Packer.AddBlob; returns 1 once Size() > MaxSize
 *                          (packerJob's flush rule, snapshot/snapshot.go:71)
 *   cdc_packer_add_chunks  TYPE_CHUNK blobs base[cuts[i]] with digests[32 i]
 *                          (k_chunk_digest's output), rows with skip[i] != 0
 *                          skipped (BlobExists); stops after the blob that
 *                          fills the packfile; returns rows consumed
 *   cdc_packer_serialize   the whole packfile; _part: 0 data, 1 index,
 *                          2 footer (PutPackfile Encode's index and footer) */
typedef struct cdc_packer cdc_packer;
int cdc_packer_new(uint32_t max_size, cdc_packer **out);
int cdc_packer_add_blob(cdc_packer *p, uint8_t type, const uint8_t checksum[32], const uint8_t *data, uint64_t len);
int64_t cdc_packer_add_chunks(cdc_packer *p, const uint8_t *base, const cdc_cut *cuts, uint64_t n,
                              const uint8_t *digests, const uint8_t *skip);
uint64_t cdc_packer_size(const cdc_packer *p);
uint32_t cdc_packer_count(const cdc_packer *p);
int cdc_packer_serialize(const cdc_packer *p, int64_t timestamp, uint8_t *out, uint64_t cap, uint64_t *len);
int cdc_packer_serialize_part(const cdc_packer *p, int part, int64_t timestamp, uint8_t *out, uint64_t cap,
                              uint64_t *len);
void cdc_packer_reset(cdc_packer *p);
void cdc_packer_free(cdc_packer *p);

/* ---- end-to-end backup: files in, packfiles out ---------------------------------
 * chunkify (snapshot/backup.go:571-687) + PutBlob (snapshot/blobs.go:9-24) +
 * packerJob (snapshot/snapshot.go:51-92) for a list of files, as a pipeline
 * over batches of whole files (at most batch_bytes each, 0: 256 MiB): reader
 * threads read each file into a pinned arena and SHA-256 it there (the
 * object checksum); the device cuts, digests (SHA-256 + byte histogram per
 * chunk) and Encodes the new chunks (LZ4 when compress, then AES-256-GCM
 * when key != NULL; a chunk whose digest is in `known` (sorted, 32 B each:
 * BlobExists) or was already seen in this run is not stored again); packer
 * threads append the blobs to their own packfiles and hand each one, at
 * Size() > packfile_max (0: 20 MiB) and at the end, to on_pack (PutPackfile;
 * calls are serialised, from packer threads).  on_file is called once per
 * file (per piece, below) in the order the pipeline processes them: every
 * file's first piece, largest file first (a large file's object hash is a
 * long serial chain), then the later pieces of large files round by round,
 * so pieces of different files interleave; from one library thread (the
 * calling thread meanwhile
 * drives the next batches through the device), with pointers valid during the
 * call only; chunk entropies come from the device (cdc_chunk_entropy_device_async).
 * An empty file is one empty chunk (backup.go:631-635); a file shorter than
 * MinSize is one chunk.  A file larger than the batch size is processed in
 * pieces of about batch_bytes, in order, each chunked from the previous
 * piece's carried chunk start (the cut points are those of the whole file),
 * so the pinned and device buffers stay bounded by batch_bytes + Max per slot
 * whatever the file sizes; on_file is then called once per piece (piece /
 * pieces; cut offsets are file-relative; checksum and object_entropy are set
 * in the last piece's call).  A file that cannot be read (missing, not a
 * regular file, shorter than when it was listed) is reported through on_file
 * with status CDC_E_IO and no chunks, and the backup goes on with the others
 * (backupCtx.recordError, snapshot/backup.go:264-267); stats.failed_files
 * counts them.  A file in pieces that fails in a later piece (it shrank
 * mid-run) has had its earlier pieces reported with status CDC_OK and their
 * chunks (and blobs packed); that piece and every later one then come with
 * status CDC_E_IO and no chunks, and the last piece's call carries no
 * checksum: the caller drops the partial object (snapshot.BackupSession does).  Returns CDC_OK, or the first failure of the run itself (a
 * device error, a negative status from on_pack). */
typedef struct cdc_backup_opts {
    cdc_opts chunking;
    uint32_t packfile_max;
    int compress;
    const uint8_t *key;       /* 32-byte repository key, or NULL: no encryption */
    int packers;              /* packer threads (0: 8, NumCPU in the reference) */
    int readers;              /* reader threads (0: 8) */
    uint64_t batch_bytes;
    const uint8_t *known;     /* sorted digests already in the repository, or NULL */
    uint64_t nknown;
    int64_t timestamp;        /* packfile footer timestamp */
} cdc_backup_opts;
typedef struct cdc_backup_file {
    int index;                /* position in paths */
    int status;
    uint8_t checksum[32];     /* SHA-256 of the whole file (Object.Checksum) */
    uint64_t size;
    uint64_t nchunks;
    const cdc_cut *cuts;      /* (offset, length) in the file */
    const uint8_t *digests;   /* 32 B per chunk (Chunk.Checksum) */
    const uint32_t *hists;    /* 256 per chunk (entropy / Distribution) */
    const uint8_t *is_new;    /* 1: stored by this run (PutBlob), 0: deduplicated */
    const double *entropy;    /* per chunk (Chunk.Entropy: entropy() with Go's math.Log2) */
    double object_entropy;    /* Object.Entropy: sum of entropy * length in chunk order / size */
    uint32_t piece, pieces;   /* this call's piece of the file (pieces == 1: the whole file) */
    /* This piece's bytes as read (file offsets [data_offset, data_offset +
     * data_len)), valid during the callback; NULL when the file failed.  The
     * piece's chunks cover [data_offset, data_offset + the sum of their
     * lengths); a piece before the last carries its tail into the next.  For
     * the Object fields the caller computes from the bytes: ContentType
     * (mime.TypeByExtension, else mimetype.Detect of the first chunk,
     * snapshot/backup.go:580, 598-601) and the classifier feed
     * (cprocessor.Write per chunk, backup.go:577, 605). */
    const uint8_t *data;
    uint64_t data_offset, data_len;
} cdc_backup_file;
typedef struct cdc_backup_stats {
    uint64_t files, bytes, chunks, new_blobs, new_bytes, encoded_bytes, packfiles, packed_bytes, batches;
    double read_s;            /* file reads, summed over reader threads */
    double objhash_s;         /* object SHA-256, summed over reader threads */
    double h2d_s, chunk_s, digest_s, d2h_s, encode_s;  /* device stages (events; Encode: host wall) */
    double device_s;          /* the calling thread's time in the device stages (callbacks excluded) */
    double callback_s;        /* in on_file (the callback thread) */
    double read_wait_s;       /* the calling thread waiting for a batch's reads (device idle) */
    double pack_s;            /* packer threads' busy time, summed */
    double wall_s;
    uint64_t failed_files;    /* files reported with status CDC_E_IO */
    uint64_t pieces;          /* units through the pipeline (files + extra pieces of large files) */
    uint64_t slot_arena_bytes;  /* pinned arena bytes per slot this run needed (<= batch_bytes + Max) */
    /* GPU_MAX_HW_QUEUES in the process environment at cdc_backup_new (0: unset,
     * HIP's default of 4).  The pipeline's eight streams (scans, H2D, two
     * digest streams, two encoder streams and one side stream per Encode
     * workspace) run independently only with >= 8 hardware queues; with fewer,
     * HIP maps several streams onto one queue and the stages serialise
     * (INTEGRATION.md).  Other streams of the process (torch's, the collector's)
     * share queues with them even at 8. */
    int32_t hw_queues;
    int32_t streams_serialised;  /* 1 when hw_queues < 8 (or unset) */
    /* What sets the wall (round 6): fill_s, the call's start until batch 0's
     * reads have landed (the device's first work); drain_s, the last batch's
     * device stages done until the call returns (Encode, packers, callbacks
     * of the tail); chain_s / chain_bytes, the longest serial object SHA-256
     * chain of one file (a file's pieces hash one after another). */
    double fill_s, drain_s, chain_s;
    uint64_t chain_bytes;
} cdc_backup_stats;
typedef void (*cdc_backup_file_fn)(void *ctx, const cdc_backup_file *f);
typedef int (*cdc_backup_pack_fn)(void *ctx, const uint8_t *packfile, uint64_t len);
/* A backup context: its options (key and known digests copied), streams and
 * pinned / device buffers kept across calls (grown on demand).  Each
 * cdc_backup_files call is one backup of the given files: its dedup set
 * starts empty (plus `known`).  One call at a time per context. */
typedef struct cdc_backup cdc_backup;
int cdc_backup_new(int device, const cdc_backup_opts *opts, cdc_backup **out);
int cdc_backup_files(cdc_backup *b, const char *const *paths, int n, cdc_backup_file_fn on_file,
                     cdc_backup_pack_fn on_pack, void *ctx, cdc_backup_stats *stats);
void cdc_backup_free(cdc_backup *b);
/* new + files + free in one call. */
int cdc_backup_run(int device, const char *const *paths, int n, const cdc_backup_opts *opts,
                   cdc_backup_file_fn on_file, cdc_backup_pack_fn on_pack, void *ctx, cdc_backup_stats *stats);

/* The library's host SHA-256 (x86 SHA extensions when the CPU has them;
 * force_scalar != 0 takes the portable path).  cdc_sha256_accelerated: 1 if
 * the SHA extensions are in use. */
int cdc_sha256(const void *data, uint64_t len, int force_scalar, uint8_t out[32]);
int cdc_sha256_accelerated(void);

/* ---- pinned batch arena: files in, host cut lists out --------------------------
 * Replaces the importer's per-file os.Open + bufio reads
 * (snapshot/importer/fs/fs.go:69-71) feeding the per-file Next() loop: a
 * batch of files is read with pread(2) straight into library-owned pinned
 * host memory, then chunked by one cdc_chunk call whose host-to-device copies
 * are pinned DMA.  The bytes stay in the arena (cdc_batch_get) for the
 * per-chunk work (processChunk) until cdc_batch_reset.  A cgo caller passes
 * only file descriptors, paths and C memory: no Go pointer is stored.
 *   cdc_batch_new        arena of `capacity` bytes (buffers are 4-KiB aligned)
 *   cdc_batch_reserve    append a buffer of len bytes; *ptr = where to write it
 *   cdc_batch_add_fd     append len bytes read from fd (pread from offset 0)
 *   cdc_batch_add_files  append n whole files, read by `threads` threads;
 *   cdc_batch_chunk_files  add_files + chunking of those files, overlapped;
 *                        sizes[i] = file sizes (may be NULL).  All or nothing.
 *   cdc_batch_chunk      cdc_chunk over the arena's buffers, in order
 * Errors: CDC_E_NOSPACE (arena full), CDC_E_IO, CDC_E_NOT_INIT. */
typedef struct cdc_batch cdc_batch;
int cdc_batch_new(uint64_t capacity, cdc_batch **out);
int cdc_batch_reserve(cdc_batch *b, uint64_t len, uint8_t **ptr);
int cdc_batch_add_fd(cdc_batch *b, int fd, uint64_t len);
int cdc_batch_add_files(cdc_batch *b, const char *const *paths, int n, int threads, uint64_t *sizes);
/* cdc_batch_add_files + cdc_chunk over the n files it adds (not the arena's
 * earlier buffers), overlapped: reader threads run ahead while each
 * sub-batch of >= 256 MiB of whole files is chunked as soon as it is read.
 * out / out_counts (n entries) / out_needed as cdc_chunk. */
int cdc_batch_chunk_files(cdc_batch *b, const char *const *paths, int n, int threads, const cdc_opts *opts,
                          cdc_cut *out, uint64_t out_cap, uint64_t *out_counts, uint64_t *out_needed,
                          uint64_t *sizes);
int cdc_batch_count(const cdc_batch *b);
int cdc_batch_get(const cdc_batch *b, int i, const uint8_t **ptr, uint64_t *len);
int cdc_batch_chunk(cdc_batch *b, const cdc_opts *opts, cdc_cut *out, uint64_t out_cap,
                    uint64_t *out_counts, uint64_t *out_needed);
void cdc_batch_reset(cdc_batch *b);
void cdc_batch_free(cdc_batch *b);

/* ---- device-resident path -----------------------------------------------------
 * d_data: device pointer to len bytes (any alignment) on `device`.
 * final != 0: the buffer is a whole stream, so the last chunk ends at len.
 * final == 0: more bytes follow.  Only chunks whose cut is decided by the
 * bytes present are written, and result->consumed tells the caller where to
 * resume (the Peek(MaxSize) window of ext chunker.go).
 * d_cuts / d_result: device memory.  d_workspace: device memory of at least
 * cdc_device_workspace_size() bytes, not shared with another in-flight call.
 * Asynchronous on `stream`: enqueues kernels and returns.  Graph-capturable. */
int cdc_device_workspace_size(uint64_t len, const cdc_opts *opts, uint64_t *bytes);
int cdc_chunk_device_async(int device, const void *d_data, uint64_t len, int final,
                           const cdc_opts *opts, cdc_cut *d_cuts, uint64_t cut_cap,
                           cdc_result *d_result, void *d_workspace, uint64_t workspace_bytes,
                           void *stream);

/* Batched device path: nbufs independent device buffers chunked by one set of
 * launches.  d_cuts[i] / cut_caps[i] / d_results[i] are per buffer.  The
 * workspace must be at least cdc_device_batch_workspace_size() bytes. */
int cdc_device_batch_workspace_size(const uint64_t *lens, int nbufs, const cdc_opts *opts,
                                    uint64_t *bytes);
int cdc_chunk_device_batch_async(int device, const void *const *d_data, const uint64_t *lens,
                                 int nbufs, int final, const cdc_opts *opts,
                                 cdc_cut *const *d_cuts, const uint64_t *cut_caps,
                                 cdc_result *const *d_results, void *d_workspace,
                                 uint64_t workspace_bytes, void *stream);

/* ---- per-chunk digests: the per-chunk work of snapshot/backup.go processChunk --
 * For each chunk of a device cut list (offsets relative to d_data), the
 * SHA-256 of the chunk's bytes into d_digests (32 bytes per chunk: the
 * chunkHasher.Sum of snapshot/backup.go:604-606, hashing "SHA256" =
 * crypto/sha256, hashing/hashing.go:31-36) and, when d_hist is not NULL, the
 * chunk's byte histogram into d_hist (256 uint32 per chunk: the freq[] that
 * entropy() counts, snapshot/backup.go:548-557; the float64 entropy and the
 * normalised Distribution are the caller's, since math.Log2 defines them).
 * The chunk count is min(cut_cap, d_result->ncuts) when d_result is not NULL
 * (a cut list still on the device), else cut_cap.  An empty chunk hashes to
 * SHA-256(""), like processChunk([]byte{}) for an empty file (backup.go:631).
 * Asynchronous on `stream`; d_digests / d_hist hold cut_cap entries. */
int cdc_chunk_digests_device_async(int device, const void *d_data, uint64_t len, const cdc_cut *d_cuts,
                                   uint64_t cut_cap, const cdc_result *d_result, uint8_t *d_digests,
                                   uint32_t *d_hist, void *stream);
/* Batched form: every chunk of nbufs buffers hashes in one launch group (the
 * time of a launch is that of its longest chunk, so batch).  d_results and
 * d_hist may be NULL; d_hist entries are all NULL or all set (a buffer with
 * cut_cap 0 may pass NULL either way).  Past 32 buffers the launch group
 * reads its descriptors from device memory (one launch, one tail). */
int cdc_chunk_digests_device_batch_async(int device, const void *const *d_data, const uint64_t *lens, int nbufs,
                                         const cdc_cut *const *d_cuts, const uint64_t *cut_caps,
                                         const cdc_result *const *d_results, uint8_t *const *d_digests,
                                         uint32_t *const *d_hist, void *stream);
/* Hybrid form, synchronous: as the batched form, except that the longest
 * chunks' SHA-256 runs on `host_threads` host cores (x86 SHA extensions) while
 * the device hashes the others and computes every histogram.  A device
 * SHA-256 chain costs ~2 us per 64-B block against ~35 ns on a host core, and
 * a device launch lasts as long as its longest chunk, so a single pass over
 * long chunks ends sooner this way.  host_min_len = 0 picks the host's share
 * from the lengths (the longest chunks, as many as balance the host's bytes
 * over its cores and PCIe against the device's longest remaining chain);
 * otherwise every chunk of at least host_min_len bytes goes to the host.
 * host_threads = 0: all on the device.  Drains `stream` first (the cut lists
 * must be final) and returns once every digest and histogram is in device
 * memory; *host_chunks / *host_bytes (may be NULL) report the host's share.
 * At most 32 buffers. */
int cdc_chunk_digests_hybrid(int device, const void *const *d_data, const uint64_t *lens, int nbufs,
                             const cdc_cut *const *d_cuts, const uint64_t *cut_caps, const cdc_result *const *d_results,
                             uint8_t *const *d_digests, uint32_t *const *d_hist, int host_threads,
                             uint64_t host_min_len, void *stream, uint64_t *host_chunks, uint64_t *host_bytes);
/* entropy() of snapshot/backup.go:548-569 for `rows` histogram rows (256
 * uint32 each, as cdc_chunk_digests* writes them; a row's sum is its chunk's
 * length) into d_entropy (float64 per row): the reference's terms with Go's
 * math.Log2, one IEEE operation at a time, summed in bin order (bit-exact);
 * 0 for an all-zero row.  Asynchronous on `stream`. */
int cdc_chunk_entropy_device_async(int device, const uint32_t *d_hist, uint64_t rows, double *d_entropy,
                                   void *stream);

/* ---- streaming chunker: chunkers.NewChunker / (*Chunker).Next -----------------
 * Push model, so cgo never hands a Go pointer to asynchronous HIP work: the
 * caller appends stream bytes into a pinned staging window the library owns
 * (cdc_stream_buffer + cdc_stream_commit), then drains chunks with
 * cdc_stream_next.  A chunk pointer aliases that window and stays valid until
 * the next call on the same stream, like the slice ext (*Chunker).Next returns
 * (it aliases the bufio buffer).
 *   cdc_stream_next -> CDC_OK        chunk and len receive the next chunk
 *                   -> CDC_NEED_DATA append bytes (or commit with eof = 1)
 *                   -> CDC_EOF       no more chunks (io.EOF)
 * window_bytes = 0 picks a default (>= 2 * max_size). */
typedef struct cdc_stream cdc_stream;
int cdc_stream_new(const char *algorithm, const cdc_opts *opts, uint64_t window_bytes, int device,
                   cdc_stream **out);
int cdc_stream_buffer(cdc_stream *s, uint8_t **write_ptr, uint64_t *space);
int cdc_stream_commit(cdc_stream *s, uint64_t nbytes, int eof);
int cdc_stream_next(cdc_stream *s, const uint8_t **chunk, uint64_t *len);
void cdc_stream_free(cdc_stream *s);

/* Pull-model convenience over cdc_stream (an io.Reader as a callback):
 * read(ctx, buf, cap) returns the number of bytes read, 0 at EOF, < 0 on error. */
typedef int64_t (*cdc_read_fn)(void *ctx, void *buf, uint64_t cap);
typedef struct cdc_chunker cdc_chunker;
int cdc_chunker_new(const char *algorithm, cdc_read_fn read, void *ctx, const cdc_opts *opts,
                    cdc_chunker **out);
int cdc_chunker_next(cdc_chunker *c, const uint8_t **chunk, uint64_t *len);
void cdc_chunker_free(cdc_chunker *c);

/* ---- diagnostics ---------------------------------------------------------------
 * Kernel selection for tests: 0 = default (scan + index + speculative
 * resolution), 1 = force the sequential single-wave resolver (reference path
 * on the device, for cross-checking the fast path). */
int cdc_set_debug_mode(int mode);

/* When and how the MaskL candidate index is built: 0 = never (walkers
 * raw-scan every MaskL region), 1 = adaptive (default: while recent launch
 * groups on the device needed it, in the same pass as the MaskS index where
 * the masks admit it, else by k_scan_l; every 16th group otherwise runs the
 * selection test alone as a probe), 2 = every launch group in the fused pass,
 * 3 = every launch group by k_scan_l.  Cut points never depend on it; tests
 * use it to cover every path.  Setting a mode clears the adaptive state.
 * Initial value from the CDC_MASKL_INDEX environment variable.  Not a
 * reference interface (the Go chunker has no index).  Returns CDC_OK or
 * CDC_E_INVALID. */
int cdc_set_maskl_index_mode(int mode);

/* Adaptive MaskL state of one device (diagnostics, after a device sync):
 * *hint = 1 while the next launch groups build the MaskL index (a recent
 * group needed it), *groups = launch groups issued on the device so far.  Not a reference interface. */
int cdc_debug_maskl_state(int device, uint32_t *hint, uint64_t *groups);

/* The measured HBM stream-read rate of the device, for the roofline beside
 * the spec peak (SURVEY.md 8(d) "also report a measured stream-read peak"):
 * `reps` launches each of three read-only kernels over [d_buf, d_buf + len)
 * (16-byte aligned), interleaved and timed with hipEvents on `stream`:
 * best_us[f] / median_us[f] (microseconds) for form f = 0 plain 16-byte
 * loads, 1 nontemporal loads, 2 the scan's LDS-DMA staging.  Synchronous.
 * Diagnostic, not a reference interface. */
int cdc_debug_stream_read(int device, const void *d_buf, uint64_t len, int reps, double best_us[3], double median_us[3],
                          void *stream);

/* Per-chunk digests: the lane count the digest kernels assume the device
 * keeps resident (a launch with more chunks than this gives each lane a run
 * of ceil(chunks / lanes) consecutive chunks).  0 (the default) derives it
 * from the device's CU count; tests set small values to cover multi-chunk
 * lanes on small inputs.  Digests never depend on it.  Not a reference
 * interface.  Returns CDC_OK. */
int cdc_debug_set_digest_lanes(uint64_t lanes);

/* Live profiling of the device path: when enabled, every launch group records
 * hipEvents on its stream before/after the scan kernel and after the last
 * resolution kernel.  collect() waits for the recorded events, returns the
 * summed scan time, summed pipeline time, number of launch groups and input
 * bytes scanned since the last collect, and resets. */
int cdc_profile_enable(int on);
int cdc_profile_collect(double *scan_ms, double *pipeline_ms, uint64_t *launches,
                        uint64_t *scan_bytes);

#ifdef __cplusplus
}
#endif
#endif /* PLAKAR_CDC_H */
