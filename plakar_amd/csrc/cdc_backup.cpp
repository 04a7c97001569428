// End-to-end backup pipeline: files in, packfiles out (SURVEY.md section 8f
// rank 3, the consumer side of the chunker).
//
// The reference runs, per file and in one goroutine per file
// (snapshot/backup.go:216-225), chunkify (backup.go:571-687): the importer's
// reads (snapshot/importer/fs/fs.go:69-71), the chunker's Next() loop
// (backup.go:647-665), per chunk processChunk (backup.go:594-629: SHA-256,
// byte histogram -> entropy, BlobExists, PutBlob), the object's SHA-256 over
// the whole file; PutBlob (snapshot/blobs.go:9-24) Encodes each new chunk
// (repository/repository.go:212-236: LZ4 then AES-256-GCM) and hands it to
// NumCPU packerJob workers (snapshot/snapshot.go:51-92), each appending to its
// own packfile and flushing it at Size() > MaxSize.
//
// Here the same work runs as a pipeline over batches of whole files, built on
// the library's own entry points:
//   reader threads   pread each file of batch k into a pinned arena slot and
//                    hash it there (the object checksum, host SHA-256 with the
//                    CPU's SHA extensions: one serial chain per file)
//   device (caller)  H2D, cut points (cdc_chunk_device_batch_async), per-chunk
//                    SHA-256 + histograms (cdc_chunk_digests_device_batch_async),
//                    D2H of the lists; host dedup (the run's own set + the
//                    caller's known digests: BlobExists); Encode of the new
//                    chunks in device memory (cdc_encode_device); D2H of the
//                    encoded blobs; per-file callback (the Object's fields)
//   packer threads   Packer.AddBlob into their own packfile (cdc_packer_*),
//                    flush at Size() > MaxSize to the packfile callback
//                    (PutPackfile)
// Six slots (arena + device buffers) rotate, so later batches are read while
// batch k is on the device and earlier ones are packed; the per-file
// callbacks run on their own thread while the device takes the next batches.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <set>
#include <new>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "cdc_internal.h"

namespace {

using Clock = std::chrono::steady_clock;

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Digest {
    uint8_t b[32];
    bool operator==(const Digest &o) const { return std::memcmp(b, o.b, 32) == 0; }
};
struct DigestHash {
    size_t operator()(const Digest &d) const
    {
        size_t h;
        std::memcpy(&h, d.b, sizeof(h));  // SHA-256 output: any 8 bytes are uniform
        return h;
    }
};

// Bytes [off, off + len) of the file; CDC_E_IO if it cannot be opened or ends
// early (a file that shrank since plan() stat'ed it).
int read_exact(const char *path, uint8_t *dst, uint64_t off, uint64_t len)
{
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return CDC_E_IO;
    uint64_t got = 0;
    int st = CDC_OK;
    while (got < len) {
        const ssize_t k =
            pread(fd, dst + got, size_t(std::min<uint64_t>(len - got, 1ull << 30)), off_t(off + got));
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) {
            st = CDC_E_IO;
            break;
        }
        got += uint64_t(k);
    }
    close(fd);
    return st;
}

// A unit is one file, or one piece of a file larger than the batch size
// (batch_bytes): piece j adds the file's bytes [nb, ne) = [j P, min((j + 1) P,
// size)) and is chunked from the previous piece's carried next start (at most
// Max - 1 bytes before nb) to ne, non-final except the last piece, so every
// slot's arena stays at most P + Max bytes whatever the file sizes (the
// reference streams a file through its chunker in the same way,
// snapshot/backup.go:647-665).  Piece j's own bytes [nb, ne) are read as soon
// as its slot is free, at a fixed place (Max bytes into its arena space); the
// carried prefix [next start, nb) (< Max bytes) is read in front of them once
// piece j - 1's cut list is back.  So a large file's pieces are read ahead
// like any other unit, and the device waits only for that short prefix.
struct Unit {
    uint32_t file, piece, pieces;
    uint64_t nb, ne;       // nominal byte range of the file (what the object hash adds)
    uint64_t cap;          // arena bytes reserved (256-B aligned)
    uint64_t arena_off;    // the unit's arena space; [nb, ne) is read to fixed_off()
    uint64_t start = 0, len = 0;  // set by the readers: file bytes [start, start + len) in the arena ...
    uint64_t data_off = 0;        // ... from data_off (arena_off for a whole file and a first piece)
    int err = CDC_OK;             // set by the readers: CDC_E_IO (the file could not be read)
};

uint64_t fixed_off(const Unit &u, uint64_t max_size) { return u.arena_off + (u.piece ? max_size : 0); }

// Per file, shared by its pieces (guarded by Run::mu unless noted).
struct FileState {
    uint64_t size = 0;
    int err = CDC_OK;             // the first failure of any of its pieces
    uint32_t dev_pieces = 0;      // pieces whose carried next start is published
    uint32_t hashed_pieces = 0;   // pieces whose bytes went into the object hash
    uint64_t next_start = 0;
    cdc::Sha256 sha;              // multi-piece files (the reader of the current piece)
    uint8_t obj[32] = {};         // the object checksum
    double ent_acc = 0.0;         // Object.Entropy's running sum (callback thread)
    bool ent_any = false;
    double chain_s = 0.0;         // its object hash so far (the pieces hash in sequence)
};

struct Batch {
    uint32_t u0, u1;      // units [u0, u1)
    uint64_t bytes;       // arena bytes (units 256-B aligned)
    uint64_t cuts_cap;    // sum of cap / Min + 2
};

// Buffers of one pipeline slot.  Kept by the context across runs and grown
// on demand (pinned allocations are slow: they are made once per session).
struct Slot {
    uint8_t *h_arena = nullptr, *d_in = nullptr;
    uint64_t arena_cap = 0;
    void *d_ws = nullptr;
    uint64_t ws_cap = 0;
    cdc_cut *d_cuts = nullptr, *h_cuts = nullptr, *d_acuts = nullptr;  // file-relative; arena-relative
    uint64_t *h_meta = nullptr, *d_meta = nullptr;                        // (cut0, cap, arena_off) per file
    cdc_result *d_res = nullptr, *h_res = nullptr;
    uint8_t *d_dig = nullptr, *h_dig = nullptr;
    uint32_t *d_hist = nullptr, *h_hist = nullptr;
    double *d_ent = nullptr, *h_ent = nullptr;
    uint64_t cuts_cap = 0, res_cap = 0;
    uint8_t *d_enc = nullptr, *h_enc = nullptr;
    uint64_t enc_cap = 0, henc_cap = 0;
    // A: H2D start / end, cut points end; D: digests start / end, lists back
    hipEvent_t ev[6] = {};
    hipEvent_t ev_enc = nullptr;  // E: the encoded blobs back
    // per run: lifecycle (guarded by Run::mu) and the enqueued batch's lists
    int batch = -1, next = 0;  // the batch in the slot; the one that takes it next
    bool read_done = false, hash_done = false, device_done = false;
    uint32_t nread = 0, nhashed = 0;
    uint64_t pending = 0;  // blobs not yet packed
    std::vector<uint64_t> lens, cut0;
    uint64_t ncut = 0;
    double t_enq = 0;
    std::vector<uint8_t> is_new;       // per chunk of the batch (BlobExists' answer)
    std::vector<uint64_t> file_new0;   // per file: its first entry in is_new
};

// Six slots: batches k + 1 .. k + 5 are read (and object-hashed: a 128-MiB
// file is one ~64-ms SHA-256 chain on a host core, and a slot is released
// only once every object hash of its batch is done) while batch k is on the
// device and earlier ones are packed; with two, reads and packing serialise;
// with four the device idled for tens of ms behind a large file's hash (c4b
// 10.1-11.3 GiB/s against 13.3-14.2 with six; eight no better).
#ifndef CDC_BACKUP_SLOTS
#define CDC_BACKUP_SLOTS 6
#endif
constexpr int kSlots = CDC_BACKUP_SLOTS;
// cdc_backup::stream: scans kA, H2D kH, digests alternate over kD, kD + 1,
// the two encoder threads kE and kE + 2
constexpr int kA = 0, kD = 1, kE = 3, kH = 4;
constexpr int kEncoders = 2;  // one's kernels run beside the other's copy-back (~10 ms per 512-MiB batch)
// The pipeline's scans run persistent (tasks from a counter, ~2 per wave): a
// static grid needs every CU, and the CUs held by the other streams' digest
// launches (66 KiB of LDS per workgroup, ~10-18 ms each) left the scan's last
// workgroups waiting 4-5 ms per batch (profiles/r04_c4b_devtrace.txt).
constexpr int kBackupScanTpw = 2;

#define HIPOK(x)                                         \
    do {                                                 \
        if ((x) != hipSuccess) return CDC_E_DEVICE;      \
    } while (0)

template <typename T>
int grow_dev(T *&p, uint64_t &cap, uint64_t need)
{
    if (need <= cap && p) return CDC_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HIPOK(hipMalloc(reinterpret_cast<void **>(&p), need ? need : 1));
    cap = need;
    return CDC_OK;
}

template <typename T>
int grow_host(T *&p, uint64_t need, uint64_t have)
{
    if (need <= have && p) return CDC_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    HIPOK(hipHostMalloc(reinterpret_cast<void **>(&p), need ? need : 1, hipHostMallocDefault));
    return CDC_OK;
}

int grow_slot(Slot &s, uint64_t arena, uint64_t ws, uint64_t ncuts, uint64_t nfiles)
{
    int st;
    if (!s.ev[0]) {
        for (auto &e : s.ev) HIPOK(hipEventCreate(&e));
        HIPOK(hipEventCreateWithFlags(&s.ev_enc, hipEventDisableTiming));
    }
    if (arena > s.arena_cap || !s.h_arena) {
        if ((st = grow_host(s.h_arena, arena, 0)) != CDC_OK) return st;
        uint64_t c = s.arena_cap;
        if ((st = grow_dev(s.d_in, c, arena)) != CDC_OK) return st;
        s.arena_cap = arena;
    }
    if ((st = grow_dev(s.d_ws, s.ws_cap, std::max<uint64_t>(ws, 256))) != CDC_OK) return st;
    if (ncuts > s.cuts_cap || !s.h_cuts) {
        uint64_t c = s.cuts_cap * sizeof(cdc_cut);
        if ((st = grow_dev(s.d_cuts, c, ncuts * sizeof(cdc_cut))) != CDC_OK) return st;
        if ((st = grow_host(s.h_cuts, ncuts * sizeof(cdc_cut), 0)) != CDC_OK) return st;
        c = s.cuts_cap * sizeof(cdc_cut);
        if ((st = grow_dev(s.d_acuts, c, ncuts * sizeof(cdc_cut))) != CDC_OK) return st;
        c = s.cuts_cap * 32;
        if ((st = grow_dev(s.d_dig, c, ncuts * 32)) != CDC_OK) return st;
        if ((st = grow_host(s.h_dig, ncuts * 32, 0)) != CDC_OK) return st;
        c = s.cuts_cap * 1024;
        if ((st = grow_dev(s.d_hist, c, ncuts * 1024)) != CDC_OK) return st;
        if ((st = grow_host(s.h_hist, ncuts * 1024, 0)) != CDC_OK) return st;
        c = s.cuts_cap * 8;
        if ((st = grow_dev(s.d_ent, c, ncuts * 8)) != CDC_OK) return st;
        if ((st = grow_host(s.h_ent, ncuts * 8, 0)) != CDC_OK) return st;
        s.cuts_cap = ncuts;
    }
    if (nfiles > s.res_cap || !s.h_res) {
        uint64_t c = s.res_cap * sizeof(cdc_result);
        if ((st = grow_dev(s.d_res, c, nfiles * sizeof(cdc_result))) != CDC_OK) return st;
        if ((st = grow_host(s.h_res, nfiles * sizeof(cdc_result), 0)) != CDC_OK) return st;
        c = s.res_cap * 24;
        if ((st = grow_dev(s.d_meta, c, nfiles * 24)) != CDC_OK) return st;
        if ((st = grow_host(s.h_meta, nfiles * 24, 0)) != CDC_OK) return st;
        s.res_cap = nfiles;
    }
    return CDC_OK;
}

void free_slot(Slot &s)
{
    for (void *p : {static_cast<void *>(s.d_in), s.d_ws, static_cast<void *>(s.d_cuts), static_cast<void *>(s.d_res),
                    static_cast<void *>(s.d_acuts), static_cast<void *>(s.d_meta),
                    static_cast<void *>(s.d_dig), static_cast<void *>(s.d_hist), static_cast<void *>(s.d_ent),
                    static_cast<void *>(s.d_enc)})
        if (p) (void)hipFree(p);
    for (void *p : {static_cast<void *>(s.h_arena), static_cast<void *>(s.h_cuts), static_cast<void *>(s.h_res),
                    static_cast<void *>(s.h_meta),
                    static_cast<void *>(s.h_dig), static_cast<void *>(s.h_hist), static_cast<void *>(s.h_ent),
                    static_cast<void *>(s.h_enc)})
        if (p) (void)hipHostFree(p);
    for (auto &e : s.ev)
        if (e) (void)hipEventDestroy(e);
    if (s.ev_enc) (void)hipEventDestroy(s.ev_enc);
    s = Slot();
}

}  // namespace

struct cdc_backup {
    int device = 0;
    cdc_backup_opts o;
    std::vector<uint8_t> key;    // the repository key, copied (o.key points here)
    std::vector<uint8_t> known;  // sorted digests, copied (o.known points here)
    Slot slot[kSlots];
    std::vector<cdc_packer *> packers;  // kept across runs (their buffers stay reserved and mapped)
    // A: H2D + cut points (ahead); D0 / D1: digests, entropy, lists of even /
    // odd batches (one batch's longest-chunk tail overlaps the next batch's
    // digests); E: Encode and the encoded blobs back.  Four streams plus
    // Encode's own: independent only with GPU_MAX_HW_QUEUES >= 8 (HIP's
    // default of 4 maps several streams onto one hardware queue, which
    // serialises them).
    hipStream_t stream[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    int hw_queues = 0;  // GPU_MAX_HW_QUEUES at cdc_backup_new (0: unset)
};

namespace {

struct Blob {
    Digest sum;
    const uint8_t *data;
    uint64_t len;
    int slot;
};

// Encode of one batch's new chunks, handed from the calling thread to the
// encoder threads once the batch is deduplicated.
struct EncJob {
    size_t k;
    std::vector<uint64_t> off, len;
    std::vector<Digest> sum;
    uint64_t bound;
};

struct Run {
    cdc_backup *B;
    const cdc_backup_opts &o;
    const char *const *paths;
    int n;
    cdc_backup_file_fn on_file;
    cdc_backup_pack_fn on_pack;
    void *ctx;
    std::vector<FileState> files;
    std::vector<Unit> units;
    std::vector<Batch> batches;
    std::vector<uint32_t> batch_of;  // per unit
    uint32_t next_read = 0;        // the next unit to read (guarded by mu)
    uint32_t reading = 0;          // reads in progress (guarded by mu)
    std::set<uint32_t> hash_q;     // units read, not yet hashed, in unit order (guarded by mu)
    std::set<uint32_t> prefix_q;   // pieces j > 0 whose [nb, ne) is read, not yet their carried prefix (mu)
    int64_t fail_file = -1, fail_piece = -1;  // CDC_BACKUP_FAIL_PIECE=file:piece (test hook): that read fails
    int64_t fail_dev_file = -1, fail_dev_piece = -1;  // CDC_BACKUP_FAIL_DEVICE=file:piece: its launch aborts (debug mode 2)
    double last_dev_end = 0.0;  // seconds into the call when the last batch's device stages were done
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<int> status{CDC_OK};
    bool stop_packers = false;
    std::deque<EncJob> enc_q;  // guarded by mu
    bool stop_encoder = false;
    size_t devices_done = 0;  // batches through finish_device (callbacks may start)
    size_t cuts = 0, digs = 0;  // batches whose stage A / stage B is enqueued (the calling thread's)
    std::deque<Blob> queue;
    std::mutex sink_mu;
    std::unordered_set<Digest, DigestHash> seen;
    cdc_backup_stats st{};
    std::mutex stat_mu;
    // CDC_BACKUP_TRACE=<path>: (seconds since the call began, event, batch,
    // unit, bytes) per pipeline event, written there as CSV at the end; the
    // device's stage events as offsets from trace_ref (recorded at the start)
    Clock::time_point t0 = Clock::now();
    const char *trace_path = std::getenv("CDC_BACKUP_TRACE");
    struct Ev {
        double t;
        const char *what;
        int64_t batch, unit;
        uint64_t bytes;
    };
    std::vector<Ev> trace;
    std::mutex trace_mu;
    hipEvent_t trace_ref = nullptr;

    void ev(const char *what, int64_t batch, int64_t unit = -1, uint64_t bytes = 0, double t = -1)
    {
        if (!trace_path) return;
        if (t < 0) t = std::chrono::duration<double>(Clock::now() - t0).count();
        std::lock_guard<std::mutex> lk(trace_mu);
        trace.push_back(Ev{t, what, batch, unit, bytes});
    }

    Run(cdc_backup *b, const char *const *p, int nn) : B(b), o(b->o), paths(p), n(nn)
    {
        if (const char *f = std::getenv("CDC_BACKUP_FAIL_PIECE")) {
            long a = -1, c = -1;
            if (std::sscanf(f, "%ld:%ld", &a, &c) == 2) {
                fail_file = a;
                fail_piece = c;
            }
        }
        if (const char *f = std::getenv("CDC_BACKUP_FAIL_DEVICE")) {
            long a = -1, c = -1;
            if (std::sscanf(f, "%ld:%ld", &a, &c) == 2) {
                fail_dev_file = a;
                fail_dev_piece = c;
            }
        }
    }

    void fail(int s)
    {
        int ok = CDC_OK;
        status.compare_exchange_strong(ok, s);
        {
            std::lock_guard<std::mutex> lk(mu);
        }
        cv.notify_all();
    }
};

int plan(Run &R, uint64_t &arena_cap, uint64_t &cuts_cap, uint64_t &ws_cap, uint64_t &files_cap)
{
    const uint64_t bb = R.o.batch_bytes ? R.o.batch_bytes : (256ull << 20);
    const uint64_t P = std::max<uint64_t>(bb, 4ull * R.o.chunking.max_size);  // piece size (>> Max)
    R.files.resize(size_t(R.n));
    for (int i = 0; i < R.n; ++i) {
        FileState &F = R.files[size_t(i)];
        struct stat sb;
        // a path that cannot be stat'ed or is not a regular file: that file
        // fails (status CDC_E_IO in its record), the others go on, as
        // backupCtx.recordError does (snapshot/backup.go:264-267)
        if (!R.paths[i] || stat(R.paths[i], &sb) != 0 || !S_ISREG(sb.st_mode)) F.err = CDC_E_IO;
        else F.size = uint64_t(sb.st_size);
        const uint32_t pieces = F.size > P ? uint32_t((F.size + P - 1) / P) : 1u;
        for (uint32_t j = 0; j < pieces; ++j) {
            Unit u;
            u.file = uint32_t(i);
            u.piece = j;
            u.pieces = pieces;
            u.nb = pieces == 1 ? 0 : uint64_t(j) * P;
            u.ne = pieces == 1 ? F.size : std::min<uint64_t>(F.size, uint64_t(j + 1) * P);
            u.cap = ((u.ne - u.nb) + (j ? R.o.chunking.max_size : 0) + 255) & ~255ull;
            R.units.push_back(u);
        }
    }
    // Largest files first: a file's object SHA-256 is one serial chain on a
    // host core (a 128-MiB file ~64 ms) and a slot is released only once
    // every hash of its batch is done, so a large file late in the run held
    // the device idle behind its hash (profiles/r03_c4b_timeline.txt: gaps of
    // 15-70 ms).  Pieces go round by round: every file's piece 0 (largest
    // file first), then every piece 1, and so on.  Piece j + 1 can only be
    // hashed after piece j, so with a large file's pieces consecutive its
    // later pieces held slots for seconds while the next large file waited
    // for one (c4bl: 4 files of 0.5-1.5 GiB hashed one after another, 1.24 s;
    // round by round their chains run side by side).  Callbacks come in this
    // processing order (each names its file and piece).
    {
        std::vector<uint32_t> first(size_t(R.n) + 1, 0);  // units of file i: [first[i], first[i + 1])
        for (size_t u = 0; u < R.units.size(); ++u) first[R.units[u].file + 1] = uint32_t(u + 1);
        for (int i = 0; i < R.n; ++i) first[size_t(i) + 1] = std::max(first[size_t(i) + 1], first[size_t(i)]);
        std::vector<uint32_t> ord(size_t(R.n));
        for (int i = 0; i < R.n; ++i) ord[size_t(i)] = uint32_t(i);
        std::stable_sort(ord.begin(), ord.end(),
                         [&](uint32_t a, uint32_t b) { return R.files[a].size > R.files[b].size; });
        std::vector<Unit> sorted;
        sorted.reserve(R.units.size());
        std::vector<uint32_t> multi;  // files in pieces, largest first
        for (uint32_t i : ord) {
            sorted.push_back(R.units[first[i]]);  // round 0: every file (a file has at least one unit)
            if (first[i + 1] - first[i] > 1) multi.push_back(i);
        }
        for (uint32_t r = 1; sorted.size() < R.units.size(); ++r)
            for (uint32_t i : multi)
                if (first[i] + r < first[i + 1]) sorted.push_back(R.units[first[i] + r]);
        R.units.swap(sorted);
    }
    R.batch_of.resize(R.units.size());
    Batch cur{0, 0, 0, 0};
    for (uint32_t k = 0; k < uint32_t(R.units.size()); ++k) {
        Unit &u = R.units[k];
        if (cur.u1 > cur.u0 && (cur.bytes + u.cap > bb || cur.u1 - cur.u0 >= 4096)) {
            R.batches.push_back(cur);
            cur = Batch{k, k, 0, 0};
        }
        R.batch_of[k] = uint32_t(R.batches.size());
        u.arena_off = cur.bytes;
        cur.bytes += u.cap;
        cur.cuts_cap += u.cap / R.o.chunking.min_size + 2;
        cur.u1 = k + 1;
    }
    if (cur.u1 > cur.u0) R.batches.push_back(cur);
    arena_cap = cuts_cap = ws_cap = files_cap = 0;
    std::vector<uint64_t> caps;
    for (const Batch &b : R.batches) {
        arena_cap = std::max(arena_cap, std::max<uint64_t>(b.bytes, 256));
        cuts_cap = std::max(cuts_cap, b.cuts_cap);
        files_cap = std::max<uint64_t>(files_cap, b.u1 - b.u0);
        for (uint32_t g = b.u0; g < b.u1; g += cdc::kMaxBufsPerLaunch) {
            const uint32_t e = std::min<uint32_t>(b.u1, g + cdc::kMaxBufsPerLaunch);
            caps.clear();
            for (uint32_t k = g; k < e; ++k) {
                const Unit &u = R.units[k];
                // a non-final piece is chunked alone in its batch (one launch, final = 0)
                if (u.piece + 1 < u.pieces && b.u1 - b.u0 != 1) return CDC_E_INVALID;
                caps.push_back(u.cap);
            }
            uint64_t ws = 0;
            const int s = cdc_device_batch_workspace_size(caps.data(), int(e - g), &R.o.chunking, &ws);
            if (s != CDC_OK) return s;
            ws_cap = std::max(ws_cap, ws);
        }
    }
    return CDC_OK;
}

// A slot is free once its batch left the device, every blob of it is packed
// and every file of it hashed.  Called with R.mu held.
void maybe_release(Run &R, Slot &s)
{
    if (s.device_done && s.hash_done && s.pending == 0 && s.batch >= 0) {
        s.batch = -1;
        R.cv.notify_all();
    }
}

// Reader threads.  Three kinds of task: reading unit after unit, in batch
// order, into its batch's slot (a slot is claimed by the first unit of its
// batch once the batch kSlots back released it); reading a piece's carried
// prefix once the previous piece's cut list is back; and hashing a unit that
// is read (the object checksum, one serial chain per file: a 124-MiB file is
// ~62 ms on a host core).  A thread takes a prefix whenever one can start
// (the device waits for it), else the next read, else the first hash in unit
// order that it can start, so the device's input is never queued behind
// object hashes (when each reader hashed what it had just read, the 16
// largest files held all 16 readers for up to 60 ms while the device waited
// for the next batch: profiles/r04_c4b_trace.txt).  Piece j > 0 of a large
// file is hashed once piece j - 1 is hashed (its own bytes are at a fixed
// place, so the hash does not wait for its prefix).  A file that cannot be
// read is marked failed and the run goes on.
bool read_ready_locked(Run &R)  // the next unit's read can start (R.mu held)
{
    if (R.next_read >= R.units.size()) return false;
    const uint32_t i = R.next_read, k = R.batch_of[i];
    const Slot &s = R.B->slot[k % kSlots];
    return s.batch == int(k) || (s.batch < 0 && s.next == int(k));
}

bool prefix_ready_locked(Run &R, uint32_t i)  // piece i's carried prefix can be read (R.mu held)
{
    const Unit &u = R.units[i];
    const FileState &F = R.files[u.file];
    return F.err != CDC_OK || u.err != CDC_OK || F.dev_pieces >= u.piece;
}

bool hash_ready_locked(Run &R, uint32_t i)  // unit i's bytes can go into its object hash (R.mu held)
{
    const Unit &u = R.units[i];
    return u.pieces == 1 || R.files[u.file].hashed_pieces >= u.piece;
}

void reader_main(Run &R)
{
    double read_s = 0, hash_s = 0;
    const uint64_t M = R.o.chunking.max_size;
    for (;;) {
        uint32_t i = 0;
        bool is_read = false, is_prefix = false;
        {
            std::unique_lock<std::mutex> lk(R.mu);
            auto h = R.hash_q.end();
            auto pq = R.prefix_q.end();
            R.cv.wait(lk, [&] {
                if (R.status.load() != CDC_OK) return true;
                for (pq = R.prefix_q.begin(); pq != R.prefix_q.end(); ++pq)
                    if (prefix_ready_locked(R, *pq)) return (is_prefix = true);
                if ((is_read = read_ready_locked(R))) return true;
                for (h = R.hash_q.begin(); h != R.hash_q.end(); ++h)
                    if (hash_ready_locked(R, *h)) return true;
                return R.next_read >= R.units.size() && R.reading == 0 && R.hash_q.empty() && R.prefix_q.empty();
            });
            if (R.status.load() != CDC_OK) break;
            if (is_prefix) {
                i = *pq;
                R.prefix_q.erase(pq);
                ++R.reading;
                Unit &u = R.units[i];
                FileState &F = R.files[u.file];
                if (u.err == CDC_OK && F.err != CDC_OK) u.err = F.err;  // an earlier piece failed
                // the carry is the previous piece's undecided tail: fewer than
                // Max bytes before nb (anything else is a device failure)
                if (u.err == CDC_OK && !(F.next_start <= u.nb && F.next_start + M > u.nb)) u.err = CDC_E_DEVICE;
                u.start = u.err == CDC_OK ? F.next_start : u.nb;
                u.len = u.err == CDC_OK ? u.ne - u.start : 0;
                u.data_off = fixed_off(u, M) - (u.nb - u.start);
            } else if (is_read) {
                i = R.next_read++;
                ++R.reading;
                const uint32_t k = R.batch_of[i];
                Slot &s = R.B->slot[k % kSlots];
                if (s.batch != int(k)) {
                    s.batch = int(k);
                    s.next = int(k) + kSlots;
                    s.read_done = s.hash_done = s.device_done = false;
                    s.nread = s.nhashed = 0;
                    s.pending = 0;
                }
                Unit &u = R.units[i];
                FileState &F = R.files[u.file];
                u.err = F.err;
                // a whole file or a first piece: [0, ne) at arena_off; a later
                // piece: its own bytes [nb, ne) now, the prefix once known
                u.start = u.nb;
                u.len = u.err == CDC_OK ? u.ne - u.nb : 0;
                u.data_off = fixed_off(u, M);
            } else if (h != R.hash_q.end()) {
                i = *h;
                R.hash_q.erase(h);
            } else {
                break;  // every unit read and hashed
            }
        }
        const uint32_t k = R.batch_of[i];
        const Batch &b = R.batches[k];
        Slot &s = R.B->slot[k % kSlots];
        Unit &u = R.units[i];
        FileState &F = R.files[u.file];
        uint8_t *fixed = s.h_arena + fixed_off(u, M);  // the unit's own bytes [nb, ne)
        if (is_read || is_prefix) {
            // is_read: [nb, ne) (a whole file: [0, size)); is_prefix: the
            // carried bytes [start, nb) in front of them
            const uint64_t off = is_read ? u.nb : u.start, n = is_read ? u.len : u.nb - u.start;
            uint8_t *dst = is_read ? fixed : s.h_arena + u.data_off;
            R.ev(is_read ? "read" : "read_prefix", k, i, n);
            const auto t0 = Clock::now();
            int st = u.err == CDC_OK ? read_exact(R.paths[u.file], dst, off, n) : CDC_OK;
            if (is_read && R.fail_file == int64_t(u.file) && R.fail_piece == int64_t(u.piece)) st = CDC_E_IO;
            read_s += secs(t0, Clock::now());
            R.ev("read_end", k, i, n);
            {
                std::lock_guard<std::mutex> lk(R.mu);
                if (st != CDC_OK) {
                    u.err = st;
                    u.len = 0;
                    if (F.err == CDC_OK) F.err = st;
                }
                // a later piece is read once its prefix is in too
                const bool whole = is_prefix || u.piece == 0;
                if (whole && ++s.nread == b.u1 - b.u0) s.read_done = true;
                if (is_read && u.piece > 0) R.prefix_q.insert(i);
                --R.reading;
                // hashes go in unit order (batch order, largest file first),
                // not in the order reads end: a large file's read ends late
                if (is_read) R.hash_q.insert(i);
            }
            R.cv.notify_all();
            continue;
        }
        const auto t1 = Clock::now();
        {
            bool go;
            {
                std::lock_guard<std::mutex> lk(R.mu);
                go = u.err == CDC_OK && (u.pieces == 1 || F.err == CDC_OK);
            }
            if (go && u.pieces == 1) {
                cdc::sha256(fixed, u.ne, F.obj);
            } else if (go) {  // the bytes this piece adds: [nb, ne) of the file
                F.sha.update(fixed, size_t(u.ne - u.nb));
                if (u.piece + 1 == u.pieces) F.sha.final(F.obj);
            }
        }
        const double dt = secs(t1, Clock::now());
        hash_s += dt;
        R.ev("hash_end", k, i, u.len);
        {
            std::lock_guard<std::mutex> lk(R.mu);
            F.chain_s += dt;
            if (u.pieces > 1) F.hashed_pieces = u.piece + 1;
            if (++s.nhashed == b.u1 - b.u0) {
                s.hash_done = true;
                maybe_release(R, s);
            }
        }
        R.cv.notify_all();
    }
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.read_s += read_s;
    R.st.objhash_s += hash_s;
}

// The packer's packfile, serialized in place, to PutPackfile (on_pack).
int sink(Run &R, cdc_packer *p)
{
    const uint8_t *data = nullptr;
    uint64_t len = 0;
    const int st = cdc::packer_seal(p, R.o.timestamp, &data, &len);
    if (st != CDC_OK) return st;
    R.ev("packfile", -1, -1, len);
    std::lock_guard<std::mutex> lk(R.sink_mu);
    ++R.st.packfiles;
    R.st.packed_bytes += len;
    return R.on_pack ? R.on_pack(R.ctx, data, len) : CDC_OK;
}

void packer_main(Run &R, cdc_packer *p)
{
    cdc_packer_reset(p);
    double busy = 0;
    for (;;) {
        Blob b;
        {
            std::unique_lock<std::mutex> lk(R.mu);
            R.cv.wait(lk, [&] { return !R.queue.empty() || R.stop_packers || R.status.load() != CDC_OK; });
            if (R.queue.empty()) break;
            b = R.queue.front();
            R.queue.pop_front();
        }
        const auto t0 = Clock::now();
        int st = R.status.load() == CDC_OK ? cdc_packer_add_blob(p, 1 /* TYPE_CHUNK */, b.sum.b, b.data, b.len) : 0;
        if (st == 1) {  // Size() > MaxSize: packerJob flushes (snapshot/snapshot.go:71)
            st = sink(R, p);
            cdc_packer_reset(p);
        }
        busy += secs(t0, Clock::now());
        if (st < 0) R.fail(st);
        {
            std::lock_guard<std::mutex> lk(R.mu);
            Slot &s = R.B->slot[b.slot];
            --s.pending;
            maybe_release(R, s);
        }
    }
    const auto t0 = Clock::now();
    if (R.status.load() == CDC_OK && cdc_packer_count(p)) {  // the last, partial packfile
        const int st = sink(R, p);
        if (st < 0) R.fail(st);
    }
    busy += secs(t0, Clock::now());
    cdc_packer_reset(p);
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.pack_s += busy;
}

int random_bytes(uint8_t *p, size_t n)
{
    while (n) {
        const ssize_t k = getrandom(p, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return CDC_E_IO;
        p += k;
        n -= size_t(k);
    }
    return CDC_OK;
}

// Object.Entropy (snapshot/backup.go:612-627, 668-670): totalEntropy +=
// entropy * float64(len) over the chunks in order, then / float64(size); one
// IEEE operation at a time.
// The running sum continues across the pieces of a large file (chunk order is
// file order); the caller divides by the size after the last piece.
#pragma clang fp contract(off)
void object_entropy_add(double &acc, bool &any, const double *e, const cdc_cut *cuts, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) {
        const double t = e[i] * double(cuts[i].length);
        acc = any ? acc + t : t;
        any = true;
    }
}
#pragma clang fp contract(on)

const uint8_t kEmptySum[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                               0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                               0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};  // SHA-256("")

// Stage A on stream 1, enqueued as soon as the batch's bytes are in its slot
// (it runs beside the previous batch's digests and Encode: the copy engine
// and a short scan): H2D, cut points of every non-empty file (a file < Min is
// one chunk, as chunkify routes it: the Algorithm returns n for n <= Min).
int enqueue_cuts(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    const Batch &b = R.batches[k];
    const cdc_opts *co = &R.o.chunking;
    const uint32_t nf = b.u1 - b.u0;
    hipStream_t st1 = R.B->stream[kA], sh = R.B->stream[kH];
    const auto w0 = Clock::now();
    R.ev("enq_cuts", int64_t(k), -1, b.bytes);
    // H2D on its own stream: batch k + 1's copy does not wait behind batch
    // k's scan (which waits for CUs beside the digest launches)
    HIPOK(hipEventRecord(s.ev[0], sh));
    HIPOK(hipMemcpyAsync(s.d_in, s.h_arena, b.bytes, hipMemcpyHostToDevice, sh));
    HIPOK(hipEventRecord(s.ev[1], sh));
    HIPOK(hipStreamWaitEvent(st1, s.ev[1], 0));
    std::vector<const void *> dp(nf);
    std::vector<uint64_t> caps(nf);
    std::vector<cdc_cut *> cp(nf);
    std::vector<cdc_result *> rp(nf);
    s.lens.assign(nf, 0);
    s.cut0.assign(nf, 0);
    uint64_t c = 0;
    for (uint32_t j = 0; j < nf; ++j) {
        const Unit &u = R.units[b.u0 + j];
        dp[j] = s.d_in + u.data_off;
        s.lens[j] = u.len;  // 0 for a file that failed (no chunk) and for an empty one (one empty chunk)
        caps[j] = u.len / co->min_size + 2;
        s.cut0[j] = c;
        cp[j] = s.d_cuts + c;
        rp[j] = s.d_res + j;
        c += caps[j];
    }
    s.ncut = c;
    // a piece before a file's last is chunked non-final (plan() puts it alone
    // in its batch): its cut list stops at the last chunk whose window lies
    // inside the piece, and the rest is carried into the next piece
    const Unit &u0 = R.units[b.u0];
    const int final_ = u0.piece + 1 < u0.pieces ? 0 : 1;
    // test hook: this piece's launch group takes the forced device abort
    cdc::t_force_abort = R.fail_dev_file == int64_t(u0.file) && R.fail_dev_piece == int64_t(u0.piece) ? 1 : 0;
    for (uint32_t g = 0; g < nf; g += cdc::kMaxBufsPerLaunch) {
        const int m = int(std::min<uint32_t>(cdc::kMaxBufsPerLaunch, nf - g));
        const int st = cdc_chunk_device_batch_async(R.B->device, dp.data() + g, s.lens.data() + g, m, final_, co,
                                                    cp.data() + g, caps.data() + g, rp.data() + g, s.d_ws, s.ws_cap,
                                                    st1);
        if (st != CDC_OK) {
            cdc::t_force_abort = 0;
            return st;
        }
    }
    cdc::t_force_abort = 0;
    HIPOK(hipEventRecord(s.ev[2], st1));
    s.t_enq = secs(w0, Clock::now());
    return CDC_OK;
}

// Stage B on stream D (after stage A): the batch's cut lists rewritten as
// one arena-relative list (k_arena_cuts), one digest launch group for every
// chunk of every file (SHA-256 + histograms), entropy per chunk, the lists
// back to pinned memory.  Batch k + 1's stage B is enqueued before batch k's
// Encode (stream E), so the device's digest chains run back to back.
int enqueue_digests(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    const Batch &b = R.batches[k];
    const uint32_t nf = b.u1 - b.u0;
    hipStream_t sd = R.B->stream[kD + int(k & 1)];
    const auto w0 = Clock::now();
    R.ev("enq_digests", int64_t(k));
    HIPOK(hipStreamWaitEvent(sd, s.ev[2], 0));
    for (uint32_t j = 0; j < nf; ++j) {
        s.h_meta[3 * j] = s.cut0[j];
        s.h_meta[3 * j + 1] = s.lens[j] / R.o.chunking.min_size + 2;
        s.h_meta[3 * j + 2] = R.units[b.u0 + j].data_off;
    }
    const uint64_t c = s.ncut;
    HIPOK(hipEventRecord(s.ev[3], sd));
    HIPOK(hipMemcpyAsync(s.d_meta, s.h_meta, 24ull * nf, hipMemcpyHostToDevice, sd));
    int st = cdc::launch_arena_cuts(s.d_meta, nf, s.d_res, s.d_cuts, s.d_acuts, sd);
    if (st != CDC_OK) return st;
    st = cdc_chunk_digests_device_async(R.B->device, s.d_in, b.bytes, s.d_acuts, c, nullptr, s.d_dig, s.d_hist, sd);
    if (st != CDC_OK) return st;
    if ((st = cdc_chunk_entropy_device_async(R.B->device, s.d_hist, c, s.d_ent, sd)) != CDC_OK) return st;
    HIPOK(hipEventRecord(s.ev[4], sd));
    HIPOK(hipMemcpyAsync(s.h_res, s.d_res, nf * sizeof(cdc_result), hipMemcpyDeviceToHost, sd));
    HIPOK(hipMemcpyAsync(s.h_cuts, s.d_cuts, c * sizeof(cdc_cut), hipMemcpyDeviceToHost, sd));
    HIPOK(hipMemcpyAsync(s.h_dig, s.d_dig, c * 32, hipMemcpyDeviceToHost, sd));
    HIPOK(hipMemcpyAsync(s.h_hist, s.d_hist, c * 1024, hipMemcpyDeviceToHost, sd));
    HIPOK(hipMemcpyAsync(s.h_ent, s.d_ent, c * 8, hipMemcpyDeviceToHost, sd));
    HIPOK(hipEventRecord(s.ev[5], sd));
    s.t_enq += secs(w0, Clock::now());
    return CDC_OK;
}

int wait_pumping(Run &R, hipEvent_t ev, size_t k);

// Batch k once its lists are back: dedup (BlobExists: the run's own chunks and
// the caller's known digests), Encode of the new chunks on stream E, the
// encoded blobs back, the blobs to the packers.
int finish_device(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    const Batch &b = R.batches[k];
    const uint32_t nf = b.u1 - b.u0;
    const auto w0 = Clock::now();
    R.ev("finish_dev", int64_t(k));
    int st = wait_pumping(R, s.ev[5], k);
    if (st != CDC_OK) return st;
    R.ev("lists_back", int64_t(k));
    if (R.trace_path && R.trace_ref) {  // the device stages of batch k on the trace's clock
        static const char *const kDevEv[6] = {"dev_h2d", "dev_h2d_end", "dev_cuts_end", "dev_dig", "dev_dig_end",
                                              "dev_back_end"};
        for (int e = 0; e < 6; ++e) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, R.trace_ref, s.ev[e]) == hipSuccess) R.ev(kDevEv[e], int64_t(k), -1, 0, ms * 1e-3);
        }
    }
    int piece_err = CDC_OK;
    {  // a non-final piece: publish where the next piece starts (its reader waits for it)
        const Unit &u = R.units[b.u0];
        if (u.piece + 1 < u.pieces) {
            std::lock_guard<std::mutex> lk(R.mu);
            FileState &F = R.files[u.file];
            if (u.err == CDC_OK && s.h_res[0].status == CDC_OK) {
                F.next_start = u.start + s.h_res[0].consumed;
                // a piece of P >> Max bytes always emits a chunk; the carry is < Max
                if (F.next_start <= u.start || u.ne - F.next_start >= R.o.chunking.max_size) piece_err = CDC_E_DEVICE;
            } else if (u.err == CDC_OK) {  // the device row failed: no carry to publish
                piece_err = s.h_res[0].status < 0 ? int(s.h_res[0].status) : CDC_E_DEVICE;
            }
            // the next piece's reader sees the failure before it takes a prefix
            if (piece_err != CDC_OK && F.err == CDC_OK) F.err = piece_err;
            F.dev_pieces = u.piece + 1;
        }
    }
    R.cv.notify_all();
    if (piece_err != CDC_OK) return piece_err;
    float t[4] = {};  // H2D, cut points, digests + entropy, lists back
    HIPOK(hipEventElapsedTime(&t[0], s.ev[0], s.ev[1]));
    HIPOK(hipEventElapsedTime(&t[1], s.ev[1], s.ev[2]));
    HIPOK(hipEventElapsedTime(&t[2], s.ev[3], s.ev[4]));
    HIPOK(hipEventElapsedTime(&t[3], s.ev[4], s.ev[5]));
    const Digest *kn = reinterpret_cast<const Digest *>(R.o.known);
    auto known = [&](const Digest &d) {
        return R.o.nknown && std::binary_search(kn, kn + R.o.nknown, d, [](const Digest &a, const Digest &x) {
                   return std::memcmp(a.b, x.b, 32) < 0;
               });
    };
    std::vector<uint64_t> enc_off, enc_len;
    std::vector<Digest> enc_sum;
    std::vector<uint8_t> &is_new = s.is_new;
    std::vector<uint64_t> &file_new0 = s.file_new0;
    is_new.clear();
    file_new0.assign(nf, 0);
    uint64_t enc_bound = 0, nchunks = 0, new_bytes = 0;
    uint64_t nfiles = 0, nbytes = 0, nfailed = 0;
    for (uint32_t j = 0; j < nf; ++j) {
        const cdc_result &r = s.h_res[j];
        const Unit &u = R.units[b.u0 + j];
        if (s.lens[j] && r.status != CDC_OK) return int(r.status);
        file_new0[j] = is_new.size();
        if (u.piece + 1 == u.pieces) {
            ++nfiles;
            nfailed += u.err != CDC_OK ? 1 : 0;
        }
        if (u.err == CDC_OK) nbytes += u.ne - u.nb;
        // an empty file is one empty chunk (backup.go:631-635); a file that
        // failed has none
        const uint64_t cn = s.lens[j] ? r.ncuts : u.err == CDC_OK ? 1 : 0;
        for (uint64_t q = 0; q < cn; ++q) {
            Digest d;
            uint64_t off = 0, len = 0;
            if (s.lens[j]) {
                const cdc_cut &cc = s.h_cuts[s.cut0[j] + q];
                std::memcpy(d.b, s.h_dig + 32 * (s.cut0[j] + q), 32);
                off = u.data_off + cc.offset;
                len = cc.length;
            } else {
                std::memcpy(d.b, kEmptySum, 32);
            }
            const bool fresh = !known(d) && R.seen.insert(d).second;
            is_new.push_back(fresh ? 1 : 0);
            if (fresh) {
                enc_off.push_back(off);
                enc_len.push_back(len);
                enc_sum.push_back(d);
                enc_bound += cdc_encode_bound(len, R.o.compress, R.o.key != nullptr);
                new_bytes += len;
            }
        }
        nchunks += cn;
    }
    const uint32_t nb = uint32_t(enc_off.size());
    const bool encode = nb && (R.o.compress || R.o.key);
    {
        // The new chunks go to the encoder threads (Encode, then the encoded
        // blobs back, then the packers), so this thread goes on driving the
        // next batches instead of waiting out Encode; the slot stays held
        // until its blobs are packed.
        std::lock_guard<std::mutex> lk(R.mu);
        if (encode) {
            R.enc_q.push_back(EncJob{k, std::move(enc_off), std::move(enc_len), std::move(enc_sum), enc_bound});
        } else {
            for (uint32_t q = 0; q < nb; ++q)
                R.queue.push_back(Blob{enc_sum[q], s.h_arena + enc_off[q], enc_len[q], int(k % kSlots)});
        }
        s.pending += nb;
    }
    R.cv.notify_all();
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.batches += 1;
    R.st.files += nfiles;
    R.st.failed_files += nfailed;
    R.st.pieces += nf;
    R.st.bytes += nbytes;
    R.st.chunks += nchunks;
    R.st.new_blobs += nb;
    R.st.new_bytes += new_bytes;
    if (!encode) R.st.encoded_bytes += new_bytes;
    R.st.h2d_s += t[0] * 1e-3;
    R.st.chunk_s += t[1] * 1e-3;
    R.st.digest_s += t[2] * 1e-3;
    R.st.d2h_s += t[3] * 1e-3;
    R.st.device_s += s.t_enq + secs(w0, Clock::now());
    return CDC_OK;
}

// The encoder threads (two, each with its own stream and Encode workspace,
// taking batches in turn): a batch's new chunks through Encode (LZ4 frame +
// AES-256-GCM on the device), the encoded blobs back to pinned memory, then
// to the packers.  The copy back of one batch (~10 ms for 512 MiB over PCIe)
// overlaps the next batch's Encode kernels; with one thread the batches'
// Encodes ran end to end and set the end of the run
// (profiles/r04_c4b_trace.txt).
int encode_job(Run &R, EncJob &J, hipStream_t se)
{
    Slot &s = R.B->slot[J.k % kSlots];
    const uint32_t nb = uint32_t(J.off.size());
    int st;
    if ((st = grow_dev(s.d_enc, s.enc_cap, J.bound)) != CDC_OK) return st;
    std::vector<uint8_t> rnd;
    if (R.o.key) {
        rnd.resize(56ull * nb);
        if ((st = random_bytes(rnd.data(), rnd.size())) != CDC_OK) return st;
    }
    std::vector<uint64_t> oo(nb + 1, 0);
    R.ev("encode", int64_t(J.k), -1, J.bound);
    const auto e0 = Clock::now();
    st = cdc_encode_device(R.B->device, s.d_in, J.off.data(), J.len.data(), nb, R.o.compress, R.o.key,
                           R.o.key ? rnd.data() : nullptr, s.d_enc, s.enc_cap, oo.data(), se);
    if (st != CDC_OK) return st;
    const auto e1 = Clock::now();
    if (oo[nb] > s.henc_cap || !s.h_enc) {
        const uint64_t want = std::max<uint64_t>(oo[nb], s.enc_cap);
        if ((st = grow_host(s.h_enc, want, 0)) != CDC_OK) return st;
        s.henc_cap = want;
    }
    HIPOK(hipMemcpyAsync(s.h_enc, s.d_enc, oo[nb], hipMemcpyDeviceToHost, se));
    HIPOK(hipStreamSynchronize(se));
    const auto e2 = Clock::now();
    R.ev("encode_end", int64_t(J.k), -1, oo[nb]);
    {
        std::lock_guard<std::mutex> lk(R.mu);
        for (uint32_t q = 0; q < nb; ++q)
            R.queue.push_back(Blob{J.sum[q], s.h_enc + oo[q], oo[q + 1] - oo[q], int(J.k % kSlots)});
    }
    R.cv.notify_all();
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.encoded_bytes += oo[nb];
    R.st.encode_s += secs(e0, e1);
    R.st.d2h_s += secs(e1, e2);
    return CDC_OK;
}

void encoder_main(Run &R, int idx)
{
    if (hipSetDevice(R.B->device) != hipSuccess) {
        R.fail(CDC_E_DEVICE);
        return;
    }
    cdc::t_encode_ws = idx;
    hipStream_t se = R.B->stream[idx ? kE + 2 : kE];
    for (;;) {
        EncJob J;
        {
            std::unique_lock<std::mutex> lk(R.mu);
            R.cv.wait(lk, [&] { return !R.enc_q.empty() || R.stop_encoder || R.status.load() != CDC_OK; });
            if (R.enc_q.empty() || R.status.load() != CDC_OK) return;
            J = std::move(R.enc_q.front());
            R.enc_q.pop_front();
        }
        int st;
        try {
            st = encode_job(R, J, se);
        } catch (const std::bad_alloc &) {
            st = CDC_E_NOMEM;
        }
        if (st != CDC_OK) {
            R.fail(st);
            return;
        }
    }
}

// Batch k's per-file callbacks (the Object's fields), on the callback thread
// while the calling thread drives the next batches through the device; the
// slot is released once its blobs are packed too.
int finish_host(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    const Batch &b = R.batches[k];
    const uint32_t nf = b.u1 - b.u0;
    {
        std::unique_lock<std::mutex> lk(R.mu);  // the batch's lists + dedup, and every object checksum
        R.cv.wait(lk, [&] { return (R.devices_done > k && s.hash_done) || R.status.load() != CDC_OK; });
    }
    if (R.status.load() != CDC_OK) return R.status.load();
    const auto cb0 = Clock::now();
    R.ev("callbacks", int64_t(k));
    if (R.on_file) {
        static const cdc_cut kEmptyCut = {0, 0, 0};
        static const uint32_t kZeroHist[256] = {};
        static const double kZeroEnt[1] = {0.0};
        for (uint32_t j = 0; j < nf; ++j) {
            const Unit &u = R.units[b.u0 + j];
            FileState &F = R.files[u.file];
            cdc_backup_file f;
            std::memset(&f, 0, sizeof(f));
            f.index = int(u.file);
            f.piece = u.piece;
            f.pieces = u.pieces;
            f.size = F.size;
            const bool last = u.piece + 1 == u.pieces;
            int err;
            {
                std::lock_guard<std::mutex> lk(R.mu);
                err = u.err != CDC_OK ? u.err : (last ? F.err : CDC_OK);
            }
            f.status = err;
            if (u.err != CDC_OK) {  // no chunk: the file (or this piece of it) could not be read
                f.nchunks = 0;
            } else if (s.lens[j] == 0) {
                f.nchunks = 1;
                f.cuts = &kEmptyCut;
                f.digests = kEmptySum;
                f.hists = kZeroHist;
                f.entropy = kZeroEnt;
            } else {
                f.nchunks = s.h_res[j].ncuts;
                cdc_cut *c = s.h_cuts + s.cut0[j];
                if (u.start)  // file-relative offsets for a piece after the first
                    for (uint64_t q = 0; q < f.nchunks; ++q) c[q].offset += u.start;
                f.cuts = c;
                f.digests = s.h_dig + 32 * s.cut0[j];
                f.hists = s.h_hist + 256 * s.cut0[j];
                f.entropy = s.h_ent + s.cut0[j];
                object_entropy_add(F.ent_acc, F.ent_any, f.entropy, f.cuts, f.nchunks);
            }
            f.is_new = s.is_new.data() + s.file_new0[j];
            if (u.err == CDC_OK) {  // the piece's bytes in the slot's arena (still held: the slot is not released yet)
                f.data = s.h_arena + u.data_off;
                f.data_offset = u.start;
                f.data_len = u.len;
            }
            if (last && err == CDC_OK) {
                std::memcpy(f.checksum, F.obj, 32);
                f.object_entropy = F.size ? F.ent_acc / double(F.size) : 0.0;
            }
            R.on_file(R.ctx, &f);
        }
    }
    {
        std::lock_guard<std::mutex> lk(R.mu);
        s.device_done = true;
        maybe_release(R, s);
    }
    R.cv.notify_all();
    R.ev("callbacks_end", int64_t(k));
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.callback_s += secs(cb0, Clock::now());
    return CDC_OK;
}

void callback_main(Run &R)
{
    for (size_t k = 0; k < R.batches.size(); ++k) {
        const int st = finish_host(R, k);
        if (st != CDC_OK) {
            R.fail(st);
            return;
        }
    }
}

// Wait until batch k's bytes are in its slot (the reader's signal).
int wait_read(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    const auto t0 = Clock::now();
    {
        std::unique_lock<std::mutex> lk(R.mu);
        R.cv.wait(lk, [&] { return (s.batch == int(k) && s.read_done) || R.status.load() != CDC_OK; });
    }
    std::lock_guard<std::mutex> lk(R.stat_mu);
    R.st.read_wait_s += secs(t0, Clock::now());
    return R.status.load();
}

bool read_ready(Run &R, size_t k)
{
    Slot &s = R.B->slot[k % kSlots];
    std::lock_guard<std::mutex> lk(R.mu);
    return s.batch == int(k) && s.read_done;
}

// While batch k is on the device: stage A of every later batch whose bytes
// are in (slots permitting) and stage B of batch k + 1 once its stage A is
// enqueued, so the device never waits for the calling thread.
int pump(Run &R, size_t k)
{
    const size_t nb = R.batches.size();
    int st = CDC_OK;
    while (st == CDC_OK && R.cuts < nb && R.cuts < k + kSlots && read_ready(R, R.cuts))
        if ((st = enqueue_cuts(R, R.cuts)) == CDC_OK) ++R.cuts;
    if (st == CDC_OK && R.digs == k + 1 && R.cuts > k + 1 && (st = enqueue_digests(R, k + 1)) == CDC_OK) ++R.digs;
    return st;
}

// Wait for an event of batch k's, pumping the pipeline meanwhile.
int wait_pumping(Run &R, hipEvent_t ev, size_t k)
{
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return CDC_OK;
        if (q != hipErrorNotReady) return CDC_E_DEVICE;
        const int st = pump(R, k);
        if (st != CDC_OK) return st;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

}  // namespace

extern "C" {

int cdc_backup_new(int device, const cdc_backup_opts *opts, cdc_backup **out)
{
    if (!opts || !out) return CDC_E_INVALID;
    *out = nullptr;
    int st = cdc_validate("fastcdc", &opts->chunking);
    if (st != CDC_OK) return st;
    if (opts->nknown && !opts->known) return CDC_E_INVALID;
    if (!cdc::device_count_initialised()) return CDC_E_NOT_INIT;
    auto *b = new (std::nothrow) cdc_backup();
    if (!b) return CDC_E_NOMEM;
    try {
        b->device = device;
        b->o = *opts;
        if (opts->key) {
            b->key.assign(opts->key, opts->key + 32);
            b->o.key = b->key.data();
        }
        if (opts->nknown) {
            b->known.assign(opts->known, opts->known + 32 * opts->nknown);
            b->o.known = b->known.data();
        }
    } catch (...) {
        delete b;
        return CDC_E_NOMEM;
    }
    if (const char *q = std::getenv("GPU_MAX_HW_QUEUES")) b->hw_queues = std::atoi(q);
    bool ok = hipSetDevice(device) == hipSuccess;
    // Every stream non-blocking.  Round 4 put the two digest streams on every
    // other CU (hipExtStreamCreateWithCUMask); measured in round 5, the mask
    // does not restrict placement on this ROCm (a masked stream's workgroups
    // ran on all 256 CUs) and such a stream blocks on the legacy null stream
    // (profiles/r05final_cu_mask_probe.txt, tools/cu_mask_probe.hip); c4b was the
    // same either way (profiles/r05_c4b_cu_mask_ab.txt), so it is gone.
    for (int i = 0; i < int(sizeof(b->stream) / sizeof(b->stream[0])); ++i)
        ok = ok && hipStreamCreateWithFlags(&b->stream[i], hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        cdc_backup_free(b);
        return CDC_E_DEVICE;
    }
    *out = b;
    return CDC_OK;
}

int cdc_backup_files(cdc_backup *B, const char *const *paths, int n, cdc_backup_file_fn on_file,
                     cdc_backup_pack_fn on_pack, void *ctx, cdc_backup_stats *stats)
{
    if (!B || n < 0 || (n && !paths)) return CDC_E_INVALID;
    const auto w0 = Clock::now();
    struct ScanMode {  // this thread's scans (workspace sizing and launches) persistent for the call
        int prev = cdc::t_scan_tpw;
        ScanMode() { cdc::t_scan_tpw = kBackupScanTpw; }
        ~ScanMode() { cdc::t_scan_tpw = prev; }
    } scan_mode;
    Run *Rp = new (std::nothrow) Run(B, paths, n);
    if (!Rp) return CDC_E_NOMEM;
    Run &R = *Rp;
    R.on_file = on_file;
    R.on_pack = on_pack;
    R.ctx = ctx;
    int st = CDC_OK;
    std::vector<std::thread> readers, packers;
    std::thread callbacks;
    std::vector<std::thread> encoders;
    try {
        uint64_t arena = 0, ncuts = 0, ws = 0, nfiles = 0;
        st = plan(R, arena, ncuts, ws, nfiles);
        R.st.slot_arena_bytes = arena;
        R.ev("planned", -1, -1, uint64_t(R.batches.size()));
        if (st == CDC_OK && hipSetDevice(B->device) != hipSuccess) st = CDC_E_DEVICE;
        if (st == CDC_OK && R.trace_path) {
            if (hipEventCreate(&R.trace_ref) != hipSuccess || hipEventRecord(R.trace_ref, B->stream[kA]) != hipSuccess ||
                hipEventSynchronize(R.trace_ref) != hipSuccess)
                R.trace_ref = nullptr;
            R.ev("trace_ref", -1);
        }
        for (int i = 0; i < kSlots && st == CDC_OK && !R.batches.empty(); ++i) {
            st = grow_slot(B->slot[i], arena, ws, ncuts, nfiles);
            B->slot[i].batch = -1;
            B->slot[i].next = i;
            B->slot[i].read_done = B->slot[i].hash_done = B->slot[i].device_done = false;
            B->slot[i].pending = 0;
        }
        if (st == CDC_OK && !R.batches.empty()) {
            const int np = std::max(1, R.o.packers ? R.o.packers : 8);
            while (int(B->packers.size()) < np) {
                cdc_packer *p = nullptr;
                if (cdc_packer_new(R.o.packfile_max ? R.o.packfile_max : (20u << 20), &p) != CDC_OK) {
                    st = CDC_E_NOMEM;
                    break;
                }
                B->packers.push_back(p);
                cdc::packer_reserve(p, cdc_encode_bound(R.o.chunking.max_size, R.o.compress, R.o.key != nullptr));
            }
            if (st != CDC_OK) throw std::bad_alloc();
            const int nr = std::max(1, R.o.readers ? R.o.readers : 8);
            for (int r = 0; r < nr; ++r) readers.emplace_back([&R] { reader_main(R); });
            callbacks = std::thread([&R] { callback_main(R); });
            for (int e = 0; e < kEncoders; ++e) encoders.emplace_back([&R, e] { encoder_main(R, e); });
            for (int p = 0; p < np; ++p) {
                cdc_packer *pk = B->packers[size_t(p)];
                packers.emplace_back([&R, pk] { packer_main(R, pk); });
            }
            // Per batch k: batch k is deduplicated, Encoded and handed to the
            // packers and the callback thread; while this thread waits on
            // the device it pumps (stage A of every later batch whose reads
            // have landed, stage B of batch k + 1).  It waits for a read only
            // when the device would otherwise idle.
            const size_t nb = R.batches.size();
            for (size_t k = 0; k < nb && st == CDC_OK; ++k) {
                if (R.digs == k) {
                    if (R.cuts == k) {
                        if ((st = wait_read(R, k)) != CDC_OK) break;
                        if (k == 0) R.st.fill_s = secs(w0, Clock::now());
                        if ((st = enqueue_cuts(R, k)) != CDC_OK) break;
                        ++R.cuts;
                    }
                    if ((st = enqueue_digests(R, k)) != CDC_OK) break;
                    ++R.digs;
                }
                if ((st = pump(R, k)) != CDC_OK) break;
                if ((st = finish_device(R, k)) != CDC_OK) break;
                R.last_dev_end = secs(w0, Clock::now());
                {
                    std::lock_guard<std::mutex> lk(R.mu);
                    R.devices_done = k + 1;
                }
                R.cv.notify_all();
            }
            {  // every batch is handed over: the encoder drains its queue and stops
                std::lock_guard<std::mutex> lk(R.mu);
                R.stop_encoder = true;
            }
            R.cv.notify_all();
            for (auto &t : encoders) t.join();
            encoders.clear();
            if (st == CDC_OK && callbacks.joinable()) {
                callbacks.join();  // the last slots are released by the callbacks
                st = R.status.load();
            }
            if (st != CDC_OK) R.fail(st);
            {
                std::lock_guard<std::mutex> lk(R.mu);
                R.stop_packers = true;
            }
            R.cv.notify_all();
        }
    } catch (const std::bad_alloc &) {
        st = CDC_E_NOMEM;
        R.fail(st);
    } catch (...) {
        st = CDC_E_DEVICE;
        R.fail(st);
    }
    if (!encoders.empty()) {
        {
            std::lock_guard<std::mutex> lk(R.mu);
            R.stop_encoder = true;
        }
        R.cv.notify_all();
        for (auto &t : encoders) t.join();
    }
    if (callbacks.joinable()) callbacks.join();
    for (auto &t : readers) t.join();
    for (auto &t : packers) t.join();
    if (st == CDC_OK) st = R.status.load();
    if (st != CDC_OK) {  // leave the context reusable: nothing of this run in flight
        for (auto &sm : B->stream) (void)hipStreamSynchronize(sm);
    }
    R.st.wall_s = secs(w0, Clock::now());
    R.st.drain_s = R.last_dev_end > 0 ? R.st.wall_s - R.last_dev_end : 0.0;
    for (const FileState &F : R.files)
        if (F.chain_s > R.st.chain_s) {
            R.st.chain_s = F.chain_s;
            R.st.chain_bytes = F.size;
        }
    R.ev("end", -1);
    if (R.trace_path) {
        if (FILE *f = std::fopen(R.trace_path, "w")) {
            std::fprintf(f, "t_s,event,batch,unit,bytes\n");
            for (const auto &e : R.trace)
                std::fprintf(f, "%.6f,%s,%lld,%lld,%llu\n", e.t, e.what, (long long)e.batch, (long long)e.unit,
                             (unsigned long long)e.bytes);
            std::fclose(f);
        }
        if (R.trace_ref) (void)hipEventDestroy(R.trace_ref);
    }
    R.st.hw_queues = B->hw_queues;
    R.st.streams_serialised = B->hw_queues < 8 ? 1 : 0;
    if (stats) *stats = R.st;
    delete Rp;
    return st;
}

void cdc_backup_free(cdc_backup *b)
{
    if (!b) return;
    for (auto &s : b->stream)
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    for (auto &s : b->slot) free_slot(s);
    for (cdc_packer *p : b->packers) cdc_packer_free(p);
    delete b;
}

int cdc_backup_run(int device, const char *const *paths, int n, const cdc_backup_opts *opts,
                   cdc_backup_file_fn on_file, cdc_backup_pack_fn on_pack, void *ctx, cdc_backup_stats *stats)
{
    cdc_backup *b = nullptr;
    int st = cdc_backup_new(device, opts, &b);
    if (st != CDC_OK) return st;
    st = cdc_backup_files(b, paths, n, on_file, on_pack, ctx, stats);
    cdc_backup_free(b);
    return st;
}

}  // extern "C"
