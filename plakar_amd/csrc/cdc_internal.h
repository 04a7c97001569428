// Internal types shared by the HIP kernels (cdc_kernels.hip) and the C-ABI
// implementation (cdc_api.cpp).  Not part of the public ABI.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "plakar_cdc.h"

namespace cdc {

constexpr int kMaxBufsPerLaunch = 32;   // buffers per launch group (kernel-arg budget)
// A result row's status between the scan kernel and k_resolve's last segment
// (never returned: the last segment or an aborting wave overwrites it).
constexpr int64_t kRowPending = -0x7FF0;
// Batch.debug bit of debug mode 2 (cdc_set_debug_mode): segment 0 of buffer 0
// never publishes its speculative exit, so segment 1's bounded wait gives up
// and the launch aborts (the device-abort path under test).
constexpr uint32_t kDbgForceAbort = 512;
constexpr uint32_t kForceAbortTicks = 20000;  // that mode's spin limit: 200 us
// Candidate index: one u64 record per scan-lane run (scan_lane bytes of one
// buffer): bits 0-7 the number of full-window MaskS candidates in the run
// (saturating), bits 8-63 the first kRunCap of them as 14-bit offsets from the
// run start, ascending.  Written once per run by the lane that scanned it (no
// atomics, no zeroing); runs and their entries are in position order, so the
// index is sorted by construction.  A run with more than kRunCap candidates is
// "dense": walkers rescan its bytes (about 0.2 runs per GiB of random data at
// 0.17 candidates per 5.75-KiB run).
constexpr uint32_t kRunCap = 4;
constexpr uint32_t kRecCntBits = 8, kRecEntBits = 14;
constexpr uint32_t kMaxScanLane = 1u << kRecEntBits;  // run offsets are 14-bit
constexpr uint32_t kMaxSegs = 1u << 22; // resolution segments per buffer (seg grows past 32 Min beyond)
constexpr uint32_t kScanLaneBytes = 16384;  // max bytes hashed+tested per scan lane (multiple of 256, <= kMaxScanLane)
#ifndef CDC_WALK_WAVES
#define CDC_WALK_WAVES 4
#endif
constexpr uint32_t kWalkWavesPerWG = CDC_WALK_WAVES;   // latency-bound walkers: registers over occupancy
constexpr uint64_t kUndet = ~0ull;      // "next chunk start not decided by the bytes present"

// Chunker parameters as the kernels use them.
struct DevParams {
    uint64_t min_size, normal_size, max_size;
    uint32_t ms_lo, ms_hi, ml_lo, ml_hi;  // MaskS / MaskL split in 32-bit halves
    uint32_t cut_adj;                     // 0: cut at i, 1: cut at i + 1
    uint32_t win;                         // W = highest mask bit + 1 (window length)
    // The scan's shifted frame: fp' = fp << fs_sh (fs_sh = 63 - highest MaskS
    // bit) and MaskS << fs_sh split in 32-bit halves (k_scan).
    uint32_t fs_sh, fs_lo, fs_hi;
    // The same frame for MaskL (k_scan_l, the MaskL candidate index).
    uint32_t fl_sh, fl_lo, fl_hi;
    // k_scan_f (both indexes in one pass): its loop rolls fp << fm_sh, the
    // frame whose hi dword holds every bit MaskS and MaskL share, and filters
    // on those bits (fm_mi: a necessary key for a MaskS or a MaskL hit); its
    // recheck rolls the MaskS frame, where MaskL << fs_sh = fm_lhi:fm_llo.
    // fm_ok = 0 (then k_scan + k_scan_l only) when MaskL has a bit above
    // MaskS's highest, or the shared bits are fewer than 8 or span more than
    // 32.
    uint32_t fm_sh, fm_mi, fm_llo, fm_lhi, fm_ok;
};

struct BufDesc {
    const uint8_t *data;
    uint64_t len;
    cdc_cut *out;
    uint64_t cap;
    cdc_result *res;
    uint32_t seg_base;   // first resolution segment (global numbering)
    uint32_t nseg;
    uint32_t task_base;  // first scan task (global numbering)
};

struct Batch {
    uint32_t nbufs;
    uint32_t final_;
    uint32_t total_segs, total_tasks;
    uint32_t force_fallback; // debug: resolve with the sequential single-wave walker
    uint32_t scan_lane;      // bytes per scan lane (= per index run); one wave (scan task) = 64 lanes
    uint32_t debug;          // profiling experiments (CDC_DEBUG_PHASE); 0 in production
    uint32_t spin_ticks;     // bounded waits give up after this many 100-MHz ticks (0: 2 s; debug mode 2: short)
    uint32_t maskl_index;    // 1: k_scan_l builds the MaskL index of long MaskS-free stretches (walkers use it)
    uint32_t maskl_fused;    // 1 (with maskl_index): k_scan_f builds both indexes of every task in one pass
    uint32_t *maskl_hint;    // mapped host word: set when some task needed the MaskL index
    uint32_t maskl_probe;    // 1: k_maskl_probe runs the selection test (adaptive mode, hint not set)
    uint64_t seg;            // resolution segment length in bytes
    uint32_t persist;        // 1: k_scan / k_scan_f run scan_wgs persistent workgroups pulling tasks
    uint32_t scan_wgs;
    BufDesc b[kMaxBufsPerLaunch];
};

// Device workspace, carved out of one caller-provided allocation.
struct Workspace {
    uint64_t *runs;      // [total_tasks * 64] candidate-index records (run q of buffer b at 64 * task_base + q)
    // k_resolve's per-segment words (see cdc_kernels.hip); xg and sg are
    // zeroed by the scan kernel of the same launch group.
    uint64_t *w1_nodes;  // [total_segs * 64] speculative chain of each segment
    uint64_t *xg;        // [total_segs] granule: published | node count | speculative exit X_q
    uint64_t *sg;        // [total_segs] granule: LOCAL (conv, cuts) or INCLUSIVE (E, O)
    uint32_t *flags;     // [kMaxBufsPerLaunch + 4] per-buffer "resolve sequentially", then the abort word
    uint32_t *tick;      // [16] [0] segment ticket, [2] persistent scan task counter
    const uint64_t *gear;  // 256 entries, device copy
    // MaskL candidate index (same record format as runs), built by k_scan_l
    // only for the scan tasks near a long MaskS-free stretch; validL[task]
    // says whether task's 64 records are this launch's (1) or absent (0).
    uint64_t *runsL;     // [total_tasks * 64]
    uint32_t *validL;    // [total_tasks]
};

struct Plan {
    uint64_t seg;            // resolution segment length
    uint32_t scan_lane;
    uint32_t total_segs, total_tasks;
    uint32_t persist, scan_wgs;
    size_t off_runs, off_w1_nodes, off_xg, off_sg, off_flags, off_tick, off_runsL, off_validL,
        bytes;
};

// Host-side helpers implemented in cdc_kernels.hip.
int make_plan(const uint64_t *lens, int nbufs, const DevParams &P, Plan *plan);
int launch_batch(const Batch &B, const DevParams &P, const Workspace &W, void *stream);
// cdc_digest.hip: per-chunk SHA-256 (+ optional byte histogram) of device cut lists.
struct DigestBuf {
    const uint8_t *data;
    uint64_t len;
    const cdc_cut *cuts;
    uint64_t cap;
    const cdc_result *res;  // nullable: count = min(cap, res->ncuts)
    uint8_t *digests;       // 32 B per chunk
    uint32_t *hist;         // 256 u32 per chunk, or null (all or none in one launch)
};
struct DigestBatch {
    uint32_t nbufs;
    uint64_t resident_lanes;  // lanes the device keeps resident at once (set by launch_digests)
    const DigestBuf *ind;     // launch_digests_many: the nbufs descriptors in device memory (b unused)
    DigestBuf b[kMaxBufsPerLaunch];
};
// parts: 1 the SHA-256 kernel only, 2 the histograms only, 3 both
int launch_digests(const DigestBatch &DB, void *stream, int parts = 3);
// cdc_chunk_digests_hybrid's device pieces: pack chunks into a staging buffer
// (dst: 16-B aligned offsets), and write 32-B digests to their rows.
struct GatherJob {
    const uint8_t *src;
    uint64_t len;
    uint64_t dst;
};
struct ScatterJob {
    uint8_t *dst;
    const uint8_t *src;
};
int launch_gather(const GatherJob *d_jobs, uint32_t n, uint8_t *d_stage, void *stream);
// The three stream-read forms over [d_buf, d_buf + len), `reps` launches each (hipEvents): best and
// median microseconds per form (plain, nontemporal, LDS-DMA) in best_us[3] / median_us[3].
int launch_stream_read(const void *d_buf, uint64_t len, int reps, double *best_us, double *median_us, void *stream);
int launch_scatter_digests(const ScatterJob *d_jobs, uint32_t n, void *stream);
// More than kMaxBufsPerLaunch buffers in ONE launch group: the descriptors go
// to device memory through a per-device pinned ring (a launch lasts as long as
// its longest chunk, so several groups of 32 would each pay that tail).
int launch_digests_many(const DigestBuf *bufs, uint32_t nbufs, void *stream);
int launch_entropy(const uint32_t *d_hist, uint64_t rows, double *d_out, void *stream);
int launch_arena_cuts(const uint64_t *d_meta, uint32_t nfiles, const cdc_result *d_res, const cdc_cut *d_cuts,
                      cdc_cut *d_out, void *stream);
extern uint64_t g_digest_lanes;
// The calling thread's scan mode for make_plan: -1 the default (static grid,
// or CDC_SCAN_TASKS_PER_WAVE), k >= 0 the persistent scan with about k tasks
// per wave (0: the static grid).
extern thread_local int t_scan_tpw;
// The calling thread's Encode workspace (0 or 1) for cdc_encode_device.
extern thread_local int t_encode_ws;
// Test hook (the backup's CDC_BACKUP_FAIL_DEVICE): the calling thread's next
// launch groups run in debug mode 2 (the forced device abort) while nonzero.
extern thread_local int t_force_abort;

// cdc_api.cpp: a host-buffer pipeline on one device that outlives one call
// (the collector's per-device worker).  The source hands out batches of at
// most kMaxBufsPerLaunch whole buffers; the pipeline stages batch k + 1 into
// one slot while batch k is chunked in the other, and hands each batch back
// with its cut lists (and a per-buffer status).
struct HostBuf {
    const uint8_t *data;
    uint64_t len;
    std::vector<cdc_cut> cuts;
    int status;
};
struct BatchSource {
    // Fill `batch` and return true, or return false: at once when nothing is
    // ready and !wait, else only once the source is stopping and empty.
    virtual bool next(std::vector<HostBuf *> &batch, bool wait) = 0;
    virtual void finished(std::vector<HostBuf *> &batch) = 0;
    virtual ~BatchSource() = default;
};
int pipeline_device(int dev_index, const cdc_opts *o, BatchSource &src);
int device_count_initialised();

// cdc_sha256.cpp: host SHA-256 (x86 SHA extensions when present).
struct Sha256 {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint8_t buf[64];
    uint64_t total = 0;
    size_t fill = 0;
    bool force_scalar = false;
    void blocks(const uint8_t *p, size_t nblocks);
    void update(const uint8_t *p, size_t n);
    void final(uint8_t out[32]);
};
void sha256(const void *data, size_t n, uint8_t out[32], bool force_scalar = false);
bool sha256_accelerated();

// cdc_packer.cpp: in-place serialization for the backup pipeline's sinks
int packer_seal(cdc_packer *p, int64_t timestamp, const uint8_t **data, uint64_t *len);
void packer_reserve(cdc_packer *p, uint64_t max_blob);

}  // namespace cdc
