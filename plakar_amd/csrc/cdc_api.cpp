// C-ABI implementation of libplakar_cdc.so (see include/plakar_cdc.h).
//
// Host runtime around the HIP kernels: per-device contexts (Gear table in
// device memory, a stream, pinned staging + device arenas for the host-buffer
// path), the batch / device-resident entry points, and the streaming chunker
// that mirrors ext go-cdc-chunkers (*Chunker).Next.  No CPU chunking fallback
// exists: without a device every compute entry point fails with a status.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "cdc_internal.h"

using namespace cdc;

namespace {

constexpr uint64_t kDefaultMaskS = 0x0003590703530000ull;  // FastCDC paper MaskS (15 bits)
constexpr uint64_t kDefaultMaskL = 0x0000d90003530000ull;  // FastCDC paper MaskL (11 bits)

// One in-flight launch group of the host-buffer path: device input, workspace,
// cut lists and results, plus the event that marks its results as copied back.
struct Slot {
    uint8_t *d_in = nullptr;
    uint64_t in_cap = 0;
    void *d_ws = nullptr;
    uint64_t ws_cap = 0;
    cdc_cut *d_cuts = nullptr;
    cdc_cut *h_cuts = nullptr;
    uint64_t cuts_cap = 0;
    cdc_result *d_res = nullptr;
    cdc_result *h_res = nullptr;
    hipEvent_t staged = nullptr;  // copy stream: input bytes are on the device
    hipEvent_t done = nullptr;    // compute stream: results are in h_res / h_cuts
};

constexpr int kBounces = 2;

struct DeviceCtx {
    int device = -1;
    uint64_t *d_gear = nullptr;
    hipStream_t stream = nullptr;  // kernels + result copies
    hipStream_t copy = nullptr;    // host -> device input copies
    std::mutex mu;
    Slot slot[2];
    uint8_t *bounce[kBounces] = {nullptr, nullptr};  // pinned staging for H2D
    uint64_t bounce_cap = 0;
    hipEvent_t bounce_ev[kBounces] = {nullptr, nullptr};
    int next_bounce = 0;
    // Adaptive MaskL index (run_group): k_maskl_probe / k_scan_l raise *hint_h
    // (mapped host memory) when some scan task needs the index; groups build it
    // while the hint is set, and every 16th group probes when it is not.
    uint32_t *hint_h = nullptr, *hint_d = nullptr;
    std::atomic<uint64_t> groups{0};
};

struct Global {
    std::mutex mu;
    // Set (release) once the contexts and the Gear table are in place; entry
    // points read it (acquire) without the lock.  g.devs changes only inside
    // cdc_init / cdc_shutdown, which must not race with other calls.
    std::atomic<bool> init{false};
    bool placeholder_gear = true;
    uint64_t gear[256];
    uint64_t mask_s = kDefaultMaskS, mask_l = kDefaultMaskL;
    uint32_t cut_adj = 0;
    int debug_mode = 0;
    std::vector<DeviceCtx *> devs;
};

Global &G()
{
    static Global g;
    return g;
}

// MaskL index mode (cdc_set_maskl_index_mode; initial value from CDC_MASKL_INDEX)
std::atomic<uint32_t> &maskl_index_mode()
{
    static std::atomic<uint32_t> m([] {
        const char *e = getenv("CDC_MASKL_INDEX");
        return e && (e[0] == '0' || e[0] == '2' || e[0] == '3') ? uint32_t(e[0] - '0') : 1u;
    }());
    return m;
}

uint64_t splitmix64(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

std::string lower(const char *s)
{
    std::string r = s ? s : "";
    for (auto &c : r) c = char(std::tolower((unsigned char)c));
    return r;
}

int validate_sizes(const cdc_opts *o)
{
    // ext chunkers/fastcdc (*FastCDC).Validate: 64 B <= sizes <= 1 GiB, Min < Normal < Max
    const uint64_t lo = 64, hi = 1ull << 30;
    if (o->normal_size < lo || o->normal_size > hi) return CDC_E_NORMAL_SIZE;
    if (o->min_size < lo || o->min_size > hi || o->min_size >= o->normal_size) return CDC_E_MIN_SIZE;
    if (o->max_size < lo || o->max_size > hi || o->max_size <= o->normal_size) return CDC_E_MAX_SIZE;
    return CDC_OK;
}

DevParams make_params(const cdc_opts *o)
{
    Global &g = G();
    DevParams P;
    P.min_size = o->min_size;
    P.normal_size = o->normal_size;
    P.max_size = o->max_size;
    P.ms_lo = uint32_t(g.mask_s);
    P.ms_hi = uint32_t(g.mask_s >> 32);
    P.ml_lo = uint32_t(g.mask_l);
    P.ml_hi = uint32_t(g.mask_l >> 32);
    P.cut_adj = g.cut_adj;
    const uint64_t m = g.mask_s | g.mask_l;
    P.win = 64u - uint32_t(__builtin_clzll(m));
    P.fs_sh = uint32_t(__builtin_clzll(g.mask_s));  // 63 - highest MaskS bit
    const uint64_t ms = g.mask_s << P.fs_sh;
    P.fs_lo = uint32_t(ms);
    P.fs_hi = uint32_t(ms >> 32);
    P.fl_sh = g.mask_l ? uint32_t(__builtin_clzll(g.mask_l)) : 0u;  // 63 - highest MaskL bit
    P.fm_sh = P.fm_mi = P.fm_llo = P.fm_lhi = P.fm_ok = 0u;
    const uint64_t mi = g.mask_s & g.mask_l;  // the bits both masks test
    // under 8 shared bits the filter fires on most groups: two passes
    // (k_scan + k_scan_l) are cheaper then
    if (g.mask_l && __builtin_clzll(g.mask_l) >= int(P.fs_sh) && __builtin_popcountll(mi) >= 8) {
        const uint32_t lb = uint32_t(__builtin_ctzll(mi)), hb = 63u - uint32_t(__builtin_clzll(mi));
        if (hb - lb <= 31u) {
            P.fm_sh = lb < 32u ? 32u - lb : 0u;  // the lowest shared bit to bit 32 (hb + fm_sh <= 63)
            P.fm_mi = uint32_t((mi << P.fm_sh) >> 32);
            const uint64_t lf = g.mask_l << P.fs_sh;  // keeps every bit (the clz test)
            P.fm_llo = uint32_t(lf);
            P.fm_lhi = uint32_t(lf >> 32);
            P.fm_ok = 1u;
        }
    }
    const uint64_t ml = g.mask_l << P.fl_sh;
    P.fl_lo = uint32_t(ml);
    P.fl_hi = uint32_t(ml >> 32);
    return P;
}

#define HIPCHK(x)                            \
    do {                                     \
        if ((x) != hipSuccess) return CDC_E_DEVICE; \
    } while (0)

void free_slot(Slot &sl)
{
    if (sl.d_in) (void)hipFree(sl.d_in);
    if (sl.d_ws) (void)hipFree(sl.d_ws);
    if (sl.d_cuts) (void)hipFree(sl.d_cuts);
    if (sl.h_cuts) (void)hipHostFree(sl.h_cuts);
    if (sl.d_res) (void)hipFree(sl.d_res);
    if (sl.h_res) (void)hipHostFree(sl.h_res);
    if (sl.staged) (void)hipEventDestroy(sl.staged);
    if (sl.done) (void)hipEventDestroy(sl.done);
    sl = Slot();
}

void free_ctx_buffers(DeviceCtx *c)
{
    for (auto &sl : c->slot) free_slot(sl);
    for (int k = 0; k < kBounces; ++k) {
        if (c->bounce[k]) (void)hipHostFree(c->bounce[k]);
        if (c->bounce_ev[k]) (void)hipEventDestroy(c->bounce_ev[k]);
        c->bounce[k] = nullptr;
        c->bounce_ev[k] = nullptr;
    }
    c->bounce_cap = 0;
}

// Grow a slot's buffers; the slot must be idle (its last group harvested).
int grow_slot(Slot &sl, uint64_t in_bytes, uint64_t ws_bytes, uint64_t ncuts)
{
    if (!sl.staged) HIPCHK(hipEventCreateWithFlags(&sl.staged, hipEventDisableTiming));
    if (!sl.done) HIPCHK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    if (in_bytes > sl.in_cap) {
        if (sl.d_in) (void)hipFree(sl.d_in);
        sl.d_in = nullptr;
        sl.in_cap = 0;
        HIPCHK(hipMalloc(reinterpret_cast<void **>(&sl.d_in), in_bytes));
        sl.in_cap = in_bytes;
    }
    if (ws_bytes > sl.ws_cap) {
        if (sl.d_ws) (void)hipFree(sl.d_ws);
        sl.d_ws = nullptr;
        sl.ws_cap = 0;
        HIPCHK(hipMalloc(&sl.d_ws, ws_bytes));
        sl.ws_cap = ws_bytes;
    }
    if (ncuts > sl.cuts_cap) {
        if (sl.d_cuts) (void)hipFree(sl.d_cuts);
        if (sl.h_cuts) (void)hipHostFree(sl.h_cuts);
        sl.d_cuts = sl.h_cuts = nullptr;
        sl.cuts_cap = 0;
        HIPCHK(hipMalloc(reinterpret_cast<void **>(&sl.d_cuts), ncuts * sizeof(cdc_cut)));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&sl.h_cuts), ncuts * sizeof(cdc_cut),
                             hipHostMallocDefault));
        sl.cuts_cap = ncuts;
    }
    if (!sl.d_res) {
        HIPCHK(hipMalloc(reinterpret_cast<void **>(&sl.d_res), kMaxBufsPerLaunch * sizeof(cdc_result)));
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&sl.h_res),
                             kMaxBufsPerLaunch * sizeof(cdc_result), hipHostMallocDefault));
    }
    return CDC_OK;
}

int grow_bounce(DeviceCtx *c, uint64_t bytes)
{
    if (bytes <= c->bounce_cap) return CDC_OK;
    HIPCHK(hipStreamSynchronize(c->copy));
    for (int k = 0; k < kBounces; ++k) {
        if (c->bounce[k]) (void)hipHostFree(c->bounce[k]);
        c->bounce[k] = nullptr;
    }
    c->bounce_cap = 0;
    for (int k = 0; k < kBounces; ++k) {
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->bounce[k]), bytes, hipHostMallocDefault));
        if (!c->bounce_ev[k]) HIPCHK(hipEventCreateWithFlags(&c->bounce_ev[k], hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->bounce_ev[k], c->copy));
    }
    c->bounce_cap = bytes;
    return CDC_OK;
}

Workspace carve(void *ws, const Plan &pl, const uint64_t *gear)
{
    char *b = static_cast<char *>(ws);
    Workspace W;
    W.runs = reinterpret_cast<uint64_t *>(b + pl.off_runs);
    W.w1_nodes = reinterpret_cast<uint64_t *>(b + pl.off_w1_nodes);
    W.xg = reinterpret_cast<uint64_t *>(b + pl.off_xg);
    W.sg = reinterpret_cast<uint64_t *>(b + pl.off_sg);
    W.flags = reinterpret_cast<uint32_t *>(b + pl.off_flags);
    W.tick = reinterpret_cast<uint32_t *>(b + pl.off_tick);
    W.gear = gear;
    W.runsL = reinterpret_cast<uint64_t *>(b + pl.off_runsL);
    W.validL = reinterpret_cast<uint32_t *>(b + pl.off_validL);
    return W;
}

// Launch one group of <= kMaxBufsPerLaunch device buffers.
int run_group(DeviceCtx *ctx, const DevParams &P, const void *const *data, const uint64_t *lens,
              int n, int final_, cdc_cut *const *cuts, const uint64_t *caps,
              cdc_result *const *res, void *ws, uint64_t ws_bytes, void *stream)
{
    Plan pl;
    int st = make_plan(lens, n, P, &pl);
    if (st != CDC_OK) return st;
    if (ws_bytes < pl.bytes) return CDC_E_INVALID;
    Batch B;
    std::memset(&B, 0, sizeof(B));
    B.nbufs = uint32_t(n);
    B.final_ = final_ ? 1u : 0u;
    B.total_segs = pl.total_segs;
    B.total_tasks = pl.total_tasks;
    B.seg = pl.seg;
    B.scan_lane = pl.scan_lane;
    B.persist = pl.persist;
    B.scan_wgs = pl.scan_wgs;
    static const uint32_t dbg = [] {
        const char *e = getenv("CDC_DEBUG_PHASE");
        return e ? uint32_t(atoi(e)) : 0u;
    }();
    B.debug = dbg;
    if (G().debug_mode == 2 || t_force_abort) {  // the device-abort path: a wait that never ends, a short spin limit
        B.debug |= kDbgForceAbort;
        B.spin_ticks = kForceAbortTicks;
    }
    // MaskL index.  CDC_MASKL_INDEX / cdc_set_maskl_index_mode: 0 off (walkers
    // raw-scan every MaskL region), 1 adaptive (default), 2 every group (in the
    // MaskS pass, k_scan_f, where the masks admit it), 3 every group by
    // k_scan_l.  Adaptive: built while the hint is set (fused where the masks
    // admit it, else k_scan_l, which re-raises it); otherwise every 16th group
    // runs the selection test alone (k_maskl_probe: no LDS, so it does not wait
    // for whole CUs beside the other stream's scan) and raises the hint; the
    // hint decays every 1024 groups.  Walkers use the index only for tasks
    // whose scan built it, so cut points never depend on this choice.
    const uint32_t mli = maskl_index_mode().load(std::memory_order_relaxed);
    {
        const uint64_t k = ctx->groups.fetch_add(1, std::memory_order_relaxed);
        volatile uint32_t *hint = ctx->hint_h;
        if (hint && k % 1024 == 1023) *hint = 0u;
        const bool hinted = !hint || *hint != 0u;
        B.maskl_index = mli >= 2 || (mli == 1 && hinted) ? 1u : 0u;
        B.maskl_fused = P.fm_ok && (mli == 2 || (mli == 1 && hinted)) ? 1u : 0u;
        B.maskl_probe = mli == 1 && !hinted && k % 16 == 0 ? 1u : 0u;
        B.maskl_hint = ctx->hint_d;
    }
    B.force_fallback = G().debug_mode == 1 ? 1u : 0u;
    uint32_t segs = 0, tasks = 0;
    for (int i = 0; i < n; ++i) {
        BufDesc &D = B.b[i];
        D.data = static_cast<const uint8_t *>(data[i]);
        D.len = lens[i];
        D.out = cuts[i];
        D.cap = caps[i];
        D.res = res[i];
        D.seg_base = segs;
        D.nseg = uint32_t((lens[i] + B.seg - 1) / B.seg);
        D.task_base = tasks;
        segs += D.nseg;
        tasks += uint32_t((lens[i] + 64ull * pl.scan_lane - 1) / (64ull * pl.scan_lane));
    }
    const Workspace W = carve(ws, pl, ctx->d_gear);
    return launch_batch(B, P, W, stream);
}

int group_ws_bytes(const uint64_t *lens, int n, const DevParams &P, uint64_t *bytes)
{
    Plan pl;
    const int st = make_plan(lens, n, P, &pl);
    if (st != CDC_OK) return st;
    *bytes = pl.bytes;
    return CDC_OK;
}

int check_ready(int device, DeviceCtx **out)
{
    Global &g = G();
    if (!g.init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    for (auto *c : g.devs)
        if (c->device == device) {
            *out = c;
            return CDC_OK;
        }
    return CDC_E_INVALID;
}

// Chunk one host buffer window-by-window on one device (used by cdc_chunk and
// the streaming path).  Appends cuts (offsets relative to `base_off`).
struct HostJob {
    const uint8_t *data;
    uint64_t len;
    std::vector<cdc_cut> cuts;
    int status = CDC_OK;
};

uint64_t max_cuts_for(uint64_t len, uint32_t min_size) { return len / min_size + 2; }

uint64_t env_mb(const char *name, uint64_t def_mb, uint64_t min_mb)
{
    if (const char *e = getenv(name)) {
        const long v = atol(e);
        if (v >= long(min_mb)) return uint64_t(v) << 20;
    }
    return def_mb << 20;
}

// Pageable -> pinned copy, split over a few host threads: one thread's
// memcpy (~10 GB/s) would otherwise cap the PCIe-inclusive rate.
constexpr int kCopyThreadsMax = 32;

int copy_threads()
{
    static const int n = [] {
        const char *e = getenv("CDC_COPY_THREADS");
        const int v = e ? atoi(e) : 4;
        return v < 1 ? 1 : (v > kCopyThreadsMax ? kCopyThreadsMax : v);
    }();
    return n;
}

void par_memcpy(uint8_t *dst, const uint8_t *src, uint64_t len)
{
    constexpr uint64_t kMinPiece = 4ull << 20;
    const int nt = int(std::min<uint64_t>(uint64_t(copy_threads()), (len + kMinPiece - 1) / kMinPiece));
    if (nt <= 1) {
        std::memcpy(dst, src, len);
        return;
    }
    const uint64_t per = ((len + nt - 1) / nt + 4095) & ~4095ull;
    std::thread th[kCopyThreadsMax];
    for (int t = 1; t < nt; ++t) {
        const uint64_t o = per * t;
        if (o >= len) break;
        th[t] = std::thread([=] { std::memcpy(dst + o, src + o, std::min(per, len - o)); });
    }
    std::memcpy(dst, src, std::min(per, len));
    for (int t = 1; t < nt; ++t)
        if (th[t].joinable()) th[t].join();
}

// Copy len host bytes to d_dst through the pinned bounce buffers on the copy
// stream.  Returns once the last piece is queued; the host fills bounce k+1
// while the copy engine drains bounce k.
int stage(DeviceCtx *c, uint8_t *d_dst, const uint8_t *src, uint64_t len)
{
    // Direct form (the default; CDC_HOST_DIRECT=0 selects the bounce buffers):
    // the runtime stages the pageable source itself, 56 GB/s for a pageable
    // 1-GiB copy on MI355X against ~34 GB/s through these bounce buffers (C4
    // 32 -> 47 GiB/s end to end).  The call returns when the copy is done; the
    // previous group's kernels run meanwhile on the compute stream.
    static const bool direct = [] {
        const char *e = getenv("CDC_HOST_DIRECT");
        return !(e && e[0] == '0');
    }();
    if (direct) {
        HIPCHK(hipMemcpyAsync(d_dst, src, len, hipMemcpyHostToDevice, c->copy));
        return CDC_OK;
    }
    uint64_t off = 0;
    while (off < len) {
        const int k = c->next_bounce;
        c->next_bounce = (k + 1) % kBounces;
        HIPCHK(hipEventSynchronize(c->bounce_ev[k]));
        const uint64_t n = std::min(c->bounce_cap, len - off);
        par_memcpy(c->bounce[k], src + off, n);
        HIPCHK(hipMemcpyAsync(d_dst + off, c->bounce[k], n, hipMemcpyHostToDevice, c->copy));
        HIPCHK(hipEventRecord(c->bounce_ev[k], c->copy));
        off += n;
    }
    return CDC_OK;
}

struct Pending {
    bool active = false;
    std::vector<HostJob *> jobs;
    std::vector<uint64_t> cut_off;
};

// Chunk one buffer too large to hold on the device as a stream of windows
// (final = 0 except the last; each window resumes at the previous one's
// `consumed`).  Sequential: the next window's start depends on this one.
int run_windowed(DeviceCtx *ctx, const DevParams &P, const cdc_opts *o, HostJob *job, uint64_t window)
{
    Slot &sl = ctx->slot[0];
    const uint64_t ncap = max_cuts_for(window, o->min_size);
    uint64_t off = 0;
    while (off < job->len) {
        const uint64_t w = std::min(window, job->len - off);
        const int fin = off + w == job->len;
        uint64_t need = 0;
        int st = group_ws_bytes(&w, 1, P, &need);
        if (st != CDC_OK) return st;
        st = grow_slot(sl, window, need, ncap);
        if (st != CDC_OK) return st;
        st = stage(ctx, sl.d_in, job->data + off, w);
        if (st != CDC_OK) return st;
        HIPCHK(hipEventRecord(sl.staged, ctx->copy));
        HIPCHK(hipStreamWaitEvent(ctx->stream, sl.staged, 0));
        const void *dp = sl.d_in;
        cdc_cut *cp = sl.d_cuts;
        const uint64_t cap = sl.cuts_cap;
        cdc_result *rp = sl.d_res;
        st = run_group(ctx, P, &dp, &w, 1, fin, &cp, &cap, &rp, sl.d_ws, sl.ws_cap, ctx->stream);
        if (st != CDC_OK) return st;
        HIPCHK(hipMemcpyAsync(sl.h_res, sl.d_res, sizeof(cdc_result), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        const cdc_result r = sl.h_res[0];
        if (r.status != CDC_OK) return int(r.status);
        if (r.ncuts) {
            HIPCHK(hipMemcpyAsync(sl.h_cuts, sl.d_cuts, r.ncuts * sizeof(cdc_cut), hipMemcpyDeviceToHost,
                                  ctx->stream));
            HIPCHK(hipStreamSynchronize(ctx->stream));
        }
        for (uint64_t k = 0; k < r.ncuts; ++k) {
            cdc_cut c = sl.h_cuts[k];
            c.offset += off;
            job->cuts.push_back(c);
        }
        if (!fin && r.consumed == 0) return CDC_E_DEVICE;  // cannot happen: window >= 4 * Max
        off += fin ? w : r.consumed;
    }
    return CDC_OK;
}

// Process host jobs on one device as a two-slot pipeline.  Buffers are packed
// into launch groups (<= kMaxBufsPerLaunch buffers, <= CDC_HOST_GROUP_MB bytes;
// one larger buffer forms a group of its own).  While the compute stream
// chunks group g in slot g % 2, the host stages group g + 1 into the other
// slot through the pinned bounce buffers on the copy stream.  Only a buffer
// larger than CDC_HOST_MAXBUF_MB (default 16 GiB of the 288 GB of HBM) is
// chunked as a stream of windows.
int run_host_jobs(DeviceCtx *ctx, const cdc_opts *o, std::vector<HostJob *> &jobs)
{
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return CDC_E_DEVICE;
    const DevParams P = make_params(o);
    const uint64_t budget = std::max<uint64_t>(env_mb("CDC_HOST_GROUP_MB", 1024, 16), 4ull * o->max_size + 4096);
    const uint64_t maxbuf = std::max<uint64_t>(env_mb("CDC_HOST_MAXBUF_MB", 16384, 16), budget);
    if (!ctx->copy) HIPCHK(hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking));
    int st = grow_bounce(ctx, std::min<uint64_t>(64ull << 20, budget));
    if (st != CDC_OK) return st;

    Pending pend[2];
    auto harvest = [&](int s) -> int {
        Pending &pd = pend[s];
        if (!pd.active) return CDC_OK;
        pd.active = false;
        Slot &sl = ctx->slot[s];
        HIPCHK(hipEventSynchronize(sl.done));
        for (size_t i = 0; i < pd.jobs.size(); ++i) {
            const cdc_result r = sl.h_res[i];
            if (r.status != CDC_OK) return int(r.status);
            pd.jobs[i]->cuts.assign(sl.h_cuts + pd.cut_off[i], sl.h_cuts + pd.cut_off[i] + r.ncuts);
        }
        return CDC_OK;
    };

    int cur = 0;
    size_t j = 0;
    while (j < jobs.size()) {
        if (jobs[j]->len > maxbuf) {
            if ((st = harvest(0)) != CDC_OK || (st = harvest(1)) != CDC_OK) return st;
            st = run_windowed(ctx, P, o, jobs[j], budget);
            if (st != CDC_OK) return st;
            ++j;
            continue;
        }
        std::vector<HostJob *> group;
        std::vector<uint64_t> offs, lens, caps, cut_off;
        uint64_t used = 0, ncuts = 0;
        while (j < jobs.size() && group.size() < size_t(kMaxBufsPerLaunch) && jobs[j]->len <= maxbuf &&
               (group.empty() || used + jobs[j]->len <= budget)) {
            HostJob *jb = jobs[j++];
            group.push_back(jb);
            offs.push_back(used);
            lens.push_back(jb->len);
            caps.push_back(max_cuts_for(jb->len, o->min_size));
            cut_off.push_back(ncuts);
            ncuts += caps.back();
            used = (used + jb->len + 255) & ~255ull;
        }
        const int s = cur;
        cur ^= 1;
        if ((st = harvest(s)) != CDC_OK) return st;  // the slot's previous group
        Slot &sl = ctx->slot[s];
        const int n = int(group.size());
        uint64_t need = 0;
        if ((st = group_ws_bytes(lens.data(), n, P, &need)) != CDC_OK) return st;
        if ((st = grow_slot(sl, used, need, ncuts)) != CDC_OK) return st;
        for (int i = 0; i < n; ++i)
            if ((st = stage(ctx, sl.d_in + offs[i], group[i]->data, lens[i])) != CDC_OK) return st;
        HIPCHK(hipEventRecord(sl.staged, ctx->copy));
        HIPCHK(hipStreamWaitEvent(ctx->stream, sl.staged, 0));
        std::vector<const void *> dp(n);
        std::vector<cdc_cut *> cp(n);
        std::vector<cdc_result *> rp(n);
        for (int i = 0; i < n; ++i) {
            dp[i] = sl.d_in + offs[i];
            cp[i] = sl.d_cuts + cut_off[i];
            rp[i] = sl.d_res + i;
        }
        st = run_group(ctx, P, dp.data(), lens.data(), n, 1, cp.data(), caps.data(), rp.data(), sl.d_ws,
                       sl.ws_cap, ctx->stream);
        if (st != CDC_OK) return st;
        HIPCHK(hipMemcpyAsync(sl.h_res, sl.d_res, n * sizeof(cdc_result), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(sl.h_cuts, sl.d_cuts, ncuts * sizeof(cdc_cut), hipMemcpyDeviceToHost,
                              ctx->stream));
        HIPCHK(hipEventRecord(sl.done, ctx->stream));
        pend[s].active = true;
        pend[s].jobs = std::move(group);
        pend[s].cut_off = std::move(cut_off);
    }
    if ((st = harvest(0)) != CDC_OK) return st;
    return harvest(1);
}

}  // namespace

namespace cdc {

int device_count_initialised()
{
    Global &g = G();
    return g.init.load(std::memory_order_acquire) ? int(g.devs.size()) : 0;
}

// The collector's per-device worker (see cdc_internal.h): run_host_jobs'
// two-slot pipeline, fed batch by batch for as long as the source has work.
// The device lock is held while groups are in flight and released whenever
// the pipeline drains, so other callers of the device interleave at idle
// points.  A failing batch is handed back with the status on every buffer.
int pipeline_device(int di, const cdc_opts *o, BatchSource &src)
{
    Global &g = G();
    if (!g.init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    if (di < 0 || size_t(di) >= g.devs.size()) return CDC_E_INVALID;
    DeviceCtx *ctx = g.devs[size_t(di)];
    const DevParams P = make_params(o);
    const uint64_t budget = std::max<uint64_t>(env_mb("CDC_HOST_GROUP_MB", 1024, 16), 4ull * o->max_size + 4096);
    const uint64_t maxbuf = std::max<uint64_t>(env_mb("CDC_HOST_MAXBUF_MB", 16384, 16), budget);
    std::unique_lock<std::mutex> lock(ctx->mu, std::defer_lock);
    std::vector<HostBuf *> fl[2];
    std::vector<uint64_t> cut_off[2];
    bool active[2] = {false, false};
    auto fail = [&](std::vector<HostBuf *> &b, int st) {
        for (HostBuf *h : b) h->status = st;
        src.finished(b);
        b.clear();
    };
    auto harvest = [&](int s) {
        if (!active[s]) return;
        active[s] = false;
        Slot &sl = ctx->slot[s];
        int st = hipEventSynchronize(sl.done) == hipSuccess ? CDC_OK : CDC_E_DEVICE;
        for (size_t i = 0; i < fl[s].size(); ++i) {
            HostBuf *h = fl[s][i];
            const cdc_result r = sl.h_res[i];
            h->status = st != CDC_OK ? st : int(r.status);
            if (h->status == CDC_OK) h->cuts.assign(sl.h_cuts + cut_off[s][i], sl.h_cuts + cut_off[s][i] + r.ncuts);
        }
        src.finished(fl[s]);
        fl[s].clear();
    };
    // stage + launch one batch into slot s (one launch group; a buffer over
    // maxbuf goes through the windowed path synchronously)
    auto submit = [&](int s, std::vector<HostBuf *> &b) -> int {
        if (b.size() == 1 && b[0]->len > maxbuf) {
            HostJob job{b[0]->data, b[0]->len, {}, CDC_OK};
            const int st = run_windowed(ctx, P, o, &job, budget);
            b[0]->status = st;
            if (st == CDC_OK) b[0]->cuts = std::move(job.cuts);
            src.finished(b);
            b.clear();
            return CDC_OK;
        }
        const int n = int(b.size());
        std::vector<uint64_t> offs(n), lens(n), caps(n);
        cut_off[s].assign(n, 0);
        uint64_t used = 0, ncuts = 0;
        for (int i = 0; i < n; ++i) {
            offs[i] = used;
            lens[i] = b[i]->len;
            caps[i] = max_cuts_for(b[i]->len, o->min_size);
            cut_off[s][i] = ncuts;
            ncuts += caps[i];
            used = (used + b[i]->len + 255) & ~255ull;
        }
        Slot &sl = ctx->slot[s];
        uint64_t need = 0;
        int st = group_ws_bytes(lens.data(), n, P, &need);
        if (st != CDC_OK) return st;
        if ((st = grow_slot(sl, std::max<uint64_t>(used, 256), need, ncuts)) != CDC_OK) return st;
        for (int i = 0; i < n; ++i)
            if (lens[i] && (st = stage(ctx, sl.d_in + offs[i], b[i]->data, lens[i])) != CDC_OK) return st;
        HIPCHK(hipEventRecord(sl.staged, ctx->copy));
        HIPCHK(hipStreamWaitEvent(ctx->stream, sl.staged, 0));
        std::vector<const void *> dp(n);
        std::vector<cdc_cut *> cp(n);
        std::vector<cdc_result *> rp(n);
        for (int i = 0; i < n; ++i) {
            dp[i] = sl.d_in + offs[i];
            cp[i] = sl.d_cuts + cut_off[s][i];
            rp[i] = sl.d_res + i;
        }
        st = run_group(ctx, P, dp.data(), lens.data(), n, 1, cp.data(), caps.data(), rp.data(), sl.d_ws, sl.ws_cap,
                       ctx->stream);
        if (st != CDC_OK) return st;
        HIPCHK(hipMemcpyAsync(sl.h_res, sl.d_res, n * sizeof(cdc_result), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(sl.h_cuts, sl.d_cuts, ncuts * sizeof(cdc_cut), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipEventRecord(sl.done, ctx->stream));
        fl[s] = std::move(b);
        active[s] = true;
        return CDC_OK;
    };
    // A failure inside the loop (an allocation of the host-side lists) hands
    // every batch it holds back with the status, after the device is done
    // with their buffers, and the worker goes on with the next batch: no
    // caller waits for a batch that nobody finishes.
    auto fail_inflight = [&](std::vector<HostBuf *> &cur_batch, int st) {
        if (lock.owns_lock()) {
            (void)hipStreamSynchronize(ctx->stream);
            if (ctx->copy) (void)hipStreamSynchronize(ctx->copy);
        }
        for (int s = 0; s < 2; ++s)
            if (active[s]) {
                active[s] = false;
                fail(fl[s], st);
            }
        if (!cur_batch.empty()) fail(cur_batch, st);
    };
    // The device lock is also released every kBatchesPerLock batches (the
    // pipeline drained first), so cdc_chunk callers of the same device are not
    // starved by a steady stream of collector batches.
    constexpr int kBatchesPerLock = 16;
    int held = 0;
    int cur = 0;
    for (;;) {
        std::vector<HostBuf *> batch;
        try {
        bool busy = active[0] || active[1];
        if (busy && held >= kBatchesPerLock) {
            harvest(cur ^ 1);  // the older group first
            harvest(cur);
            busy = false;
        }
        if (!busy && lock.owns_lock()) {  // drained: other callers may use the device
            lock.unlock();
            held = 0;
        }
        if (!src.next(batch, !busy)) {
            if (!busy) return CDC_OK;  // the source is stopping
            harvest(active[cur] ? cur : cur ^ 1);  // the older group first (cur is the slot used next)
            continue;
        }
        if (batch.empty()) continue;
        ++held;
        if (!lock.owns_lock()) {
            lock.lock();
            int st = hipSetDevice(ctx->device) == hipSuccess ? CDC_OK : CDC_E_DEVICE;
            if (st == CDC_OK && !ctx->copy && hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking) != hipSuccess)
                st = CDC_E_DEVICE;
            if (st == CDC_OK) st = grow_bounce(ctx, std::min<uint64_t>(64ull << 20, budget));
            if (st != CDC_OK) {
                fail(batch, st);
                continue;
            }
        }
        const int s = cur;
        cur ^= 1;
        harvest(s);  // the slot's previous group
        const int st = submit(s, batch);
        if (st != CDC_OK) {
            fail(batch, st);
            harvest(s ^ 1);
        }
        } catch (const std::bad_alloc &) {
            fail_inflight(batch, CDC_E_NOMEM);
        } catch (...) {
            fail_inflight(batch, CDC_E_DEVICE);
        }
    }
}

}  // namespace cdc

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int cdc_abi_version(void) { return CDC_ABI_VERSION; }

const char *cdc_strerror(int s)
{
    switch (s) {
    case CDC_OK: return "ok";
    case CDC_EOF: return "EOF";
    case CDC_NEED_DATA: return "need more data";
    case CDC_E_INVALID: return "invalid argument";
    case CDC_E_UNSUPPORTED: return "unsupported chunking algorithm";
    case CDC_E_NOSPACE: return "output capacity too small";
    case CDC_E_DEVICE: return "HIP device error";
    case CDC_E_NOMEM: return "out of memory";
    case CDC_E_NORMAL_SIZE: return "NormalSize is required and must be 64B <= NormalSize <= 1GB";
    case CDC_E_MIN_SIZE: return "MinSize is required and must be 64B <= MinSize <= 1GB && MinSize < NormalSize";
    case CDC_E_MAX_SIZE: return "MaxSize is required and must be 64B <= MaxSize <= 1GB && MaxSize > NormalSize";
    case CDC_E_IO: return "reader error";
    case CDC_E_NOT_INIT: return "cdc_init() has not been called";
    case CDC_E_NO_DEVICE: return "no HIP device available";
    default: return "unknown status";
    }
}

void cdc_default_gear(uint64_t out[256])
{
    uint64_t s = 0x504C414B4152ull;  // "PLAKAR"
    for (int i = 0; i < 256; ++i) out[i] = splitmix64(s);
}

uint64_t cdc_default_mask_s(void) { return kDefaultMaskS; }
uint64_t cdc_default_mask_l(void) { return kDefaultMaskL; }

void cdc_default_opts(cdc_opts *out)
{
    if (!out) return;
    out->min_size = 64 * 1024;
    out->normal_size = 1 * 1024 * 1024;
    out->max_size = 4 * 1024 * 1024;
    out->reserved = 0;
}

int cdc_validate(const char *algorithm, const cdc_opts *opts)
{
    if (!algorithm || !opts) return CDC_E_INVALID;
    const std::string a = lower(algorithm);
    if (a != "fastcdc") return CDC_E_UNSUPPORTED;
    return validate_sizes(opts);
}

int cdc_set_debug_mode(int mode)
{
    G().debug_mode = mode;
    return CDC_OK;
}

int cdc_set_maskl_index_mode(int mode)
{
    if (mode < 0 || mode > 3) return CDC_E_INVALID;
    maskl_index_mode().store(uint32_t(mode), std::memory_order_relaxed);
    // a new mode starts the adaptive state afresh (no recent MaskL request)
    Global &g = G();
    std::lock_guard<std::mutex> lock(g.mu);
    for (DeviceCtx *c : g.devs)
        if (c && c->hint_h) *static_cast<volatile uint32_t *>(c->hint_h) = 0u;
    return CDC_OK;
}

int cdc_debug_set_digest_lanes(uint64_t lanes)
{
    cdc::g_digest_lanes = lanes;
    return CDC_OK;
}

int cdc_debug_maskl_state(int device, uint32_t *hint, uint64_t *groups)
{
    if (!hint || !groups) return CDC_E_INVALID;
    DeviceCtx *ctx = nullptr;
    const int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    if (hipSetDevice(device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return CDC_E_DEVICE;
    *hint = ctx->hint_h ? *static_cast<volatile uint32_t *>(ctx->hint_h) : 1u;
    *groups = ctx->groups.load(std::memory_order_relaxed);
    return CDC_OK;
}

int cdc_debug_stream_read(int device, const void *d_buf, uint64_t len, int reps, double best_us[3], double median_us[3],
                          void *stream)
{
    if (!d_buf || !best_us || !median_us) return CDC_E_INVALID;
    DeviceCtx *ctx = nullptr;
    const int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    return launch_stream_read(d_buf, len, reps, best_us, median_us, stream);
}

int cdc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static void destroy_ctx(DeviceCtx *c)
{
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipDeviceSynchronize();  // caller streams may still run kernels that write the hint
    if (c->hint_h) (void)hipHostFree(c->hint_h);
    if (c->d_gear) (void)hipFree(c->d_gear);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    free_ctx_buffers(c);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    delete c;
}

static int create_ctx(int d, DeviceCtx **out)
{
    auto *c = new DeviceCtx();
    c->device = d;
    *out = nullptr;
    if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&c->d_gear), 256 * sizeof(uint64_t)) != hipSuccess) {
        destroy_ctx(c);
        return CDC_E_DEVICE;
    }
    if (hipHostMalloc(reinterpret_cast<void **>(&c->hint_h), 64, hipHostMallocMapped | hipHostMallocCoherent) ==
        hipSuccess) {
        *c->hint_h = 0u;
        if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c->hint_d), c->hint_h, 0) != hipSuccess) {
            (void)hipHostFree(c->hint_h);
            c->hint_h = c->hint_d = nullptr;
        }
    }
    *out = c;
    return CDC_OK;
}

// Re-initialisation keeps the device set (a different one needs cdc_shutdown
// first) and waits for every device to go idle before it rewrites the Gear
// table; cdc_stream objects pick up the new parameters at their next run.  A
// failure while creating contexts leaves the library uninitialised with
// nothing allocated.
int cdc_init(uint32_t dev_mask, const uint64_t gear[256], uint64_t mask_s, uint64_t mask_l,
             int cut_convention)
{
    Global &g = G();
    std::lock_guard<std::mutex> lock(g.mu);
    if (cut_convention != 0 && cut_convention != 1) return CDC_E_INVALID;
    uint64_t tab[256];
    if (gear)
        std::memcpy(tab, gear, sizeof(tab));
    else
        cdc_default_gear(tab);
    const uint64_t ms = mask_s ? mask_s : kDefaultMaskS, ml = mask_l ? mask_l : kDefaultMaskL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return g.devs.empty() ? CDC_E_NO_DEVICE : CDC_E_DEVICE;
    std::vector<int> want;
    for (int d = 0; d < n && d < 32; ++d)
        if (!dev_mask || (dev_mask & (1u << d))) want.push_back(d);
    if (want.empty()) return CDC_E_NO_DEVICE;
    if (!g.devs.empty()) {
        std::vector<int> have;
        for (auto *c : g.devs) have.push_back(c->device);
        if (have != want) return CDC_E_INVALID;  // cdc_shutdown() first
        const bool same = std::memcmp(tab, g.gear, sizeof(tab)) == 0 && ms == g.mask_s && ml == g.mask_l &&
                          uint32_t(cut_convention) == g.cut_adj;
        if (same && g.init.load(std::memory_order_acquire)) return CDC_OK;
        for (auto *c : g.devs)
            if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return CDC_E_DEVICE;
    } else {
        std::vector<DeviceCtx *> made;
        for (int d : want) {
            DeviceCtx *c = nullptr;
            const int st = create_ctx(d, &c);
            if (st != CDC_OK) {
                for (auto *m : made) destroy_ctx(m);
                return st;
            }
            made.push_back(c);
        }
        g.devs = made;
    }
    g.init.store(false, std::memory_order_release);
    std::memcpy(g.gear, tab, sizeof(tab));
    g.placeholder_gear = gear == nullptr;
    g.mask_s = ms;
    g.mask_l = ml;
    g.cut_adj = uint32_t(cut_convention);
    for (auto *c : g.devs) {
        if (hipSetDevice(c->device) != hipSuccess ||
            hipMemcpy(c->d_gear, g.gear, sizeof(g.gear), hipMemcpyHostToDevice) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) {
            // a partial update would leave devices on different tables: tear
            // everything down, so a failed cdc_init leaves the library
            // uninitialised with nothing allocated (the header's contract)
            for (auto *d : g.devs) destroy_ctx(d);
            g.devs.clear();
            return CDC_E_DEVICE;
        }
    }
    g.init.store(true, std::memory_order_release);
    return CDC_OK;
}

int cdc_gear_is_placeholder(void) { return G().placeholder_gear ? 1 : 0; }

void cdc_shutdown(void)
{
    Global &g = G();
    std::lock_guard<std::mutex> lock(g.mu);
    g.init.store(false, std::memory_order_release);
    for (auto *c : g.devs) destroy_ctx(c);
    g.devs.clear();
}

int cdc_device_workspace_size(uint64_t len, const cdc_opts *opts, uint64_t *bytes)
{
    return cdc_device_batch_workspace_size(&len, 1, opts, bytes);
}

int cdc_device_batch_workspace_size(const uint64_t *lens, int nbufs, const cdc_opts *opts,
                                    uint64_t *bytes)
{
    if (!lens || nbufs < 0 || !opts || !bytes) return CDC_E_INVALID;
    const int v = validate_sizes(opts);
    if (v != CDC_OK) return v;
    const DevParams P = make_params(opts);
    uint64_t best = 0;
    for (int i = 0; i < nbufs; i += kMaxBufsPerLaunch) {
        const int n = std::min(kMaxBufsPerLaunch, nbufs - i);
        uint64_t b = 0;
        const int st = group_ws_bytes(lens + i, n, P, &b);
        if (st != CDC_OK) return st;
        best = std::max(best, b);
    }
    *bytes = best;
    return CDC_OK;
}

int cdc_chunk_device_async(int device, const void *d_data, uint64_t len, int final_,
                           const cdc_opts *opts, cdc_cut *d_cuts, uint64_t cut_cap,
                           cdc_result *d_result, void *d_workspace, uint64_t workspace_bytes,
                           void *stream)
{
    return cdc_chunk_device_batch_async(device, &d_data, &len, 1, final_, opts, &d_cuts, &cut_cap,
                                        &d_result, d_workspace, workspace_bytes, stream);
}

int cdc_chunk_device_batch_async(int device, const void *const *d_data, const uint64_t *lens,
                                 int nbufs, int final_, const cdc_opts *opts,
                                 cdc_cut *const *d_cuts, const uint64_t *cut_caps,
                                 cdc_result *const *d_results, void *d_workspace,
                                 uint64_t workspace_bytes, void *stream)
{
    if (!d_data || !lens || nbufs < 0 || !opts || !d_cuts || !cut_caps || !d_results ||
        !d_workspace)
        return CDC_E_INVALID;
    const int v = validate_sizes(opts);
    if (v != CDC_OK) return v;
    DeviceCtx *ctx = nullptr;
    int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    for (int i = 0; i < nbufs; ++i)
        if (!d_results[i] || (lens[i] && (!d_data[i] || !d_cuts[i]))) return CDC_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    const DevParams P = make_params(opts);
    for (int i = 0; i < nbufs; i += kMaxBufsPerLaunch) {
        const int n = std::min(kMaxBufsPerLaunch, nbufs - i);
        st = run_group(ctx, P, d_data + i, lens + i, n, final_, d_cuts + i, cut_caps + i,
                       d_results + i, d_workspace, workspace_bytes, stream);
        if (st != CDC_OK) return st;
    }
    return CDC_OK;
}

int cdc_chunk_digests_device_batch_async(int device, const void *const *d_data, const uint64_t *lens, int nbufs,
                                         const cdc_cut *const *d_cuts, const uint64_t *cut_caps,
                                         const cdc_result *const *d_results, uint8_t *const *d_digests,
                                         uint32_t *const *d_hist, void *stream)
{
    if (nbufs < 0 || (nbufs > 0 && (!d_data || !lens || !d_cuts || !cut_caps || !d_digests))) return CDC_E_INVALID;
    bool want_hist = false;  // histograms for all buffers or none (a buffer without chunks may pass NULL)
    for (int i = 0; i < nbufs && d_hist; ++i) want_hist |= cut_caps[i] && d_hist[i];
    for (int i = 0; i < nbufs; ++i) {
        if ((lens[i] && !d_data[i]) || (cut_caps[i] && (!d_cuts[i] || !d_digests[i]))) return CDC_E_INVALID;
        if (want_hist && cut_caps[i] && !d_hist[i]) return CDC_E_INVALID;
    }
    if (!want_hist) d_hist = nullptr;
    DeviceCtx *ctx = nullptr;
    int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    if (nbufs > kMaxBufsPerLaunch) {  // one launch group, descriptors in device memory
        std::vector<DigestBuf> bufs(static_cast<size_t>(nbufs));
        for (int i = 0; i < nbufs; ++i)
            bufs[size_t(i)] = DigestBuf{static_cast<const uint8_t *>(d_data[i]), lens[i], d_cuts[i], cut_caps[i],
                                        d_results ? d_results[i] : nullptr, d_digests[i], d_hist ? d_hist[i] : nullptr};
        return launch_digests_many(bufs.data(), uint32_t(nbufs), stream);
    }
    for (int i0 = 0; i0 < nbufs; i0 += kMaxBufsPerLaunch) {
        DigestBatch DB;
        std::memset(&DB, 0, sizeof(DB));
        DB.nbufs = uint32_t(std::min(kMaxBufsPerLaunch, nbufs - i0));
        for (uint32_t j = 0; j < DB.nbufs; ++j) {
            const int i = i0 + int(j);
            DB.b[j] = DigestBuf{static_cast<const uint8_t *>(d_data[i]), lens[i], d_cuts[i], cut_caps[i],
                                d_results ? d_results[i] : nullptr, d_digests[i], d_hist ? d_hist[i] : nullptr};
        }
        st = launch_digests(DB, stream);
        if (st != CDC_OK) return st;
    }
    return CDC_OK;
}

int cdc_chunk_digests_device_async(int device, const void *d_data, uint64_t len, const cdc_cut *d_cuts,
                                   uint64_t cut_cap, const cdc_result *d_result, uint8_t *d_digests,
                                   uint32_t *d_hist, void *stream)
{
    return cdc_chunk_digests_device_batch_async(device, &d_data, &len, 1, &d_cuts, &cut_cap, &d_result, &d_digests,
                                                d_hist ? &d_hist : nullptr, stream);
}

// ---- hybrid digests: the longest chunks' SHA-256 on host cores -------------
// One device chain costs ~2.05 us per 64-B block (cdc_digest.hip), a host
// core with the SHA extensions ~35 ns, so the device's launch, which lasts as
// long as its longest chunk, ends sooner when the longest chunks go to the
// host.  Per device, one call at a time; scratch grown on demand and kept.
}  // extern "C"
namespace {
struct HybridScratch {
    std::mutex mu;
    hipStream_t side = nullptr;
    hipEvent_t ev_dig = nullptr;
    hipEvent_t ev_part[4] = {};
    // device / pinned host buffers and their capacities in bytes
    void *d_cuts = nullptr, *d_stage = nullptr, *d_gj = nullptr, *d_sj = nullptr, *d_dig = nullptr;
    void *h_stage = nullptr, *h_gj = nullptr, *h_sj = nullptr, *h_dig = nullptr;
    uint64_t c_cuts = 0, c_stage = 0, c_gj = 0, c_sj = 0, c_dig = 0;
    uint64_t hc_stage = 0, hc_gj = 0, hc_sj = 0, hc_dig = 0;
};

HybridScratch &hybrid_scratch(int device)
{
    static HybridScratch h[64];
    return h[device & 63];
}

// Host threads for the hybrid digests' SHA-256, kept between calls (one pool
// per device, used under that device's HybridScratch lock): starting 23
// threads per call cost about a millisecond.  The threads are detached and
// live for the process (a forked child, which has none of them, starts its
// own).
struct HostPool {
    std::mutex mu;
    std::condition_variable go, done;
    const std::function<void()> *job = nullptr;
    uint64_t gen = 0;
    int nthreads = 0, want = 0, busy = 0;
    pid_t pid = 0;  // the process the threads belong to (a forked child has none of them)

    // f on n - 1 pool threads and the caller; returns when every one is done
    void run(int n, const std::function<void()> &f)
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (pid != getpid()) {
                pid = getpid();
                nthreads = 0;
            }
            try {
                while (nthreads < n - 1) {
                    std::thread([this, id = nthreads] { loop(id); }).detach();
                    ++nthreads;
                }
            } catch (...) {  // fewer threads: the work is shared by the ones there are
            }
            job = &f;
            want = std::min(n - 1, nthreads);
            busy = want;
            ++gen;
        }
        go.notify_all();
        f();
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return busy == 0; });
        job = nullptr;
    }

    void loop(int id)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void()> *j;
            {
                std::unique_lock<std::mutex> lk(mu);
                go.wait(lk, [&] { return gen != seen; });
                seen = gen;
                if (id >= want) continue;  // not counted for this job
                j = job;
            }
            (*j)();
            std::lock_guard<std::mutex> lk(mu);
            if (--busy == 0) done.notify_all();
        }
    }
};

HostPool &host_pool(int device)
{
    static HostPool *p = new HostPool[64];  // never destroyed: its threads outlive static destruction
    return p[device & 63];
}

bool hy_dev(void *&p, uint64_t &cap, uint64_t need)
{
    if (need <= cap && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const uint64_t n = need + need / 4 + 256;
    if (hipMalloc(&p, n) != hipSuccess) return false;
    cap = n;
    return true;
}

bool hy_host(void *&p, uint64_t &cap, uint64_t need)
{
    if (need <= cap && p) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const uint64_t n = need + need / 4 + 256;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return false;
    cap = n;
    return true;
}

// One host core's SHA-256 rate, measured once per process (8 MiB through the
// same sha256() the workers call): the split below depends on it, and it
// differs between hosts (SHA extensions or not, clock).
double host_sha_rate()
{
    static const double rate = [] {
        std::vector<uint8_t> buf(8u << 20, 0x5a);
        uint8_t d[32];
        sha256(buf.data(), 1u << 20, d);  // warm the code and the pages
        const auto t0 = std::chrono::steady_clock::now();
        sha256(buf.data(), buf.size(), d);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return s > 0 ? std::max(2e8, std::min(8e9, double(buf.size()) / s)) : 1.6e9;
    }();
    return rate;
}

// The host's share: the longest chunks, as many as balance the two sides.
// Device: the longest chunk left to it (its chain, ~2.05 us per 64-B block).
// Host: its chunks come back over PCIe in `parts` pieces while the threads
// hash the pieces already landed, so its time is the first piece's copy plus
// the slower of the copy of the rest and the hashing (bytes over `threads`
// cores, the longest chunk's own chain at least).
size_t hybrid_split(const std::vector<uint64_t> &sorted_desc, int threads, int parts)
{
    constexpr double kDevPerByte = 2.05e-6 / 64.0, kPcie = 40e9;
    const double rate = host_sha_rate();
    double best = 1e30, bytes = 0;
    size_t k_best = 0;
    const size_t n = std::min<size_t>(sorted_desc.size(), 1u << 16);
    for (size_t k = 0; k <= n; ++k) {
        const double dev = k < sorted_desc.size() ? double(sorted_desc[k]) * kDevPerByte : 0.0;
        const double host =
            k ? bytes / double(std::min<size_t>(size_t(parts), k)) / kPcie +
                    std::max({double(sorted_desc[0]) / rate, bytes / (threads * rate), bytes / kPcie})
              : 0.0;
        const double t = std::max(dev, host);
        if (t < best) {
            best = t;
            k_best = k;
        }
        if (k < n) bytes += double(sorted_desc[k]);
    }
    return k_best;
}
}  // namespace
extern "C" {

int cdc_chunk_digests_hybrid(int device, const void *const *d_data, const uint64_t *lens, int nbufs,
                             const cdc_cut *const *d_cuts, const uint64_t *cut_caps, const cdc_result *const *d_results,
                             uint8_t *const *d_digests, uint32_t *const *d_hist, int host_threads,
                             uint64_t host_min_len, void *stream, uint64_t *host_chunks, uint64_t *host_bytes)
{
    if (host_chunks) *host_chunks = 0;
    if (host_bytes) *host_bytes = 0;
    if (nbufs < 0 || (nbufs > 0 && (!d_data || !lens || !d_cuts || !cut_caps || !d_digests)) || host_threads < 0 ||
        host_threads > 256)
        return CDC_E_INVALID;
    bool want_hist = false;
    for (int i = 0; i < nbufs && d_hist; ++i) want_hist |= cut_caps[i] && d_hist[i];
    for (int i = 0; i < nbufs; ++i) {
        if ((lens[i] && !d_data[i]) || (cut_caps[i] && (!d_cuts[i] || !d_digests[i]))) return CDC_E_INVALID;
        if (want_hist && cut_caps[i] && !d_hist[i]) return CDC_E_INVALID;
    }
    DeviceCtx *ctx = nullptr;
    int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    if (host_threads == 0 || nbufs == 0 || nbufs > kMaxBufsPerLaunch)  // all on the device
        return cdc_chunk_digests_device_batch_async(device, d_data, lens, nbufs, d_cuts, cut_caps, d_results,
                                                    d_digests, d_hist, stream);
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    hipStream_t sm = reinterpret_cast<hipStream_t>(stream);
    HybridScratch &H = hybrid_scratch(device);
    std::lock_guard<std::mutex> lk(H.mu);
    if (!H.side) {
        if (hipStreamCreateWithFlags(&H.side, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&H.ev_dig, hipEventDisableTiming) != hipSuccess)
            return CDC_E_DEVICE;
        for (auto &e : H.ev_part)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return CDC_E_DEVICE;
    }
    // the cut lists, final once the caller's stream is drained
    if (hipStreamSynchronize(sm) != hipSuccess) return CDC_E_DEVICE;
    std::vector<uint64_t> cnt(static_cast<size_t>(nbufs)), base(static_cast<size_t>(nbufs) + 1, 0);
    for (int i = 0; i < nbufs; ++i) {
        uint64_t c = cut_caps[i];
        if (d_results && d_results[i] && c) {
            cdc_result r;
            if (hipMemcpy(&r, d_results[i], sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return CDC_E_DEVICE;
            c = std::min<uint64_t>(c, r.ncuts);
        }
        cnt[size_t(i)] = c;
        base[size_t(i) + 1] = base[size_t(i)] + c;
    }
    const uint64_t total = base[size_t(nbufs)];
    std::vector<cdc_cut> cuts(total);
    for (int i = 0; i < nbufs; ++i)
        if (cnt[size_t(i)] && hipMemcpy(cuts.data() + base[size_t(i)], d_cuts[i], cnt[size_t(i)] * sizeof(cdc_cut),
                                        hipMemcpyDeviceToHost) != hipSuccess)
            return CDC_E_DEVICE;
    // chunk lengths as the kernels see them (clipped to the buffer), buffer of each row
    std::vector<uint64_t> L(total);
    std::vector<int> bof(total);
    for (int i = 0; i < nbufs; ++i)
        for (uint64_t q = base[size_t(i)]; q < base[size_t(i) + 1]; ++q) {
            const cdc_cut &c = cuts[q];
            L[q] = c.offset >= lens[i] ? 0ull : std::min<uint64_t>(c.length, lens[i] - c.offset);
            bof[q] = i;
        }
    // longest first, ties in row order: one sort of (~length, row) keys
    // (lengths are clipped chunk lengths, < 2^32)
    std::vector<uint64_t> order(total);
    if (total < (1ull << 32)) {
        for (uint64_t q = 0; q < total; ++q) order[q] = (uint64_t(0xFFFFFFFFu - uint32_t(std::min<uint64_t>(L[q], 0xFFFFFFFFu))) << 32) | q;
        std::sort(order.begin(), order.end());
        for (uint64_t q = 0; q < total; ++q) order[q] &= 0xFFFFFFFFull;
    } else {
        for (uint64_t q = 0; q < total; ++q) order[q] = q;
        std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return L[a] > L[b]; });
    }
    size_t k = 0;
    if (host_min_len) {
        while (k < total && L[order[k]] >= host_min_len) ++k;
    } else {
        std::vector<uint64_t> sd(total);
        for (uint64_t q = 0; q < total; ++q) sd[q] = L[order[q]];
        k = hybrid_split(sd, host_threads, 4);
    }
    while (k > 0 && L[order[k - 1]] == 0) --k;  // empty chunks stay on the device
    if (k == 0)
        return cdc_chunk_digests_device_batch_async(device, d_data, lens, nbufs, d_cuts, cut_caps, d_results,
                                                    d_digests, d_hist, stream);
    // the device's lists: the host's chunks as empty ones (their rows are overwritten below)
    std::vector<cdc_cut> mod(cuts);
    uint64_t hbytes = 0;
    std::vector<uint64_t> soff(k);  // staging offset of host chunk j (16-B aligned)
    for (size_t j = 0; j < k; ++j) {
        mod[order[j]].length = 0;
        soff[j] = hbytes;
        hbytes += (L[order[j]] + 15) & ~15ull;
    }
    if (!hy_dev(H.d_cuts, H.c_cuts, total * sizeof(cdc_cut)) || !hy_dev(H.d_stage, H.c_stage, hbytes + 64) ||
        !hy_host(H.h_stage, H.hc_stage, hbytes + 64) || !hy_dev(H.d_gj, H.c_gj, k * sizeof(GatherJob)) ||
        !hy_host(H.h_gj, H.hc_gj, k * sizeof(GatherJob)) || !hy_dev(H.d_sj, H.c_sj, k * sizeof(ScatterJob)) ||
        !hy_host(H.h_sj, H.hc_sj, k * sizeof(ScatterJob)) || !hy_dev(H.d_dig, H.c_dig, 32 * k) ||
        !hy_host(H.h_dig, H.hc_dig, 32 * k))
        return CDC_E_DEVICE;
    cdc_cut *dcuts = static_cast<cdc_cut *>(H.d_cuts);
    uint8_t *dstage = static_cast<uint8_t *>(H.d_stage), *hstage = static_cast<uint8_t *>(H.h_stage);
    GatherJob *hgj = static_cast<GatherJob *>(H.h_gj), *dgj = static_cast<GatherJob *>(H.d_gj);
    ScatterJob *hsj = static_cast<ScatterJob *>(H.h_sj), *dsj = static_cast<ScatterJob *>(H.d_sj);
    uint8_t *hdig = static_cast<uint8_t *>(H.h_dig), *ddig = static_cast<uint8_t *>(H.d_dig);
    // From the first enqueue on, every return drains both streams: copies out
    // of the scratch buffers (and gathers from the caller's data) must not
    // outlive this call, whose scratch the next call may free or reuse.
    struct Drain {
        hipStream_t a, b;
        ~Drain()
        {
            (void)hipStreamSynchronize(a);
            (void)hipStreamSynchronize(b);
        }
    } drain{H.side, sm};
    // the copy from pageable memory completes before hipMemcpyAsync returns
    if (hipMemcpyAsync(dcuts, mod.data(), total * sizeof(cdc_cut), hipMemcpyHostToDevice, sm) != hipSuccess)
        return CDC_E_DEVICE;
    // device: SHA-256 of every other chunk (the modified lists), histograms of all (the caller's lists)
    {
        DigestBatch DB;
        std::memset(&DB, 0, sizeof(DB));
        DB.nbufs = uint32_t(nbufs);
        for (int i = 0; i < nbufs; ++i)
            DB.b[i] = DigestBuf{static_cast<const uint8_t *>(d_data[i]), lens[i], dcuts + base[size_t(i)],
                                cnt[size_t(i)], nullptr, d_digests[i], nullptr};
        if ((st = launch_digests(DB, sm, 1)) != CDC_OK) return st;
        if (want_hist) {
            for (int i = 0; i < nbufs; ++i)
                DB.b[i] = DigestBuf{static_cast<const uint8_t *>(d_data[i]), lens[i], d_cuts[i], cnt[size_t(i)],
                                    nullptr, d_digests[i], cnt[size_t(i)] ? d_hist[i] : nullptr};
            if ((st = launch_digests(DB, sm, 2)) != CDC_OK) return st;
        }
        if (hipEventRecord(H.ev_dig, sm) != hipSuccess) return CDC_E_DEVICE;
    }
    // host: the chunks packed on the side stream and copied back in up to
    // four parts (longest first), each hashed as it lands
    for (size_t j = 0; j < k; ++j) {
        const uint64_t q = order[j];
        const int i = bof[q];
        hgj[j] = GatherJob{static_cast<const uint8_t *>(d_data[i]) + cuts[q].offset, L[q], soff[j]};
        hsj[j] = ScatterJob{d_digests[i] + 32 * (q - base[size_t(i)]), ddig + 32 * j};
    }
    if (hipMemcpyAsync(dgj, hgj, k * sizeof(GatherJob), hipMemcpyHostToDevice, H.side) != hipSuccess)
        return CDC_E_DEVICE;
    const size_t nparts = std::min<size_t>(4, k);
    std::vector<size_t> pend(nparts + 1, 0);  // part p: jobs [pend[p], pend[p + 1]), about equal bytes
    for (size_t p = 1; p < nparts; ++p) {
        const uint64_t want = hbytes * p / nparts;
        size_t j = pend[p - 1] + 1;
        while (j < k && soff[j] < want) ++j;
        pend[p] = std::min(j, k);
    }
    pend[nparts] = k;
    for (size_t p = 0; p < nparts; ++p) {
        const size_t j0 = pend[p], j1 = pend[p + 1];
        if (j1 > j0) {
            const uint64_t b0 = soff[j0], b1 = j1 < k ? soff[j1] : hbytes;
            if ((st = launch_gather(dgj + j0, uint32_t(j1 - j0), dstage, H.side)) != CDC_OK) return st;
            if (hipMemcpyAsync(hstage + b0, dstage + b0, b1 - b0, hipMemcpyDeviceToHost, H.side) != hipSuccess)
                return CDC_E_DEVICE;
        }
        if (hipEventRecord(H.ev_part[p], H.side) != hipSuccess) return CDC_E_DEVICE;
    }
    std::atomic<size_t> next{0};
    std::atomic<int> fail{CDC_OK};
    std::vector<std::atomic<int>> landed(nparts);
    for (auto &x : landed) x.store(0);
    std::mutex pmu;
    auto worker = [&]() {
        for (;;) {
            const size_t j = next.fetch_add(1);
            if (j >= k || fail.load() != CDC_OK) return;
            size_t p = 0;
            while (p + 1 < nparts && j >= pend[p + 1]) ++p;
            if (!landed[p].load(std::memory_order_acquire)) {
                std::lock_guard<std::mutex> g(pmu);
                if (!landed[p].load()) {
                    if (hipEventSynchronize(H.ev_part[p]) != hipSuccess) {
                        fail.store(CDC_E_DEVICE);
                        return;
                    }
                    landed[p].store(1, std::memory_order_release);
                }
            }
            sha256(hstage + soff[j], size_t(L[order[j]]), hdig + 32 * j);
        }
    };
    {
        const std::function<void()> job = worker;
        host_pool(device).run(host_threads, job);
    }
    if (fail.load() != CDC_OK) return fail.load();
    // the host's digests into their rows, after the device's digest kernel
    if (hipStreamWaitEvent(H.side, H.ev_dig, 0) != hipSuccess ||
        hipMemcpyAsync(ddig, hdig, 32 * k, hipMemcpyHostToDevice, H.side) != hipSuccess ||
        hipMemcpyAsync(dsj, hsj, k * sizeof(ScatterJob), hipMemcpyHostToDevice, H.side) != hipSuccess)
        return CDC_E_DEVICE;
    if ((st = launch_scatter_digests(dsj, uint32_t(k), H.side)) != CDC_OK) return st;
    if (hipStreamSynchronize(H.side) != hipSuccess || hipStreamSynchronize(sm) != hipSuccess) return CDC_E_DEVICE;
    if (host_chunks) *host_chunks = k;
    if (host_bytes) {
        uint64_t b = 0;
        for (size_t j = 0; j < k; ++j) b += L[order[j]];
        *host_bytes = b;
    }
    return CDC_OK;
}

int cdc_chunk_entropy_device_async(int device, const uint32_t *d_hist, uint64_t rows, double *d_entropy, void *stream)
{
    if (rows && (!d_hist || !d_entropy)) return CDC_E_INVALID;
    DeviceCtx *ctx = nullptr;
    int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    if (hipSetDevice(device) != hipSuccess) return CDC_E_DEVICE;
    return launch_entropy(d_hist, rows, d_entropy, stream);
}

int cdc_chunk(const cdc_buf *bufs, int nbufs, const cdc_opts *opts, cdc_cut *out, uint64_t out_cap,
              uint64_t *out_counts, uint64_t *out_needed)
{
    if (nbufs < 0 || (nbufs > 0 && (!bufs || !out_counts)) || !opts) return CDC_E_INVALID;
    const int v = validate_sizes(opts);
    if (v != CDC_OK) return v;
    Global &g = G();
    if (!g.init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    for (int i = 0; i < nbufs; ++i)
        if (bufs[i].len && !bufs[i].data) return CDC_E_INVALID;
    std::vector<HostJob> jobs(nbufs);
    for (int i = 0; i < nbufs; ++i) {
        jobs[i].data = static_cast<const uint8_t *>(bufs[i].data);
        jobs[i].len = bufs[i].len;
    }
    // LPT assignment of buffers to devices (largest first onto the least loaded)
    const size_t nd = g.devs.size();
    std::vector<std::vector<HostJob *>> per(nd);
    std::vector<uint64_t> load(nd, 0);
    std::vector<int> order(nbufs);
    for (int i = 0; i < nbufs; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return jobs[a].len > jobs[b].len; });
    for (int i : order) {
        if (jobs[i].len == 0) continue;
        const size_t d = size_t(std::min_element(load.begin(), load.end()) - load.begin());
        per[d].push_back(&jobs[i]);
        load[d] += jobs[i].len;
    }
    std::vector<int> status(nd, CDC_OK);
    std::vector<std::thread> threads;
    for (size_t d = 0; d < nd; ++d) {
        if (per[d].empty()) continue;
        threads.emplace_back([&, d] {
            // keep each device's buffers in input order inside its packing
            std::sort(per[d].begin(), per[d].end());
            status[d] = run_host_jobs(g.devs[d], opts, per[d]);
        });
    }
    for (auto &t : threads) t.join();
    for (int s : status)
        if (s != CDC_OK) return s;
    uint64_t total = 0;
    for (auto &j : jobs) total += j.cuts.size();
    if (out_needed) *out_needed = total;
    if (total > out_cap || (total && !out)) {
        for (int i = 0; i < nbufs; ++i) out_counts[i] = jobs[i].cuts.size();
        return CDC_E_NOSPACE;
    }
    uint64_t k = 0;
    for (int i = 0; i < nbufs; ++i) {
        out_counts[i] = jobs[i].cuts.size();
        if (!jobs[i].cuts.empty()) std::memcpy(out + k, jobs[i].cuts.data(), jobs[i].cuts.size() * sizeof(cdc_cut));
        k += jobs[i].cuts.size();
    }
    return CDC_OK;
}

}  // extern "C"

// ===========================================================================
// Pinned batch arena: files read straight into library-owned pinned memory
// (the importer's os.Open + read, snapshot/importer/fs/fs.go:69-71), then one
// cdc_chunk over them (pinned hipMemcpyAsync, no staging copy).  A cgo caller
// hands the library only C memory and file descriptors, never a Go pointer to
// keep.
// ===========================================================================
struct cdc_batch {
    uint8_t *base = nullptr;
    uint64_t cap = 0, used = 0;
    std::vector<cdc_buf> bufs;
};

static constexpr uint64_t kBatchAlign = 4096;

extern "C" int cdc_batch_new(uint64_t capacity, cdc_batch **out)
{
    if (!out) return CDC_E_INVALID;
    *out = nullptr;
    if (!G().init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    auto *b = new cdc_batch();
    b->cap = (capacity + kBatchAlign - 1) & ~(kBatchAlign - 1);
    if (b->cap && hipHostMalloc(reinterpret_cast<void **>(&b->base), b->cap, hipHostMallocPortable) != hipSuccess) {
        delete b;
        return CDC_E_NOMEM;
    }
    *out = b;
    return CDC_OK;
}

extern "C" int cdc_batch_reserve(cdc_batch *b, uint64_t len, uint8_t **ptr)
{
    if (!b || !ptr) return CDC_E_INVALID;
    const uint64_t need = (len + kBatchAlign - 1) & ~(kBatchAlign - 1);
    if (need > b->cap - b->used) return CDC_E_NOSPACE;
    *ptr = b->base + b->used;
    b->bufs.push_back(cdc_buf{len ? b->base + b->used : nullptr, len});
    b->used += need;
    return CDC_OK;
}

static int read_full(int fd, uint8_t *dst, uint64_t len)
{
    uint64_t got = 0;
    while (got < len) {
        const ssize_t k = pread(fd, dst + got, size_t(std::min<uint64_t>(len - got, 1ull << 30)), off_t(got));
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return CDC_E_IO;
        got += uint64_t(k);
    }
    return CDC_OK;
}

// One file into its reserved slot: open, read exactly len bytes, close.  Each
// reader thread holds at most one descriptor, so a batch of any number of
// files stays within RLIMIT_NOFILE.
static int read_path(const char *path, uint8_t *dst, uint64_t len)
{
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return CDC_E_IO;
    const int st = read_full(fd, dst, len);
    close(fd);
    return st;
}

extern "C" int cdc_batch_add_fd(cdc_batch *b, int fd, uint64_t len)
{
    uint8_t *p = nullptr;
    const int st = cdc_batch_reserve(b, len, &p);
    if (st != CDC_OK) return st;
    const int r = read_full(fd, p, len);
    if (r != CDC_OK) {  // drop the slot again
        b->bufs.pop_back();
        b->used = uint64_t(p - b->base);
    }
    return r;
}

extern "C" int cdc_batch_add_files(cdc_batch *b, const char *const *paths, int n, int threads, uint64_t *sizes)
{
    if (!b || n < 0 || (n > 0 && !paths)) return CDC_E_INVALID;
    const size_t first = b->bufs.size();
    const uint64_t used0 = b->used;
    auto undo = [&](int st) {
        b->bufs.resize(first);
        b->used = used0;
        return st;
    };
    for (int i = 0; i < n; ++i) {  // sizes by stat(): no descriptor is held across the batch
        struct stat sb;
        if (!paths[i] || stat(paths[i], &sb) != 0 || !S_ISREG(sb.st_mode)) return undo(CDC_E_IO);
        uint8_t *p = nullptr;
        const int st = cdc_batch_reserve(b, uint64_t(sb.st_size), &p);
        if (st != CDC_OK) return undo(st);
        if (sizes) sizes[i] = uint64_t(sb.st_size);
    }
    const int nt = std::max(1, std::min(threads, n));
    std::atomic<int> next{0}, err{CDC_OK};
    auto work = [&] {
        for (int i; (i = next.fetch_add(1)) < n && err.load() == CDC_OK;) {
            const cdc_buf &cb = b->bufs[first + size_t(i)];
            const int st = read_path(paths[i], static_cast<uint8_t *>(const_cast<void *>(cb.data)), cb.len);
            if (st != CDC_OK) err.store(st);
        }
    };
    try {
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
        work();
        for (auto &t : pool) t.join();
    } catch (...) {
        return undo(CDC_E_NOMEM);
    }
    if (err.load() != CDC_OK) return undo(err.load());
    return CDC_OK;
}

// cdc_batch_add_files + chunking of the added files, overlapped: the files
// are split into consecutive sub-batches of >= kSubBatchBytes; reader threads
// run ahead through the files in order while this thread chunks each
// sub-batch (pinned H2D + kernels, cdc_chunk) as soon as all of its files are
// in the arena.
static constexpr uint64_t kSubBatchBytes = 256ull << 20;

extern "C" int cdc_batch_chunk_files(cdc_batch *b, const char *const *paths, int n, int threads, const cdc_opts *opts,
                                     cdc_cut *out, uint64_t out_cap, uint64_t *out_counts, uint64_t *out_needed,
                                     uint64_t *sizes)
{
    if (!b || n < 0 || (n > 0 && (!paths || !out_counts)) || !opts) return CDC_E_INVALID;
    const int v = validate_sizes(opts);
    if (v != CDC_OK) return v;
    if (!G().init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    const size_t first = b->bufs.size();
    const uint64_t used0 = b->used;
    auto undo = [&](int st) {
        b->bufs.resize(first);
        b->used = used0;
        return st;
    };
    std::vector<int> sub_end;  // file index one past each sub-batch
    uint64_t acc = 0;
    for (int i = 0; i < n; ++i) {  // sizes by stat(); readers open, read and close one file at a time
        struct stat sb;
        if (!paths[i] || stat(paths[i], &sb) != 0 || !S_ISREG(sb.st_mode)) return undo(CDC_E_IO);
        uint8_t *p = nullptr;
        const int st = cdc_batch_reserve(b, uint64_t(sb.st_size), &p);
        if (st != CDC_OK) return undo(st);
        if (sizes) sizes[i] = uint64_t(sb.st_size);
        acc += uint64_t(sb.st_size);
        if (acc >= kSubBatchBytes || i + 1 == n) {
            sub_end.push_back(i + 1);
            acc = 0;
        }
    }
    std::vector<int> sub_of(static_cast<size_t>(n));
    for (size_t j = 0, i = 0; j < sub_end.size(); ++j)
        for (; int(i) < sub_end[j]; ++i) sub_of[i] = int(j);
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> left(sub_end.size());  // files of each sub-batch still being read
    for (size_t j = 0; j < sub_end.size(); ++j) left[j] = sub_end[j] - (j ? sub_end[j - 1] : 0);
    std::atomic<int> next{0}, err{CDC_OK};
    auto work = [&] {
        for (int i; (i = next.fetch_add(1)) < n && err.load() == CDC_OK;) {
            const cdc_buf &cb = b->bufs[first + size_t(i)];
            const int st = read_path(paths[i], static_cast<uint8_t *>(const_cast<void *>(cb.data)), cb.len);
            if (st != CDC_OK) err.store(st);
            std::lock_guard<std::mutex> lk(mu);
            --left[size_t(sub_of[size_t(i)])];
            cv.notify_all();
        }
        std::lock_guard<std::mutex> lk(mu);
        cv.notify_all();
    };
    const int nt = std::max(1, std::min(threads, n));
    std::vector<std::thread> pool;
    try {
        for (int t = 0; t < nt; ++t) pool.emplace_back(work);
    } catch (...) {
        err.store(CDC_E_NOMEM);
        for (auto &t : pool) t.join();
        return undo(CDC_E_NOMEM);
    }
    int status = CDC_OK;
    uint64_t k = 0, needed = 0;
    for (size_t j = 0; j < sub_end.size() && status != CDC_E_IO; ++j) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return left[j] == 0 || err.load() != CDC_OK; });
        }
        if (err.load() != CDC_OK) break;
        const int s0 = j ? sub_end[j - 1] : 0, cnt = sub_end[j] - s0;
        uint64_t need = 0;
        const bool room = status == CDC_OK;
        const int st = cdc_chunk(b->bufs.data() + first + size_t(s0), cnt, opts, room ? out + k : nullptr,
                                 room ? out_cap - k : 0, out_counts + s0, &need);
        needed += need;
        if (st == CDC_OK) k += need;
        else if (st == CDC_E_NOSPACE) status = CDC_E_NOSPACE;  // keep counting what is needed
        else {
            status = st;
            break;
        }
    }
    if (status != CDC_OK && status != CDC_E_NOSPACE) err.store(status);  // readers stop early
    for (auto &t : pool) t.join();
    if (err.load() != CDC_OK) return undo(err.load());
    if (out_needed) *out_needed = needed;
    return status;
}

extern "C" int cdc_batch_count(const cdc_batch *b) { return b ? int(b->bufs.size()) : 0; }

extern "C" int cdc_batch_get(const cdc_batch *b, int i, const uint8_t **ptr, uint64_t *len)
{
    if (!b || i < 0 || size_t(i) >= b->bufs.size() || !ptr || !len) return CDC_E_INVALID;
    *ptr = static_cast<const uint8_t *>(b->bufs[size_t(i)].data);
    *len = b->bufs[size_t(i)].len;
    return CDC_OK;
}

extern "C" int cdc_batch_chunk(cdc_batch *b, const cdc_opts *opts, cdc_cut *out, uint64_t out_cap,
                               uint64_t *out_counts, uint64_t *out_needed)
{
    if (!b) return CDC_E_INVALID;
    return cdc_chunk(b->bufs.data(), int(b->bufs.size()), opts, out, out_cap, out_counts, out_needed);
}

extern "C" void cdc_batch_reset(cdc_batch *b)
{
    if (!b) return;
    b->bufs.clear();
    b->used = 0;
}

extern "C" void cdc_batch_free(cdc_batch *b)
{
    if (!b) return;
    if (b->base) (void)hipHostFree(b->base);
    delete b;
}

// ===========================================================================
// Streaming chunker: ext go-cdc-chunkers (*Chunker).Next over a pinned window.
// ===========================================================================
struct cdc_stream {
    int device = 0;
    cdc_opts opts{};
    DevParams P{};
    uint64_t win = 0;
    uint8_t *h_win = nullptr;  // pinned window; chunks alias it
    uint8_t *d_win = nullptr;
    void *d_ws = nullptr;
    uint64_t ws_bytes = 0;
    cdc_cut *d_cuts = nullptr, *h_cuts = nullptr;
    uint64_t cuts_cap = 0;
    cdc_result *d_res = nullptr, *h_res = nullptr;
    hipStream_t stream = nullptr;
    uint64_t fill = 0;      // bytes in the window
    uint64_t consumed = 0;  // bytes covered by decided chunks of the last run
    uint64_t ncuts = 0, next_cut = 0;
    bool eof = false;
    bool ran = false;
};

static void stream_release(cdc_stream *s)
{
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->h_win) (void)hipHostFree(s->h_win);
    if (s->d_win) (void)hipFree(s->d_win);
    if (s->d_ws) (void)hipFree(s->d_ws);
    if (s->d_cuts) (void)hipFree(s->d_cuts);
    if (s->h_cuts) (void)hipHostFree(s->h_cuts);
    if (s->d_res) (void)hipFree(s->d_res);
    if (s->h_res) (void)hipHostFree(s->h_res);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

extern "C" int cdc_stream_new(const char *algorithm, const cdc_opts *opts, uint64_t window_bytes,
                              int device, cdc_stream **out)
{
    if (!out || !opts) return CDC_E_INVALID;
    *out = nullptr;
    const int v = cdc_validate(algorithm, opts);
    if (v != CDC_OK) return v;
    DeviceCtx *ctx = nullptr;
    int st = check_ready(device, &ctx);
    if (st != CDC_OK) return st;
    auto *s = new cdc_stream();
    s->device = device;
    s->opts = *opts;
    s->P = make_params(opts);
    uint64_t w = window_bytes ? window_bytes : (64ull << 20);
    w = std::max<uint64_t>(w, 2ull * opts->max_size + 4096);
    s->win = w;
    s->cuts_cap = w / opts->min_size + 2;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&s->h_win), w, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&s->d_win), w) != hipSuccess ||
        cdc_device_workspace_size(w, opts, &s->ws_bytes) != CDC_OK ||
        hipMalloc(&s->d_ws, s->ws_bytes) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&s->d_cuts), s->cuts_cap * sizeof(cdc_cut)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&s->h_cuts), s->cuts_cap * sizeof(cdc_cut),
                      hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&s->d_res), sizeof(cdc_result)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&s->h_res), sizeof(cdc_result),
                      hipHostMallocDefault) != hipSuccess) {
        stream_release(s);
        return CDC_E_DEVICE;
    }
    *out = s;
    return CDC_OK;
}

extern "C" int cdc_stream_buffer(cdc_stream *s, uint8_t **write_ptr, uint64_t *space)
{
    if (!s || !write_ptr || !space) return CDC_E_INVALID;
    // drop the bytes of chunks already handed out once every decided chunk was served
    if (s->ran && s->next_cut >= s->ncuts && s->consumed) {
        std::memmove(s->h_win, s->h_win + s->consumed, s->fill - s->consumed);
        s->fill -= s->consumed;
        s->consumed = 0;
        s->ncuts = s->next_cut = 0;
        s->ran = false;
    }
    *write_ptr = s->h_win + s->fill;
    *space = s->win - s->fill;
    return CDC_OK;
}

extern "C" int cdc_stream_commit(cdc_stream *s, uint64_t nbytes, int eof)
{
    if (!s || nbytes > s->win - s->fill) return CDC_E_INVALID;
    s->fill += nbytes;
    if (eof) s->eof = true;
    return CDC_OK;
}

static int stream_run(cdc_stream *s)
{
    if (hipSetDevice(s->device) != hipSuccess) return CDC_E_DEVICE;
    // The plan is not monotonic in the length (the scan lane rounds up to
    // 256 B), so a shorter final fill can need more workspace than the window.
    s->P = make_params(&s->opts);  // the library's current masks (cdc_init may have changed them)
    uint64_t need = 0;
    int wst = cdc_device_workspace_size(s->fill, &s->opts, &need);
    if (wst != CDC_OK) return wst;
    if (need > s->ws_bytes) {
        HIPCHK(hipStreamSynchronize(s->stream));
        if (s->d_ws) (void)hipFree(s->d_ws);
        s->d_ws = nullptr;
        s->ws_bytes = 0;
        if (hipMalloc(&s->d_ws, need) != hipSuccess) return CDC_E_NOMEM;
        s->ws_bytes = need;
    }
    HIPCHK(hipMemcpyAsync(s->d_win, s->h_win, s->fill, hipMemcpyHostToDevice, s->stream));
    const int st = cdc_chunk_device_async(s->device, s->d_win, s->fill, s->eof ? 1 : 0, &s->opts,
                                          s->d_cuts, s->cuts_cap, s->d_res, s->d_ws, s->ws_bytes,
                                          s->stream);
    if (st != CDC_OK) return st;
    HIPCHK(hipMemcpyAsync(s->h_res, s->d_res, sizeof(cdc_result), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    const cdc_result r = *s->h_res;
    if (r.status != CDC_OK) return int(r.status);
    if (r.ncuts)
        HIPCHK(hipMemcpy(s->h_cuts, s->d_cuts, r.ncuts * sizeof(cdc_cut), hipMemcpyDeviceToHost));
    s->ncuts = r.ncuts;
    s->next_cut = 0;
    s->consumed = s->eof ? s->fill : r.consumed;
    s->ran = true;
    return CDC_OK;
}

extern "C" int cdc_stream_next(cdc_stream *s, const uint8_t **chunk, uint64_t *len)
{
    if (!s || !chunk || !len) return CDC_E_INVALID;
    *chunk = nullptr;
    *len = 0;
    for (;;) {
        if (s->ran && s->next_cut < s->ncuts) {
            const cdc_cut c = s->h_cuts[s->next_cut++];
            *chunk = s->h_win + c.offset;
            *len = c.length;
            return CDC_OK;
        }
        if (s->ran) {
            // every decided chunk served: drop them from the window
            std::memmove(s->h_win, s->h_win + s->consumed, s->fill - s->consumed);
            s->fill -= s->consumed;
            s->consumed = 0;
            s->ncuts = s->next_cut = 0;
            s->ran = false;
        }
        if (s->eof && s->fill == 0) return CDC_EOF;
        if (!s->eof && s->fill < s->win) return CDC_NEED_DATA;
        const int st = stream_run(s);
        if (st != CDC_OK) return st;
    }
}

extern "C" void cdc_stream_free(cdc_stream *s) { stream_release(s); }

// Pull-model chunker over a read callback.
struct cdc_chunker {
    cdc_stream *s = nullptr;
    cdc_read_fn read = nullptr;
    void *ctx = nullptr;
};

extern "C" int cdc_chunker_new(const char *algorithm, cdc_read_fn read, void *ctx,
                               const cdc_opts *opts, cdc_chunker **out)
{
    if (!read || !out) return CDC_E_INVALID;
    *out = nullptr;
    cdc_stream *s = nullptr;
    Global &g = G();
    if (!g.init.load(std::memory_order_acquire)) return CDC_E_NOT_INIT;
    const int st = cdc_stream_new(algorithm, opts, 0, g.devs.front()->device, &s);
    if (st != CDC_OK) return st;
    auto *c = new cdc_chunker();
    c->s = s;
    c->read = read;
    c->ctx = ctx;
    *out = c;
    return CDC_OK;
}

extern "C" int cdc_chunker_next(cdc_chunker *c, const uint8_t **chunk, uint64_t *len)
{
    if (!c) return CDC_E_INVALID;
    for (;;) {
        const int st = cdc_stream_next(c->s, chunk, len);
        if (st != CDC_NEED_DATA) return st;
        uint8_t *p = nullptr;
        uint64_t space = 0;
        int r = cdc_stream_buffer(c->s, &p, &space);
        if (r != CDC_OK) return r;
        while (space > 0) {
            const int64_t n = c->read(c->ctx, p, space);
            if (n < 0) return CDC_E_IO;
            if (n == 0) {
                r = cdc_stream_commit(c->s, 0, 1);
                break;
            }
            r = cdc_stream_commit(c->s, uint64_t(n), 0);
            if (r != CDC_OK) return r;
            p += n;
            space -= uint64_t(n);
        }
        if (r != CDC_OK) return r;
    }
}

extern "C" void cdc_chunker_free(cdc_chunker *c)
{
    if (!c) return;
    cdc_stream_free(c->s);
    delete c;
}
