// Per-process collector: concurrent per-file callers -> device batches.
//
// plakar chunks each file in its own goroutine (the scanner fan-out of
// snapshot/backup.go:216-225, up to NumCPU x 8 + 1 at once, each running the
// per-file Next() loop of snapshot/backup.go:647-665).  One launch group per
// file would leave the GPU mostly idle on small files and pay a PCIe round
// trip per call.  A collector takes those calls from any number of threads
// and queues them; one worker per device pulls batches from the shared queue
// (dynamic balance across devices) and runs them through a two-slot pipeline
// that outlives a batch (cdc::pipeline_device): batch k + 1 is staged (H2D)
// while batch k is chunked, and batch k's cut lists come back while k + 1
// runs.  A batch closes when its bytes reach batch_bytes, when it holds
// kMaxBufsPerLaunch files, or max_wait_us after its first file arrived (the
// wait applies while the device is idle; with a batch in flight a closed
// batch is taken as soon as it is closed).  Every caller blocks until its own
// cut list is back: the calling contract is the synchronous one of cdc_chunk
// for one buffer.  No C++ exception crosses the C ABI.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "cdc_internal.h"

namespace {

struct Request : cdc::HostBuf {
    cdc_cut *out;
    uint64_t cap;
    uint64_t count = 0;
    bool done = false;
};

constexpr size_t kMaxBatchFiles = cdc::kMaxBufsPerLaunch;

}  // namespace

struct cdc_collector final : cdc::BatchSource {
    cdc_opts opts;
    uint64_t batch_bytes;
    std::chrono::microseconds max_wait;
    std::mutex mu;
    std::condition_variable cv_work;  // workers: a request arrived / shutting down
    std::condition_variable cv_done;  // callers: a batch finished; free(): the last caller left
    std::deque<Request *> queue;
    uint64_t queued_bytes = 0;
    std::chrono::steady_clock::time_point first_arrival;
    bool stop = false;
    uint64_t n_requests = 0, n_batches = 0;
    uint64_t callers = 0;  // threads inside cdc_collector_chunk
    int live = 0;          // workers still serving the queue
    std::vector<std::thread> workers;

    bool closed(std::chrono::steady_clock::time_point now) const
    {
        return stop || queued_bytes >= batch_bytes || queue.size() >= kMaxBatchFiles || now >= first_arrival + max_wait;
    }

    bool next(std::vector<cdc::HostBuf *> &batch, bool wait) override
    {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (queue.empty()) {
                if (stop || !wait) return false;
                cv_work.wait(lk);
                continue;
            }
            const auto now = std::chrono::steady_clock::now();
            if (closed(now)) break;
            if (!wait) return false;
            cv_work.wait_until(lk, first_arrival + max_wait);
        }
        uint64_t bytes = 0;
        while (!queue.empty() && batch.size() < kMaxBatchFiles && (batch.empty() || bytes + queue.front()->len <= batch_bytes)) {
            batch.push_back(static_cast<cdc::HostBuf *>(queue.front()));
            bytes += queue.front()->len;
            queue.pop_front();
        }
        queued_bytes -= bytes;
        if (!queue.empty()) first_arrival = std::chrono::steady_clock::now();
        ++n_batches;
        return true;
    }

    void finished(std::vector<cdc::HostBuf *> &batch) override
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            for (cdc::HostBuf *h : batch) {
                Request *r = static_cast<Request *>(h);
                r->count = h->cuts.size();
                if (h->status != CDC_OK) {
                    r->count = 0;
                } else if (r->count > r->cap || (r->count && !r->out)) {
                    h->status = CDC_E_NOSPACE;
                } else if (r->count) {
                    std::memcpy(r->out, h->cuts.data(), r->count * sizeof(cdc_cut));
                }
                r->done = true;
            }
        }
        cv_done.notify_all();
    }

    void fail_all(int st)  // a worker could not run: nobody may wait forever
    {
        std::vector<cdc::HostBuf *> b;
        {
            std::lock_guard<std::mutex> lk(mu);
            for (Request *r : queue) b.push_back(r);
            queue.clear();
            queued_bytes = 0;
        }
        for (cdc::HostBuf *h : b) h->status = st;
        if (!b.empty()) finished(b);
    }

    void run(int dev)
    {
        int st;
        try {
            st = cdc::pipeline_device(dev, &opts, *this);
        } catch (const std::bad_alloc &) {
            st = CDC_E_NOMEM;
        } catch (...) {
            st = CDC_E_DEVICE;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            --live;  // the last worker gone: new calls fail at once (cdc_collector_chunk)
        }
        if (st != CDC_OK) fail_all(st);
    }
};

extern "C" {

int cdc_collector_new(const cdc_opts *opts, uint64_t batch_bytes, uint32_t max_wait_us, cdc_collector **out)
{
    if (!opts || !out) return CDC_E_INVALID;
    const int v = cdc_validate("fastcdc", opts);
    if (v != CDC_OK) return v;
    const int ndev = cdc::device_count_initialised();
    if (ndev <= 0) return CDC_E_NOT_INIT;
    auto *c = new (std::nothrow) cdc_collector();
    if (!c) return CDC_E_NOMEM;
    c->opts = *opts;
    c->batch_bytes = batch_bytes ? batch_bytes : (256ull << 20);
    c->max_wait = std::chrono::microseconds(max_wait_us);
    try {
        c->live = ndev;
        for (int d = 0; d < ndev; ++d) c->workers.emplace_back([c, d] { c->run(d); });
    } catch (...) {
        {
            std::lock_guard<std::mutex> lk(c->mu);
            c->stop = true;
        }
        c->cv_work.notify_all();
        for (auto &t : c->workers) t.join();
        delete c;
        return CDC_E_NOMEM;
    }
    *out = c;
    return CDC_OK;
}

// Chunk one whole buffer (a file) through the collector: blocks until the
// batch holding it is done.  Same outputs as cdc_chunk for one buffer:
// *count = its cuts; CDC_E_NOSPACE (with *count set) when cap is too small.
int cdc_collector_chunk(cdc_collector *c, const void *data, uint64_t len, cdc_cut *out, uint64_t cap,
                        uint64_t *count)
{
    if (!c || !count || (len && !data)) return CDC_E_INVALID;
    Request r;
    r.data = static_cast<const uint8_t *>(data);
    r.len = len;
    r.status = CDC_OK;
    r.out = out;
    r.cap = cap;
    std::unique_lock<std::mutex> lk(c->mu);
    if (c->stop) return CDC_E_INVALID;
    if (c->live <= 0) return CDC_E_DEVICE;  // every worker failed: nobody would serve the call
    ++c->callers;
    try {
        if (c->queue.empty()) c->first_arrival = std::chrono::steady_clock::now();
        c->queue.push_back(&r);
    } catch (...) {
        --c->callers;
        c->cv_done.notify_all();
        return CDC_E_NOMEM;
    }
    c->queued_bytes += len;
    ++c->n_requests;
    c->cv_work.notify_all();
    c->cv_done.wait(lk, [&] { return r.done; });
    *count = r.count;
    const int st = r.status;
    --c->callers;              // after this, free() may delete c: touch nothing of c below
    c->cv_done.notify_all();
    return st;
}

int cdc_collector_stats(cdc_collector *c, uint64_t *requests, uint64_t *batches)
{
    if (!c || !requests || !batches) return CDC_E_INVALID;
    std::lock_guard<std::mutex> lk(c->mu);
    *requests = c->n_requests;
    *batches = c->n_batches;
    return CDC_OK;
}

// Stops taking new calls, lets the workers finish every queued call (pending
// callers still get their results), joins them, and waits until every caller
// has left cdc_collector_chunk before freeing c.  It may run while callers
// are blocked in cdc_collector_chunk; no call may START on c once free began.
void cdc_collector_free(cdc_collector *c)
{
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->stop = true;
    }
    c->cv_work.notify_all();
    for (auto &t : c->workers)
        if (t.joinable()) t.join();
    {
        std::unique_lock<std::mutex> lk(c->mu);
        c->cv_done.wait(lk, [&] { return c->callers == 0; });
    }
    delete c;
}

}  // extern "C"
