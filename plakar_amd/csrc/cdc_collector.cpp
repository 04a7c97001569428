// Per-process collector: concurrent per-file callers -> device batches.
//
// plakar chunks each file in its own goroutine (the scanner fan-out of
// snapshot/backup.go:216-225, up to NumCPU x 8 + 1 at once, each running the
// per-file Next() loop of snapshot/backup.go:647-665).  One launch group per
// file would leave the GPU mostly idle on small files and pay a PCIe round
// trip per call.  A collector takes those calls from any number of threads,
// queues them, and a worker thread hands them to the device as batches: a
// batch closes when its bytes reach batch_bytes, when it holds 64 files, or
// max_wait_us after its first file arrived.  Each batch is one cdc_chunk call
// (LPT over the devices, pipelined H2D); every caller blocks until its own cut
// list is back, so the calling contract is the synchronous one of cdc_chunk
// for one buffer.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "cdc_internal.h"

namespace {

struct Request {
    const void *data;
    uint64_t len;
    cdc_cut *out;
    uint64_t cap;
    uint64_t count = 0;
    int status = CDC_OK;
    bool done = false;
};

constexpr size_t kMaxBatchFiles = 64;

}  // namespace

struct cdc_collector {
    cdc_opts opts;
    uint64_t batch_bytes;
    std::chrono::microseconds max_wait;
    std::mutex mu;
    std::condition_variable cv_work;  // worker: a request arrived / shutting down
    std::condition_variable cv_done;  // callers: a batch finished
    std::deque<Request *> queue;
    uint64_t queued_bytes = 0;
    std::chrono::steady_clock::time_point first_arrival;
    bool stop = false;
    uint64_t n_requests = 0, n_batches = 0;
    std::thread worker;

    void run();
};

void cdc_collector::run()
{
    std::vector<Request *> batch;
    std::vector<cdc_buf> bufs;
    std::vector<uint64_t> counts;
    std::vector<cdc_cut> cuts;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                if (queue.empty()) {
                    if (stop) return;
                    cv_work.wait(lk);
                    continue;
                }
                if (stop || queued_bytes >= batch_bytes || queue.size() >= kMaxBatchFiles) break;
                const auto deadline = first_arrival + max_wait;
                if (std::chrono::steady_clock::now() >= deadline) break;
                cv_work.wait_until(lk, deadline);
            }
            batch.clear();
            uint64_t bytes = 0;
            while (!queue.empty() && batch.size() < kMaxBatchFiles && (batch.empty() || bytes < batch_bytes)) {
                batch.push_back(queue.front());
                bytes += queue.front()->len;
                queue.pop_front();
            }
            queued_bytes -= bytes;
            if (!queue.empty()) first_arrival = std::chrono::steady_clock::now();
            ++n_batches;
        }
        // one cdc_chunk over the batch: cut lists into a scratch array sized by
        // the bound len / Min + 2 per buffer, then copied to each caller
        bufs.resize(batch.size());
        counts.assign(batch.size(), 0);
        uint64_t cap = 0;
        for (size_t i = 0; i < batch.size(); ++i) {
            bufs[i].data = batch[i]->data;
            bufs[i].len = batch[i]->len;
            cap += batch[i]->len / (opts.min_size ? opts.min_size : 1) + 2;
        }
        cuts.resize(cap);
        uint64_t needed = 0;
        const int st = cdc_chunk(bufs.data(), int(bufs.size()), &opts, cuts.data(), cap, counts.data(), &needed);
        {
            std::lock_guard<std::mutex> lk(mu);
            uint64_t k = 0;
            for (size_t i = 0; i < batch.size(); ++i) {
                Request *r = batch[i];
                r->count = counts[i];
                if (st != CDC_OK) {
                    r->status = st;
                } else if (counts[i] > r->cap || (counts[i] && !r->out)) {
                    r->status = CDC_E_NOSPACE;
                } else {
                    if (counts[i]) std::memcpy(r->out, cuts.data() + k, counts[i] * sizeof(cdc_cut));
                    r->status = CDC_OK;
                }
                k += counts[i];
                r->done = true;
            }
        }
        cv_done.notify_all();
    }
}

extern "C" {

int cdc_collector_new(const cdc_opts *opts, uint64_t batch_bytes, uint32_t max_wait_us, cdc_collector **out)
{
    if (!opts || !out) return CDC_E_INVALID;
    const int v = cdc_validate("fastcdc", opts);
    if (v != CDC_OK) return v;
    auto *c = new cdc_collector();
    c->opts = *opts;
    c->batch_bytes = batch_bytes ? batch_bytes : (256ull << 20);
    c->max_wait = std::chrono::microseconds(max_wait_us);
    c->worker = std::thread([c] { c->run(); });
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
    Request r{data, len, out, cap};
    {
        std::unique_lock<std::mutex> lk(c->mu);
        if (c->stop) return CDC_E_INVALID;
        if (c->queue.empty()) c->first_arrival = std::chrono::steady_clock::now();
        c->queue.push_back(&r);
        c->queued_bytes += len;
        ++c->n_requests;
        c->cv_work.notify_one();
        c->cv_done.wait(lk, [&] { return r.done; });
    }
    *count = r.count;
    return r.status;
}

int cdc_collector_stats(cdc_collector *c, uint64_t *requests, uint64_t *batches)
{
    if (!c || !requests || !batches) return CDC_E_INVALID;
    std::lock_guard<std::mutex> lk(c->mu);
    *requests = c->n_requests;
    *batches = c->n_batches;
    return CDC_OK;
}

// Drains the queue (pending callers still get their results), then stops the
// worker.  No call may be made on c afterwards.
void cdc_collector_free(cdc_collector *c)
{
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->stop = true;
    }
    c->cv_work.notify_all();
    if (c->worker.joinable()) c->worker.join();
    delete c;
}

}  // extern "C"
