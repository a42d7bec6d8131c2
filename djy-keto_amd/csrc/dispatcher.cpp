// Request coalescing for serving: the batching dispatcher a Go
// cgo shim puts behind check.Engine.CheckIsMember / the gRPC CheckService handler
// (check/handler.go:304-331).
//
// The reference evaluates every request on its own goroutine.  Here concurrent callers
// block in keto_dispatcher_check while `inflight` slots (a worker thread + a HIP stream
// with its own scratch each) do the batching:
//   - a free slot takes every request queued since the last launch (up to max_batch
//     queries; a request is never split);
//   - it packs them into pinned host memory and runs them as one batch (H2D -> resolve +
//     interpreter kernels -> D2H, one stream, one synchronisation);
//   - it scatters the decisions back to the callers.
// While batches are on the GPU, new requests queue up, so the batch size follows the load
// with no timer (max_wait_us > 0 adds an explicit coalescing window).  A batch lasts as
// long as its longest query; several batches in flight on their own streams keep the CUs
// busy that a small batch's finished lanes leave idle.  The snapshot can be
// swapped between batches (keto_dispatcher_set_snapshot), which is how a new snaptoken's
// snapshot goes live without stopping the service: a slot captures the current snapshot
// (and counts itself as a user of it) when it takes a batch, a swap replaces the pointer at
// once and then waits only for the old snapshot's users to drain -- it cannot be starved by
// a stream of overlapping batches.
//
// Expand requests (expand.Engine.BuildTree behind ExpandService.Expand, expand/handler.go:
// 115-152) coalesce the same way on their own queue: a slot takes either Check or Expand
// requests, runs one keto_expand_batch over all their roots and hands every caller its own
// trees (node ranges rebased to the caller's buffer).
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"

namespace keto {
namespace {

struct Request {
    const keto_query *q = nullptr;
    uint64_t n = 0;
    uint8_t *allowed = nullptr;
    int32_t *err = nullptr;
    // Expand requests: roots in, nodes + offsets[n+1] out
    const keto_subject_set *roots = nullptr;
    keto_tree_node *nodes = nullptr;
    uint64_t cap = 0;
    uint64_t *offsets = nullptr;
    int rc = KETO_OK;
    std::string msg;
    bool done = false;
    std::condition_variable cv;
};

struct Dispatcher;

// one in-flight batch: its own stream (and so its own scratch), staging and worker thread
struct Slot {
    Dispatcher *d = nullptr;
    keto_stream *stream = nullptr;
    keto_query *hq = nullptr;  // pinned staging for max_batch records
    uint8_t *ha = nullptr;
    int32_t *he = nullptr;
    void *dq = nullptr, *da = nullptr, *de = nullptr;
    std::thread th;

    // Expand: pinned node buffer grown on demand (keto_expand_batch_spans writes the trees into it
    // as their walks end), each root's run and error
    keto_tree_node *xnodes = nullptr;
    uint64_t xcap = 0;
    std::vector<uint64_t> xfirst;
    std::vector<uint32_t> xcount;
    std::vector<int32_t> xerr;

    void run();
    int launch(keto_snapshot *snap, uint64_t n, std::string &msg);
    void run_expand(keto_snapshot *snap, std::vector<Request *> &take);
};

struct Dispatcher {
    keto_snapshot *snap = nullptr;
    keto_limits limits{5, 100};
    uint32_t max_batch = 1u << 16, max_wait_us = 0, flags = 0;
    int device = 0;
    std::mutex m;                // queues, stats, snapshot pointer and its users
    std::condition_variable cv_in;
    std::condition_variable cv_idle;  // a snapshot's last in-flight batch finished
    std::deque<Request *> queue, xqueue;
    uint64_t queued = 0;
    std::unordered_map<keto_snapshot *, uint32_t> users;  // batches in flight per snapshot
    bool stop = false;
    std::vector<std::unique_ptr<Slot>> slots;
    keto_dispatcher_stats stats{};
    keto_batch_hook on_batch = nullptr;
    void *hook_ctx = nullptr;
};

double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// one packed batch through the device: async copies around the kernels, one sync
int Slot::launch(keto_snapshot *snap, uint64_t n, std::string &msg) {
    hipStream_t hs = reinterpret_cast<Stream *>(stream)->stream;
    int rc = KETO_OK;
    try {
        KETO_HIP(hipMemcpyAsync(dq, hq, n * sizeof(keto_query), hipMemcpyHostToDevice, hs));
        rc = keto_check_batch(snap, stream, static_cast<const keto_query *>(dq), n, &d->limits,
                              static_cast<uint8_t *>(da), static_cast<int32_t *>(de),
                              KETO_F_DEVICE_PTRS | KETO_F_ASYNC | d->flags);
        if (rc == KETO_OK) {
            KETO_HIP(hipMemcpyAsync(ha, da, n, hipMemcpyDeviceToHost, hs));
            KETO_HIP(hipMemcpyAsync(he, de, n * sizeof(int32_t), hipMemcpyDeviceToHost, hs));
            if (keto_stream_sync(stream) != KETO_OK) throw Error(KETO_E_DEVICE, "stream synchronisation failed");
        } else {
            char buf[512];
            keto_last_error(buf, sizeof(buf));
            msg = buf;
        }
    } catch (const Error &e) {
        rc = e.code;
        msg = e.what();
    }
    return rc;
}

// Expand batch for every taken request: one keto_expand_batch_spans over all roots (each tree
// lands in the pinned buffer as its walk ends), then each caller's trees are copied to its
// buffer in its roots' order, with offsets from 0
void Slot::run_expand(keto_snapshot *snap, std::vector<Request *> &take) {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t n = 0;
    for (auto *r : take) n += r->n;
    int rc = KETO_OK;
    std::string msg;
    std::vector<keto_subject_set> roots;
    roots.reserve(n);
    for (auto *r : take) roots.insert(roots.end(), r->roots, r->roots + r->n);
    xfirst.assign(n, 0);
    xcount.assign(n, 0);
    xerr.assign(n, 0);
    uint64_t total = 1u << 16;
    for (int attempt = 0; attempt < 3; attempt++) {
        if (xcap < total) {  // (first call, or the size the last attempt reported)
            if (xnodes) (void)hipHostFree(xnodes);
            xnodes = nullptr;
            xcap = 0;
            const uint64_t want = std::max<uint64_t>(total + total / 4, 1u << 16);
            if (keto_host_alloc(want * sizeof(keto_tree_node), reinterpret_cast<void **>(&xnodes)) != KETO_OK) {
                rc = KETO_E_DEVICE;
                break;
            }
            xcap = want;
        }
        keto_stream_expand_time(stream, nullptr, nullptr, 1);
        rc = keto_expand_batch_spans(snap, stream, roots.data(), n, &d->limits, xnodes, xcap, xfirst.data(), xcount.data(),
                                     xerr.data(), &total);
        if (rc != KETO_E_CAPACITY) break;
    }
    if (rc != KETO_OK) {
        char buf[512];
        keto_last_error(buf, sizeof(buf));
        msg = buf;
    }
    double dms = 0;
    keto_stream_expand_time(stream, &dms, nullptr, 1);
    const keto_batch_event ev{1, (uint32_t)take.size(), n, ms_since(t0), dms, rc};
    uint64_t o = 0;
    std::unique_lock<std::mutex> lk(d->m);
    for (auto *r : take) {
        int rrc = rc;
        std::string rmsg = msg;
        if (rc == KETO_OK) {
            uint64_t need = 0;
            r->offsets[0] = 0;
            for (uint64_t i = 0; i < r->n; i++) r->offsets[i + 1] = need += xcount[o + i];
            std::memcpy(r->err, xerr.data() + o, r->n * sizeof(int32_t));
            if (need > r->cap || (need && !r->nodes)) {
                rrc = KETO_E_CAPACITY;
                rmsg = "expand output needs " + std::to_string(need) + " nodes";
            } else {
                for (uint64_t i = 0; i < r->n; i++)
                    if (xcount[o + i]) std::memcpy(r->nodes + r->offsets[i], xnodes + xfirst[o + i], xcount[o + i] * sizeof(keto_tree_node));
            }
        }
        o += r->n;
        r->rc = rrc;
        r->msg = rmsg;
        r->done = true;
        r->cv.notify_one();
    }
    d->stats.batches++;
    d->stats.queries += n;
    d->stats.requests += take.size();
    d->stats.wall_ms_sum += ev.wall_ms;
    d->stats.device_ms_sum += ev.device_ms;
    if (n > d->stats.max_batch_seen) d->stats.max_batch_seen = n;
    lk.unlock();
    if (d->on_batch) d->on_batch(d->hook_ctx, &ev);
}

void Slot::run() {
    std::vector<Request *> take;
    for (;;) {
        keto_snapshot *snap = nullptr;
        bool expand = false;
        {
            std::unique_lock<std::mutex> lk(d->m);
            d->cv_in.wait(lk, [&] { return d->stop || !d->queue.empty() || !d->xqueue.empty(); });
            if (d->stop && d->queue.empty() && d->xqueue.empty()) return;
            if (d->max_wait_us && !d->queue.empty()) {
                const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(d->max_wait_us);
                d->cv_in.wait_until(lk, until, [&] { return d->stop || d->queued >= d->max_batch; });
            }
            // Check first; Expand requests (rare, latency-tolerant) when no Check is waiting
            std::deque<Request *> &qq = !d->queue.empty() ? d->queue : d->xqueue;
            if (qq.empty()) continue;  // another slot took them
            expand = &qq == &d->xqueue;
            take.clear();
            uint64_t n = 0;
            while (!qq.empty() && (take.empty() || n + qq.front()->n <= d->max_batch)) {
                n += qq.front()->n;
                if (!expand) d->queued -= qq.front()->n;
                take.push_back(qq.front());
                qq.pop_front();
            }
            snap = d->snap;  // captured with the batch: a swap never waits on later batches
            d->users[snap]++;
        }
        auto release = [&] {  // called with d->m held
            if (--d->users[snap] == 0) {
                d->users.erase(snap);
                d->cv_idle.notify_all();
            }
        };
        if (expand) {
            run_expand(snap, take);
            std::lock_guard<std::mutex> lk(d->m);
            release();
            continue;
        }
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t n = 0;
        for (auto *r : take) n += r->n;
        int rc = KETO_OK;
        std::string msg;
        const bool staged = n <= d->max_batch;
        if (staged) {
            uint64_t o = 0;
            for (auto *r : take) {
                std::memcpy(hq + o, r->q, r->n * sizeof(keto_query));
                o += r->n;
            }
            rc = launch(snap, n, msg);
        } else {  // a single request larger than the staging: the host-pointer path
            Request *r = take[0];
            rc = keto_check_batch(snap, stream, r->q, r->n, &d->limits, r->allowed, r->err, d->flags);
            if (rc != KETO_OK) {
                char buf[512];
                keto_last_error(buf, sizeof(buf));
                msg = buf;
            }
        }
        double dms = 0;
        keto_stream_last_kernel_ms(stream, &dms);
        const keto_batch_event ev{0, (uint32_t)take.size(), n, ms_since(t0), dms, rc};
        uint64_t o = 0;
        std::unique_lock<std::mutex> lk(d->m);
        release();
        for (auto *r : take) {
            if (rc == KETO_OK && staged) {
                std::memcpy(r->allowed, ha + o, r->n);
                std::memcpy(r->err, he + o, r->n * sizeof(int32_t));
            }
            o += r->n;
            r->rc = rc;
            r->msg = msg;
            r->done = true;
            r->cv.notify_one();
        }
        d->stats.batches++;
        d->stats.queries += n;
        d->stats.requests += take.size();
        d->stats.wall_ms_sum += ev.wall_ms;
        d->stats.device_ms_sum += ev.device_ms;
        if (n > d->stats.max_batch_seen) d->stats.max_batch_seen = n;
        lk.unlock();
        if (d->on_batch) d->on_batch(d->hook_ctx, &ev);
    }
}

Dispatcher *DP(keto_dispatcher *d) { return reinterpret_cast<Dispatcher *>(d); }

void release_slot(Slot *x) {
    if (x->stream) keto_stream_destroy(x->stream);
    if (x->hq) (void)hipHostFree(x->hq);
    if (x->ha) (void)hipHostFree(x->ha);
    if (x->he) (void)hipHostFree(x->he);
    if (x->xnodes) (void)hipHostFree(x->xnodes);
    if (x->dq) (void)hipFree(x->dq);
    if (x->da) (void)hipFree(x->da);
    if (x->de) (void)hipFree(x->de);
}

void shutdown(Dispatcher *d) {
    {
        std::lock_guard<std::mutex> lk(d->m);
        d->stop = true;
    }
    d->cv_in.notify_all();
    for (auto &x : d->slots)
        if (x->th.joinable()) x->th.join();
    for (auto &x : d->slots) release_slot(x.get());
    delete d;
}

}  // namespace

void dispatcher_create(keto_snapshot *snap, const keto_dispatcher_config *cfg, keto_dispatcher **out) {
    if (!snap || !cfg || !out) throw Error(KETO_E_INVALID, "null argument");
    if (cfg->max_batch == 0 || cfg->max_batch > (1u << 24)) throw Error(KETO_E_INVALID, "max_batch out of range");
    if (cfg->inflight > 16) throw Error(KETO_E_INVALID, "inflight out of range (0..16)");
    const keto_limits &l = cfg->limits;
    if (l.max_read_depth < 1 || l.max_read_depth > 65535 || l.max_read_width < 1 || l.max_read_width > 65535)
        throw Error(KETO_E_INVALID, "limits out of range");
    auto *d = new Dispatcher();
    d->snap = snap;
    d->limits = l;
    d->max_batch = cfg->max_batch;
    d->max_wait_us = cfg->max_wait_us;
    d->flags = cfg->flags & KETO_F_ERR_DETAIL;
    d->on_batch = cfg->on_batch;
    d->hook_ctx = cfg->hook_ctx;
    d->device = reinterpret_cast<Snapshot *>(snap)->device;
    try {
        KETO_HIP(hipSetDevice(d->device));
        const size_t nb = cfg->max_batch;
        const uint32_t k = cfg->inflight ? cfg->inflight : 4;
        for (uint32_t i = 0; i < k; i++) {
            d->slots.push_back(std::make_unique<Slot>());
            Slot *x = d->slots.back().get();
            x->d = d;
            if (keto_stream_create(d->device, &x->stream) != KETO_OK)
                throw Error(KETO_E_DEVICE, "stream creation failed");
            KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&x->hq), nb * sizeof(keto_query), 0));
            KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&x->ha), nb, 0));
            KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&x->he), nb * sizeof(int32_t), 0));
            KETO_HIP(hipMalloc(&x->dq, nb * sizeof(keto_query)));
            KETO_HIP(hipMalloc(&x->da, nb));
            KETO_HIP(hipMalloc(&x->de, nb * sizeof(int32_t)));
        }
        // every slot's scratch is allocated now, for its largest batch (one max_batch batch of
        // empty queries on its stream), not by its first live batches: an allocation synchronises
        // the device, which would stall the other slots' batches in flight
        for (auto &x : d->slots) {
            std::memset(x->hq, 0, nb * sizeof(keto_query));
            if (keto_check_batch(snap, x->stream, x->hq, nb, &d->limits, x->ha, x->he, 0) != KETO_OK)
                throw Error(KETO_E_DEVICE, "dispatcher slot warm-up failed");
        }
        for (auto &x : d->slots) {
            Slot *p = x.get();
            p->th = std::thread([p] {
                (void)hipSetDevice(p->d->device);
                p->run();
            });
        }
    } catch (...) {
        shutdown(d);
        throw;
    }
    *out = reinterpret_cast<keto_dispatcher *>(d);
}

void dispatcher_destroy(keto_dispatcher *hd) {
    if (Dispatcher *d = DP(hd)) shutdown(d);
}

int dispatcher_check(keto_dispatcher *hd, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err,
                     std::string &msg) {
    Dispatcher *d = DP(hd);
    if (!d) throw Error(KETO_E_INVALID, "null dispatcher");
    if (n == 0) return KETO_OK;
    if (!q || !allowed || !err) throw Error(KETO_E_INVALID, "null buffer");
    Request r;
    r.q = q;
    r.n = n;
    r.allowed = allowed;
    r.err = err;
    std::unique_lock<std::mutex> lk(d->m);
    if (d->stop) throw Error(KETO_E_INVALID, "dispatcher is shutting down");
    d->queue.push_back(&r);
    d->queued += n;
    d->cv_in.notify_one();
    r.cv.wait(lk, [&] { return r.done; });
    msg = r.msg;
    return r.rc;
}

void dispatcher_set_snapshot(keto_dispatcher *hd, keto_snapshot *snap) {
    Dispatcher *d = DP(hd);
    if (!d || !snap) throw Error(KETO_E_INVALID, "null argument");
    if (reinterpret_cast<Snapshot *>(snap)->device != d->device)
        throw Error(KETO_E_INVALID, "snapshot is on another device");
    std::unique_lock<std::mutex> lk(d->m);
    keto_snapshot *old = d->snap;
    d->snap = snap;  // batches taken from now on run on the new snapshot
    if (old == snap) return;
    // when this returns the old snapshot is idle: only batches taken before the swap use it
    d->cv_idle.wait(lk, [&] { return d->users.find(old) == d->users.end(); });
}

int dispatcher_expand(keto_dispatcher *hd, const keto_subject_set *roots, uint64_t n, keto_tree_node *nodes,
                      uint64_t cap, uint64_t *offsets, int32_t *err, std::string &msg) {
    Dispatcher *d = DP(hd);
    if (!d) throw Error(KETO_E_INVALID, "null dispatcher");
    if (!offsets) throw Error(KETO_E_INVALID, "null buffer");
    offsets[0] = 0;
    if (n == 0) return KETO_OK;
    if (!roots || !err) throw Error(KETO_E_INVALID, "null buffer");
    Request r;
    r.roots = roots;
    r.n = n;
    r.nodes = nodes;
    r.cap = cap;
    r.offsets = offsets;
    r.err = err;
    std::unique_lock<std::mutex> lk(d->m);
    if (d->stop) throw Error(KETO_E_INVALID, "dispatcher is shutting down");
    d->xqueue.push_back(&r);
    d->cv_in.notify_one();
    r.cv.wait(lk, [&] { return r.done; });
    msg = r.msg;
    return r.rc;
}

void dispatcher_stats(keto_dispatcher *hd, keto_dispatcher_stats *out) {
    Dispatcher *d = DP(hd);
    if (!d || !out) throw Error(KETO_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(d->m);
    *out = d->stats;
}

}  // namespace keto
