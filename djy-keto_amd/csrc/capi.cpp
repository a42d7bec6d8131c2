// extern "C" boundary (include/keto_mi355x.h): plain pointers and sizes, status codes,
// thread-local error text.  No CPU evaluation path exists behind it: every Check and
// Expand runs on the gfx950 kernels, and a missing/failed device is an error.
#include <cstring>
#include <memory>
#include <new>
#include <numeric>

#include "engine.hpp"

using keto::Error;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

template <class F>
int guarded(F &&f) {
    try {
        f();
        return KETO_OK;
    } catch (const Error &e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc &) {
        return fail(KETO_E_LIMIT, "host allocation failed");
    } catch (const std::exception &e) {
        return fail(KETO_E_INVALID, e.what());
    }
}

void grow(void *&p, size_t &cap, size_t need) {
    if (cap >= need) return;
    if (p) KETO_HIP(hipFree(p));
    p = nullptr;
    cap = 0;
    KETO_HIP(hipMalloc(&p, need));
    cap = need;
}

}  // namespace

namespace keto {
void Stream::flush_d2h() {
    if (!pend.on) return;
    pend.on = false;
    Slot &sl = slot[pend.slot];
    const char *o = static_cast<const char *>(pend.src);
    KETO_HIP(hipStreamWaitEvent(h2d, sl.out, 0));
    KETO_HIP(hipMemcpyAsync(pend.allowed, o, pend.n, hipMemcpyDeviceToHost, h2d));
    KETO_HIP(hipMemcpyAsync(pend.err, o + ((pend.n + 63) / 64) * 64, pend.n * sizeof(int32_t), hipMemcpyDeviceToHost, h2d));
    KETO_HIP(hipEventRecord(sl.free, h2d));
}

Stream::~Stream() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (check_scratch.mem) (void)hipFree(check_scratch.mem);
    if (expand_scratch.mem) (void)hipFree(expand_scratch.mem);
    if (frontier.mem) (void)hipFree(frontier.mem);
    if (frontier.stash) (void)hipFree(frontier.stash);
    if (frontier.host_ctrl) (void)hipHostFree(frontier.host_ctrl);
    if (frontier.host_gens) (void)hipHostFree(frontier.host_gens);
    if (frontier.gens_ev) (void)hipEventDestroy(frontier.gens_ev);
    if (frontier_block.mem) (void)hipFree(frontier_block.mem);
    if (frontier_block.fb_list) (void)hipFree(frontier_block.fb_list);
    if (frontier_block.host) (void)hipHostFree(frontier_block.host);
    if (xw.mem) (void)hipFree(xw.mem);
    if (xw.outbuf) (void)hipFree(xw.outbuf);
    if (xw.hpin) (void)hipHostFree(xw.hpin);
    for (hipEvent_t e : xw.ev)
        if (e) (void)hipEventDestroy(e);
    if (lists) (void)hipFree(lists);
    if (qbuf) (void)hipFree(qbuf);
    if (obuf) (void)hipFree(obuf);
    // every stream this object destroys first retires the scratch-cache events recorded on it
    // (scratch_forget_stream: a later scratch_get must never wait on a dead stream's event)
    for (hipStream_t c : {h2d, d2h})
        if (c) {
            (void)hipStreamSynchronize(c);
            scratch_forget_stream(c);
            (void)hipStreamDestroy(c);
        }
    for (Slot &sl : slot) {
        if (sl.q) (void)hipFree(sl.q);
        if (sl.o) (void)hipFree(sl.o);
        for (hipEvent_t e : {sl.in, sl.out, sl.free})
            if (e) (void)hipEventDestroy(e);
    }
    if (counters) (void)hipFree(counters);
    for (int i = 0; i < TIMER_SLOTS; i++) {
        if (ev_a[i]) (void)hipEventDestroy(ev_a[i]);
        if (ev_b[i]) (void)hipEventDestroy(ev_b[i]);
    }
    if (stream) {
        scratch_forget_stream(stream);
        (void)hipStreamDestroy(stream);
    }
}

void Stream::mark_begin() {
    if (timer_issued - timer_harvested == (uint64_t)TIMER_SLOTS) {  // ring full: wait for the oldest
        const int o = (int)(timer_harvested % TIMER_SLOTS);
        KETO_HIP(hipEventSynchronize(ev_b[o]));
        float ms = 0;
        if (hipEventElapsedTime(&ms, ev_a[o], ev_b[o]) == hipSuccess) {
            timer_ms_sum += ms;
            timer_count++;
            last_kernel_ms = ms;
        }
        timer_harvested++;
    }
    KETO_HIP(hipEventRecord(ev_a[timer_issued % TIMER_SLOTS], stream));
}

void Stream::mark_end() {
    KETO_HIP(hipEventRecord(ev_b[timer_issued % TIMER_SLOTS], stream));
    timer_issued++;
}

void Stream::harvest() {
    for (; timer_harvested < timer_issued; timer_harvested++) {
        const int o = (int)(timer_harvested % TIMER_SLOTS);
        float ms = 0;
        if (hipEventElapsedTime(&ms, ev_a[o], ev_b[o]) != hipSuccess) break;  // not complete yet
        timer_ms_sum += ms;
        timer_count++;
        last_kernel_ms = ms;
    }
}
}  // namespace keto

// the opaque ABI handles are the internal objects themselves
static keto::Snapshot *SN(keto_snapshot *p) { return reinterpret_cast<keto::Snapshot *>(p); }
static const keto::Snapshot *SN(const keto_snapshot *p) { return reinterpret_cast<const keto::Snapshot *>(p); }
// a snapshot whose in-place advance failed after its first write (Snapshot::broken)
static const char *BROKEN = "snapshot unusable: an in-place advance failed after its first write; cut a fresh one";
static keto::Stream *ST(keto_stream *p) { return reinterpret_cast<keto::Stream *>(p); }

extern "C" {

int keto_abi_version(void) { return KETO_ABI_VERSION; }

int keto_shutdown(void) {
    return guarded([&] { keto::pool_shutdown(); });
}

size_t keto_last_error(char *buf, size_t len) {
    if (buf && len) {
        size_t n = std::min(len - 1, g_err.size());
        std::memcpy(buf, g_err.data(), n);
        buf[n] = 0;
    }
    return g_err.size();
}

int keto_device_count(int32_t *out) {
    return guarded([&] {
        int n = 0;
        KETO_HIP(hipGetDeviceCount(&n));
        if (out) *out = n;
    });
}

int keto_snapshot_build(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, keto_snapshot **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    return guarded([&] {
        *out = reinterpret_cast<keto_snapshot *>(keto::build_snapshot(cfg, tuples, n, false));
    });
}

int keto_snapshot_build_device(const keto_snapshot_config *cfg, const keto_tuple *device_tuples, uint64_t n,
                               keto_snapshot **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    return guarded([&] {
        *out = reinterpret_cast<keto_snapshot *>(keto::build_snapshot(cfg, device_tuples, n, true));
    });
}

int keto_snapshot_save(const keto_snapshot *snap, const char *path) {
    if (!snap || !path) return fail(KETO_E_INVALID, "null argument");
    if (SN(snap)->broken) return fail(KETO_E_INVALID, BROKEN);
    return guarded([&] { keto::save_snapshot(*SN(snap), path); });
}

int keto_snapshot_load(const char *path, int32_t device, keto_snapshot **out) {
    if (!out || !path) return fail(KETO_E_INVALID, "null argument");
    *out = nullptr;
    return guarded([&] { *out = reinterpret_cast<keto_snapshot *>(keto::load_snapshot(path, device)); });
}

int keto_snapshot_free(keto_snapshot *snap) {
    delete SN(snap);
    return KETO_OK;
}

int keto_snapshot_info_get(const keto_snapshot *snap, keto_snapshot_info *out) {
    if (!snap || !out) return fail(KETO_E_INVALID, "null argument");
    *out = SN(snap)->info;
    return KETO_OK;
}

int keto_stream_create(int32_t device, keto_stream **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    return guarded([&] {
        KETO_HIP(hipSetDevice(device));
        auto s = std::make_unique<keto::Stream>();
        s->device = device;
        if (const char *be = getenv("KETO_FR_BUDGET")) s->fr_budget = (uint32_t)std::max(1, atoi(be));
        KETO_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        for (int i = 0; i < keto::Stream::TIMER_SLOTS; i++) {
            KETO_HIP(hipEventCreate(&s->ev_a[i]));
            KETO_HIP(hipEventCreate(&s->ev_b[i]));
        }
        KETO_HIP(hipMalloc(&s->counters, 24 * sizeof(unsigned long long)));
        KETO_HIP(hipMemsetAsync(s->counters, 0, 24 * sizeof(unsigned long long), s->stream));
        KETO_HIP(hipStreamSynchronize(s->stream));
        *out = reinterpret_cast<keto_stream *>(s.release());
    });
}

int keto_stream_destroy(keto_stream *s) {
    delete ST(s);
    return KETO_OK;
}

int keto_stream_sync(keto_stream *hs) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        s->flush_d2h();  // (an asynchronous batch's last copy)
        KETO_HIP(hipStreamSynchronize(s->stream));
        if (s->h2d) KETO_HIP(hipStreamSynchronize(s->h2d));
        if (s->d2h) KETO_HIP(hipStreamSynchronize(s->d2h));
        s->harvest();
    });
}

int keto_stream_kernel_time(keto_stream *hs, double *ms_sum, uint64_t *launches, int32_t reset) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        KETO_HIP(hipStreamSynchronize(s->stream));
        s->harvest();
        if (ms_sum) *ms_sum = s->timer_ms_sum;
        if (launches) *launches = s->timer_count;
        if (reset) {
            s->timer_ms_sum = 0;
            s->timer_count = 0;
        }
    });
}

int keto_stream_counters(keto_stream *hs, keto_work_counters *out, int32_t reset) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        unsigned long long c[24];
        KETO_HIP(hipMemcpyAsync(c, s->counters, sizeof c, hipMemcpyDeviceToHost, s->stream));
        KETO_HIP(hipStreamSynchronize(s->stream));
        if (out)
            for (int t = 0; t < 3; t++) {
                out->rows[t] = c[8 * t + 0];
                out->edges[t] = c[8 * t + 1];
                out->probes[t] = c[8 * t + 2];
                out->out_nodes[t] = c[8 * t + 3];
                out->queries[t] = c[8 * t + 4];
                out->wave_steps[t] = c[8 * t + 5];
                out->lane_steps[t] = c[8 * t + 6];
            }
        if (reset) {  // stream-ordered: later kernels on this (non-blocking) stream see the zeros
            KETO_HIP(hipMemsetAsync(s->counters, 0, sizeof c, s->stream));
            KETO_HIP(hipStreamSynchronize(s->stream));
        }
    });
}

int keto_stream_frontier_stats(keto_stream *hs, keto_frontier_stats *out, int32_t reset) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        if (out) *out = s->frontier.stats;
        if (reset) s->frontier.stats = keto_frontier_stats{};
    });
}

int keto_stream_expand_time(keto_stream *hs, double *ms_sum, uint64_t *batches, int32_t reset) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    if (ms_sum) *ms_sum = s->xw.ms_sum;
    if (batches) *batches = s->xw.batches;
    if (reset) {
        s->xw.ms_sum = 0;
        s->xw.batches = 0;
    }
    return KETO_OK;
}

int keto_stream_last_kernel_ms(keto_stream *hs, double *ms) {
    keto::Stream *s = ST(hs);
    if (!s || !ms) return fail(KETO_E_INVALID, "null argument");
    *ms = s->last_kernel_ms;
    return KETO_OK;
}

// keto_check_batch / keto_check_batch16: queries are `rec` bytes each (keto_query, keto_query16)
static int check_batch(keto_snapshot *hsnap, keto_stream *hs, const void *queries, size_t rec, uint64_t n,
                       const keto_limits *limits, uint8_t *out_allowed, int32_t *out_err, uint32_t flags) {
    keto::Snapshot *snap = SN(hsnap);
    keto::Stream *s = ST(hs);
    if (!snap || !s) return fail(KETO_E_INVALID, "null snapshot or stream");
    if (snap->broken) return fail(KETO_E_INVALID, BROKEN);
    if (n && (!queries || !out_allowed || !out_err)) return fail(KETO_E_INVALID, "null buffer");
    keto_limits lim = limits ? *limits : keto_limits{5, 100};
    if (lim.max_read_depth < 1 || lim.max_read_depth > 65535 || lim.max_read_width < 1 || lim.max_read_width > 65535)
        return fail(KETO_E_INVALID, "limits out of range (embedx/config.schema.json:368-383: 1..65535)");
    if (s->device != snap->device) return fail(KETO_E_INVALID, "stream and snapshot are on different devices");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        keto::CheckLaunch L{};
        L.n = n;
        L.max_depth = lim.max_read_depth;
        L.max_width = lim.max_read_width;
        L.count = (flags & KETO_F_COUNT_WORK) != 0;
        L.err_detail = (flags & KETO_F_ERR_DETAIL) != 0;
        L.budget = s->fr_budget;
        L.async = (flags & KETO_F_ASYNC) != 0 && !L.count;
        L.q16 = rec == sizeof(keto_query16);
        if (!(flags & KETO_F_ASYNC) || (flags & KETO_F_DEVICE_PTRS)) s->flush_d2h();  // (an earlier async batch's copy first)
        if (flags & KETO_F_DEVICE_PTRS) {
            L.queries = queries;
            L.out_allowed = out_allowed;
            L.out_err = out_err;
            keto::run_check(*snap, *s, L);
            if (!(flags & KETO_F_ASYNC)) {
                KETO_HIP(hipStreamSynchronize(s->stream));
                s->harvest();
            }
            return;
        }
        const size_t qb = n * rec, ob = n * (1 + sizeof(int32_t));
        if (flags & KETO_F_ASYNC) {
            // host buffers, enqueue only: slot b's H2D on the h2d stream (after the slot's previous
            // D2H), the kernels on the compute stream (after the H2D), the D2H on the d2h stream
            // (after the kernels).  Consecutive batches alternate slots, so the copies of one
            // overlap the kernels of its neighbours and the kernels never share the GPU.
            if (!s->h2d) {
                KETO_HIP(hipStreamCreateWithFlags(&s->h2d, hipStreamNonBlocking));
                KETO_HIP(hipStreamCreateWithFlags(&s->d2h, hipStreamNonBlocking));
                for (auto &sl : s->slot)
                    for (hipEvent_t *e : {&sl.in, &sl.out, &sl.free}) KETO_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
                const char *cs = getenv("KETO_COPY_STREAMS");
                s->one_copy = !(cs && cs[0] == '2');
            }
            const uint32_t si = (uint32_t)(s->slot_seq++ & 1);
            keto::Stream::Slot &sl = s->slot[si];
            if (sl.qb < qb || sl.ob < ob + 64) {  // (growing a slot: wait until its last batch is done)
                s->flush_d2h();
                KETO_HIP(hipStreamSynchronize(s->h2d));
                KETO_HIP(hipStreamSynchronize(s->d2h));
                grow(sl.q, sl.qb, std::max<size_t>(qb, 64));
                grow(sl.o, sl.ob, std::max<size_t>(ob + 64, 64));
            }
            auto *d_allowed = static_cast<uint8_t *>(sl.o);
            auto *d_err = reinterpret_cast<int32_t *>(static_cast<char *>(sl.o) + ((n + 63) / 64) * 64);
            KETO_HIP(hipStreamWaitEvent(s->h2d, sl.free, 0));
            KETO_HIP(hipMemcpyAsync(sl.q, queries, qb, hipMemcpyHostToDevice, s->h2d));
            KETO_HIP(hipEventRecord(sl.in, s->h2d));
            s->flush_d2h();  // (one copy stream: the previous batch's D2H behind this H2D)
            KETO_HIP(hipStreamWaitEvent(s->stream, sl.in, 0));
            L.queries = sl.q;
            L.out_allowed = d_allowed;
            L.out_err = d_err;
            keto::run_check(*snap, *s, L);
            KETO_HIP(hipEventRecord(sl.out, s->stream));
            if (s->one_copy) {  // enqueued by the next batch, or keto_stream_sync
                s->pend = keto::Stream::PendingD2H{true, out_allowed, out_err, sl.o, n, si};
                return;
            }
            KETO_HIP(hipStreamWaitEvent(s->d2h, sl.out, 0));
            KETO_HIP(hipMemcpyAsync(out_allowed, d_allowed, n, hipMemcpyDeviceToHost, s->d2h));
            KETO_HIP(hipMemcpyAsync(out_err, d_err, n * sizeof(int32_t), hipMemcpyDeviceToHost, s->d2h));
            KETO_HIP(hipEventRecord(sl.free, s->d2h));
            return;  // the caller synchronises the stream (keto_stream_sync)
        }
        // host buffers: stage through device memory owned by the stream
        grow(s->qbuf, s->qbuf_bytes, std::max<size_t>(qb, 64));
        grow(s->obuf, s->obuf_bytes, std::max<size_t>(ob + 64, 64));
        auto *d_allowed = static_cast<uint8_t *>(s->obuf);
        auto *d_err = reinterpret_cast<int32_t *>(static_cast<char *>(s->obuf) + ((n + 63) / 64) * 64);
        KETO_HIP(hipMemcpyAsync(s->qbuf, queries, qb, hipMemcpyHostToDevice, s->stream));
        L.queries = s->qbuf;
        L.out_allowed = d_allowed;
        L.out_err = d_err;
        keto::run_check(*snap, *s, L);
        KETO_HIP(hipMemcpyAsync(out_allowed, d_allowed, n, hipMemcpyDeviceToHost, s->stream));
        KETO_HIP(hipMemcpyAsync(out_err, d_err, n * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
        KETO_HIP(hipStreamSynchronize(s->stream));
        s->harvest();
    });
}

int keto_check_batch(keto_snapshot *hsnap, keto_stream *hs, const keto_query *queries, uint64_t n,
                     const keto_limits *limits, uint8_t *out_allowed, int32_t *out_err, uint32_t flags) {
    return check_batch(hsnap, hs, queries, sizeof(keto_query), n, limits, out_allowed, out_err, flags);
}

int keto_check_batch16(keto_snapshot *hsnap, keto_stream *hs, const keto_query16 *queries, uint64_t n,
                       const keto_limits *limits, uint8_t *out_allowed, int32_t *out_err, uint32_t flags) {
    return check_batch(hsnap, hs, queries, sizeof(keto_query16), n, limits, out_allowed, out_err, flags);
}

int keto_pack_query16(const keto_query *in, uint64_t n, keto_query16 *out) {
    if (n && (!in || !out)) return fail(KETO_E_INVALID, "null buffer");
    for (uint64_t i = 0; i < n; i++) {
        const keto_query &q = in[i];
        const bool set = q.subj_kind == 1;
        if (q.ns >= 4096 || q.rel >= 1024 || q.subj_kind > 1 || (set && (q.s_ns >= 4096 || q.s_rel >= 1024)) ||
            q.max_depth < -32768 || q.max_depth > 32767)
            return fail(KETO_E_LIMIT, "query " + std::to_string(i) + " does not fit the 16-byte record");
        // (a subject id's namespace and relation are never read: resolve_query.inc)
        out[i] = keto_query16{q.obj, q.s_obj, q.ns | (q.rel << 12) | ((set ? q.s_rel : 0u) << 22),
                              (set ? q.s_ns : 0u) | (q.subj_kind << 12) | ((uint32_t)(uint16_t)(int16_t)q.max_depth << 16)};
    }
    return KETO_OK;
}

int keto_expand_batch(keto_snapshot *hsnap, keto_stream *hs, const keto_subject_set *roots, uint64_t n,
                      const keto_limits *limits, keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_offsets,
                      int32_t *out_err) {
    keto::Snapshot *snap = SN(hsnap);
    keto::Stream *s = ST(hs);
    if (!snap || !s) return fail(KETO_E_INVALID, "null snapshot or stream");
    if (snap->broken) return fail(KETO_E_INVALID, BROKEN);
    if (n && (!roots || !out_offsets || !out_err)) return fail(KETO_E_INVALID, "null buffer");
    keto_limits lim = limits ? *limits : keto_limits{5, 100};
    if (lim.max_read_depth < 1 || lim.max_read_depth > 65535) return fail(KETO_E_INVALID, "max_read_depth out of range");
    if (s->device != snap->device) return fail(KETO_E_INVALID, "stream and snapshot are on different devices");
    int rc = KETO_OK;
    int g = guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        out_offsets[0] = 0;
        if (n == 0) return;
        grow(s->qbuf, s->qbuf_bytes, n * sizeof(keto_subject_set));
        auto *d_roots = static_cast<keto_subject_set *>(s->qbuf);
        KETO_HIP(hipMemcpyAsync(d_roots, roots, n * sizeof(keto_subject_set), hipMemcpyHostToDevice, s->stream));
        if (!keto::expand_batch(*snap, *s, d_roots, n, lim.max_read_depth, out_nodes, out_cap, out_offsets, out_err))
            rc = fail(KETO_E_CAPACITY, "expand output needs " + std::to_string(out_offsets[n]) + " nodes");
    });
    return g != KETO_OK ? g : rc;
}

int keto_expand_batch_spans(keto_snapshot *hsnap, keto_stream *hs, const keto_subject_set *roots, uint64_t n,
                            const keto_limits *limits, keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_first,
                            uint32_t *out_count, int32_t *out_err, uint64_t *out_total) {
    keto::Snapshot *snap = SN(hsnap);
    keto::Stream *s = ST(hs);
    if (!snap || !s) return fail(KETO_E_INVALID, "null snapshot or stream");
    if (snap->broken) return fail(KETO_E_INVALID, BROKEN);
    if (!out_total || (n && (!roots || !out_first || !out_count || !out_err))) return fail(KETO_E_INVALID, "null buffer");
    keto_limits lim = limits ? *limits : keto_limits{5, 100};
    if (lim.max_read_depth < 1 || lim.max_read_depth > 65535) return fail(KETO_E_INVALID, "max_read_depth out of range");
    if (s->device != snap->device) return fail(KETO_E_INVALID, "stream and snapshot are on different devices");
    int rc = KETO_OK;
    int g = guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        *out_total = 0;
        if (n == 0) return;
        grow(s->qbuf, s->qbuf_bytes, n * sizeof(keto_subject_set));
        auto *d_roots = static_cast<keto_subject_set *>(s->qbuf);
        KETO_HIP(hipMemcpyAsync(d_roots, roots, n * sizeof(keto_subject_set), hipMemcpyHostToDevice, s->stream));
        if (!keto::expand_batch_spans(*snap, *s, d_roots, n, lim.max_read_depth, out_nodes, out_cap, out_first, out_count, out_err,
                                      out_total))
            rc = fail(KETO_E_CAPACITY, "expand output needs " + std::to_string(*out_total) + " nodes");
    });
    return g != KETO_OK ? g : rc;
}

int keto_host_alloc(uint64_t bytes, void **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    return guarded([&] { KETO_HIP(hipHostMalloc(out, bytes ? bytes : 1, 0)); });
}

int keto_host_free(void *p) {
    return guarded([&] { KETO_HIP(hipHostFree(p)); });
}

int keto_device_alloc(int32_t device, uint64_t bytes, void **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    return guarded([&] {
        KETO_HIP(hipSetDevice(device));
        KETO_HIP(hipMalloc(out, bytes ? bytes : 1));
    });
}

int keto_device_free(void *p) {
    return guarded([&] { KETO_HIP(hipFree(p)); });
}

int keto_memcpy_h2d(keto_stream *hs, void *dst, const void *src, uint64_t bytes) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        KETO_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s->stream));
        KETO_HIP(hipStreamSynchronize(s->stream));
    });
}

int keto_memcpy_d2h(keto_stream *hs, void *dst, const void *src, uint64_t bytes) {
    keto::Stream *s = ST(hs);
    if (!s) return fail(KETO_E_INVALID, "null stream");
    return guarded([&] {
        KETO_HIP(hipSetDevice(s->device));
        KETO_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s->stream));
        KETO_HIP(hipStreamSynchronize(s->stream));
    });
}

}  // extern "C"

int keto_trees_to_json(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                       const keto_name_tables *names, char *out, uint64_t cap, uint64_t *out_offsets) {
    return guarded([&] { keto::trees_to_json(nodes, offsets, n_trees, names, out, cap, out_offsets); });
}

int keto_trees_to_proto(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                        const keto_name_tables *names, uint8_t *out, uint64_t cap, uint64_t *out_offsets) {
    return guarded([&] { keto::trees_to_proto(nodes, offsets, n_trees, names, out, cap, out_offsets); });
}

int keto_dispatcher_create(keto_snapshot *snap, const keto_dispatcher_config *cfg, keto_dispatcher **out) {
    if (out) *out = nullptr;
    if (snap && SN(snap)->broken) return fail(KETO_E_INVALID, BROKEN);
    return guarded([&] { keto::dispatcher_create(snap, cfg, out); });
}

int keto_dispatcher_destroy(keto_dispatcher *d) {
    return guarded([&] { keto::dispatcher_destroy(d); });
}

int keto_dispatcher_check(keto_dispatcher *d, const keto_query *queries, uint64_t n, uint8_t *out_allowed,
                          int32_t *out_err) {
    int rc = KETO_OK;
    const int g = guarded([&] {
        std::string msg;
        rc = keto::dispatcher_check(d, queries, n, out_allowed, out_err, msg);
        if (rc != KETO_OK) g_err = msg;
    });
    return g != KETO_OK ? g : rc;
}

int keto_dispatcher_expand(keto_dispatcher *d, const keto_subject_set *roots, uint64_t n, keto_tree_node *out_nodes,
                           uint64_t out_cap, uint64_t *out_offsets, int32_t *out_err) {
    int rc = KETO_OK;
    const int g = guarded([&] {
        std::string msg;
        rc = keto::dispatcher_expand(d, roots, n, out_nodes, out_cap, out_offsets, out_err, msg);
        if (rc != KETO_OK) g_err = msg;
    });
    return g != KETO_OK ? g : rc;
}

int keto_dispatcher_set_snapshot(keto_dispatcher *d, keto_snapshot *snap) {
    if (snap && SN(snap)->broken) return fail(KETO_E_INVALID, BROKEN);
    return guarded([&] { keto::dispatcher_set_snapshot(d, snap); });
}

int keto_dispatcher_stats_get(keto_dispatcher *d, keto_dispatcher_stats *out) {
    return guarded([&] { keto::dispatcher_stats(d, out); });
}

int keto_partition_create_placed(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, uint32_t flags,
                                 const keto_collective *coll, const keto_limits *limits, const keto_placement *placement,
                                 keto_partition **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    return guarded([&] {
        keto::Placement pl{};
        if (placement)
            for (uint32_t i = 0; i < keto::PLACE_NS; i++) pl.block[i] = placement->block[i];
        *out = reinterpret_cast<keto_partition *>(keto::partition_create(cfg, tuples, n, (flags & KETO_F_DEVICE_PTRS) != 0, coll,
                                                                         limits, (flags & KETO_F_PART_DIST) != 0, pl));
    });
}

int keto_partition_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, uint32_t flags,
                          const keto_collective *coll, const keto_limits *limits, keto_partition **out) {
    return keto_partition_create_placed(cfg, tuples, n, flags, coll, limits, nullptr, out);
}

int keto_partition_check(keto_partition *p, const keto_query *queries, uint64_t n, uint8_t *out_allowed,
                         int32_t *out_err, uint32_t flags) {
    if (!p) return fail(KETO_E_INVALID, "null partition");
    if (n && (!queries || !out_allowed || !out_err)) return fail(KETO_E_INVALID, "null buffer");
    return guarded([&] {
        keto::partition_check(reinterpret_cast<keto::PartitionHandle *>(p), queries, n, out_allowed, out_err, flags);
    });
}

int keto_partition_check_many(keto_partition *p, uint32_t n_batches, const keto_query *const *queries, const uint64_t *n,
                              uint8_t *const *out_allowed, int32_t *const *out_err, uint32_t flags) {
    if (!p) return fail(KETO_E_INVALID, "null partition");
    if (n_batches && (!queries || !n || !out_allowed || !out_err)) return fail(KETO_E_INVALID, "null buffer");
    for (uint32_t k = 0; k < n_batches; k++)
        if (n[k] && (!queries[k] || !out_allowed[k] || !out_err[k])) return fail(KETO_E_INVALID, "null buffer");
    return guarded([&] {
        keto::partition_check_many(reinterpret_cast<keto::PartitionHandle *>(p), n_batches, queries, n, out_allowed, out_err,
                                   flags);
    });
}

int keto_partition_expand(keto_partition *p, const keto_subject_set *roots, uint64_t n, uint64_t *out_nodes_needed) {
    if (!p || !out_nodes_needed) return fail(KETO_E_INVALID, "null argument");
    if (n && !roots) return fail(KETO_E_INVALID, "null roots");
    return guarded([&] { *out_nodes_needed = keto::partition_expand(reinterpret_cast<keto::PartitionHandle *>(p), roots, n); });
}

int keto_partition_expand_result(keto_partition *p, keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_offsets,
                                 int32_t *out_err) {
    if (!p) return fail(KETO_E_INVALID, "null partition");
    return guarded([&] {
        keto::partition_expand_result(reinterpret_cast<keto::PartitionHandle *>(p), out_nodes, out_cap, out_offsets, out_err);
    });
}

int keto_partition_stats_get(keto_partition *p, keto_partition_stats *out) {
    if (!p || !out) return fail(KETO_E_INVALID, "null argument");
    keto::partition_stats(reinterpret_cast<keto::PartitionHandle *>(p), out);
    return KETO_OK;
}

int keto_partition_generations_get(keto_partition *p, keto_partition_generation *out, uint32_t cap, uint32_t *n) {
    if (!p || !n || (cap && !out)) return fail(KETO_E_INVALID, "null argument");
    return guarded([&] { keto::partition_generations(reinterpret_cast<keto::PartitionHandle *>(p), out, cap, n); });
}

int keto_partition_levels_get(keto_partition *p, keto_partition_level *out, uint32_t cap, uint32_t *n) {
    if (!p || !n || (cap && !out)) return fail(KETO_E_INVALID, "null argument");
    return guarded([&] { keto::partition_levels(reinterpret_cast<keto::PartitionHandle *>(p), out, cap, n); });
}

int keto_partition_free(keto_partition *p) {
    return guarded([&] { keto::partition_free(reinterpret_cast<keto::PartitionHandle *>(p)); });
}

int keto_store_create(int32_t device, const keto_tuple *tuples, uint64_t n, uint32_t flags, keto_store **out) {
    if (!out) return fail(KETO_E_INVALID, "null output pointer");
    *out = nullptr;
    if (n && !tuples) return fail(KETO_E_INVALID, "null tuples");
    return guarded([&] {
        *out = reinterpret_cast<keto_store *>(keto::store_create(device, tuples, n, (flags & KETO_F_DEVICE_PTRS) != 0));
    });
}

int keto_store_transact(keto_store *st, const keto_tuple *ins, uint64_t n_ins, const keto_tuple *del, uint64_t n_del,
                        uint32_t flags) {
    if (!st) return fail(KETO_E_INVALID, "null store");
    if ((n_ins && !ins) || (n_del && !del)) return fail(KETO_E_INVALID, "null delta");
    return guarded([&] {
        keto::store_transact(*reinterpret_cast<keto::TupleStore *>(st), ins, n_ins, del, n_del,
                             (flags & KETO_F_DEVICE_PTRS) != 0);
    });
}

int keto_store_snapshot(keto_store *st, const keto_snapshot_config *cfg, keto_snapshot **out) {
    if (!st || !out) return fail(KETO_E_INVALID, "null argument");
    *out = nullptr;
    return guarded([&] {
        *out = reinterpret_cast<keto_snapshot *>(keto::store_snapshot(*reinterpret_cast<keto::TupleStore *>(st), cfg));
    });
}

int keto_store_snapshot_patch(keto_store *st, const keto_snapshot *base, const keto_snapshot_config *cfg,
                              keto_snapshot **out, int32_t *patched) {
    if (!st || !base || !out) return fail(KETO_E_INVALID, "null argument");
    *out = nullptr;
    if (SN(base)->broken) return fail(KETO_E_INVALID, BROKEN);
    return guarded([&] {
        bool p = false;
        *out = reinterpret_cast<keto_snapshot *>(
            keto::store_snapshot_patch(*reinterpret_cast<keto::TupleStore *>(st), *SN(base), cfg, &p));
        if (patched) *patched = p ? 1 : 0;
    });
}

int keto_store_snapshot_advance(keto_store *st, keto_snapshot *snap, int32_t *advanced) {
    if (!st || !snap) return fail(KETO_E_INVALID, "null argument");
    if (advanced) *advanced = 0;
    if (SN(snap)->broken) return fail(KETO_E_INVALID, BROKEN);
    return guarded([&] {
        const bool a = keto::store_snapshot_advance(*reinterpret_cast<keto::TupleStore *>(st), *SN(snap));
        if (advanced) *advanced = a ? 1 : 0;
    });
}

int keto_store_info(keto_store *st, uint64_t *n_tuples, uint64_t *version) {
    if (!st) return fail(KETO_E_INVALID, "null store");
    keto::store_info(*reinterpret_cast<keto::TupleStore *>(st), n_tuples, version);
    return KETO_OK;
}

int keto_store_free(keto_store *st) {
    keto::store_free(reinterpret_cast<keto::TupleStore *>(st));
    return KETO_OK;
}
