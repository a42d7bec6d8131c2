// Check over a graph partitioned by object across the ranks of a job (BASELINE config 5,
// SURVEY.md 8.1 (e)): every rank keeps its partition as a resident snapshot, built once, and the
// frontier engine (frontier.hip) runs over it with the goals that cross to another rank's
// objects exchanged once per generation -- no closure gather, no per-batch build.
//
// The partition.  keto_object_owner(ns, obj, world) owns every tuple of (ns, obj), so a goal on
// one of its nodes reads rows of that rank only: its set row (expand-subject, tuple-to-userset),
// its computed usersets and OR candidates (sibling slots of the same object), and the membership
// of the query subject in them (the reverse rows and probe hash of the tuples held there).
// Each rank's snapshot is the ordinary device build of its own tuples with three job-wide
// agreements, so node arithmetic and every spawn decision are the same on every rank:
//   * the relation slots (the (ns, rel) pairs some tuple of the job uses, OR over the ranks),
//   * the relation flags RI_SETROWS / RI_IDROWS (OR over the ranks),
//   * global uuid ids: a subject-set object held elsewhere is an ordinary entity here ("ghost":
//     its rows are empty) whose ent_obj is the object's global id.
// Subject-set edges into ghosts carry EDGE_REMOTE (build::remote_mark).
//
// A generation on every rank (frontier_goal.inc / frontier_kernels.inc, DIST instantiations):
//   * a child on a ghost node is the IA goal checkIsAllowed(child, depth, skip) of its owner --
//     it leaves as a 20-byte wire record {global obj, ns | rel << 16, word, scope, query home}
//     (WIRE_BYTES below: the outbox's 32-byte form without the query subject, which every rank
//     looks up by the record's home in the chunk's subject table, and without the sender's proxy
//     index, which the sender keeps in send order) and a G_PROXY goal keeps its place among its
//     parent's children;
//   * an expand-subject's found-lookahead on a ghost child (traverser.go:73-80: the EXISTS on the
//     child's own row) is run by the owner before anything else (GF_FOUND; past the width cut
//     GF_PROBE: the lookahead only);
//   * the records go to their owners in one all-to-all, where each becomes a goal of the next
//     generation at a position of its own (its start records resolved against that rank's rows,
//     resolve_query.inc).
// Bottom-up, after each generation's fr_reduce on every rank, the values of the goals that came
// from other ranks go back (4 bytes each by default -- membership, found bit, error code and
// relation name beside the subtree's saturated goal count; 8 with KETO_DIST_WIDE_VALUES=1 --
// in receive order) into their proxies, before the
// generation above is reduced; a query's root runs at its object's owner and its value goes back
// to its home, which decides.  So each goal's value is the one the single-snapshot engine
// computes over the whole graph: first decisive in add order (H0), AND / NOT, the depth ledger
// (engine.go:102-164, 214-249), the tuple-to-userset hop (rewrites.go:242-293).
//
// Visited-scope routing stays exact job-wide.  Scopes and keys are global: a scope is the goal
// that opened it (gscope: goal index and rank), a key UUIDv5(obj, ns+"-"+rel) as (global object,
// visited class) (gkey).  Occurrences stay where they were written; the decisive (scope, key)
// entries -- a few per thousand queries -- are gathered by every rank, each counts its own
// occurrences of them, the counts are summed, and a key seen twice routes its query at its home
// (graph_utils.go:38-53: H3).  Routed queries -- that, the goal budget, a full arena or outbox --
// are answered by the caller's exact path (partition.hip: the per-batch closure of those queries).
// Anything that could make a query look repeated without being so (a 32-bit key collision, the
// speculative children of an expand-subject whose lookahead then finds the subject) only routes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "device_common.hpp"
#include "frontier_dist.hpp"

namespace keto {
namespace {

#include "frontier_goal.inc"
#include "frontier_kernels.inc"
#include "resolve_query.inc"

constexpr uint32_t DBLK = 256;
// a goal record on the wire: {obj, ns | rel << 16, word, scope, home} -- the outbox's 32 bytes
// without the query subject (every rank holds the batch's subjects, exchanged once per chunk:
// subject = the table's entry for the record's home) and without the sender's proxy word (the
// sender keeps its proxies in send order, sent_px; values come back in receive order)
constexpr uint32_t WIRE_WORDS = 5, WIRE_BYTES = 4 * WIRE_WORDS;
constexpr uint32_t HOME_BITS = 21;  // home = rank << 21 | query index (batches of <= FR_MAX_BATCH)
constexpr uint32_t DIST_MAX_WORLD = 1u << (32 - HOME_BITS);

inline dim3 dgrid(uint64_t n, uint64_t cap = 1u << 16) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + DBLK - 1) / DBLK, cap)));
}
__device__ __forceinline__ uint64_t dgid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t dstride() { return (uint64_t)gridDim.x * blockDim.x; }
// a record's destination: its node's owner (keto_object_owner, or the job's keto_placement)
__device__ __forceinline__ uint32_t rec_owner(const uint4 &r0, const Dest &D) { return D.owner(r0.y & 0x7FFFu, r0.x); }

// ------------------------------------------------------------------------------ kernels

// the batch's queries as root records: checkIsAllowed(query, depth) at the object's owner; the
// depth clamp of engine.go:82-84 here, a depth past the goal word's field routes at home
__global__ __launch_bounds__(DBLK) void k_root_records(const keto_query *q, uint32_t n, int32_t max_depth, uint32_t rank,
                                                       uint4 *rec, uint32_t *deep) {
    for (uint64_t i = dgid(); i < n; i += dstride()) {
        const keto_query x = q[i];
        int32_t d0 = x.max_depth;
        if (d0 <= 0 || max_depth < d0) d0 = max_depth;
        const uint32_t d = (uint32_t)d0;
        if (d > GD_MAX) atomicOr(&deep[i >> 5], 1u << (i & 31u));
        rec[2 * i] = make_uint4(x.obj, dist_pack_ns_rel(x.ns, x.rel), x.s_obj,
                                std::min(x.s_ns, 0x7FFFu) | ((x.subj_kind & 1u) << 15) | (std::min(x.s_rel, 0xFFFFu) << 16));
        rec[2 * i + 1] = make_uint4(gword(G_IA, std::min(d, GD_MAX)), NONE32, (rank << HOME_BITS) | (uint32_t)i, (uint32_t)i);
    }
}

// the chunk's query subjects as the records carry them, for the job-wide subject table
__global__ __launch_bounds__(DBLK) void k_subjects(const uint4 *rec, uint32_t n, uint2 *out) {
    for (uint64_t i = dgid(); i < n; i += dstride()) {
        const uint4 r0 = rec[2 * i];
        out[i] = make_uint2(r0.z, r0.w);
    }
}

// records per destination rank (word 0: a null record, never sent); a block's counts in LDS
constexpr uint32_t LDS_W = 2048;  // DIST_MAX_WORLD
__global__ __launch_bounds__(DBLK) void k_dest_count(const uint4 *rec, uint32_t n, Dest D, uint32_t *hist) {
    __shared__ uint32_t h[LDS_W];
    const uint32_t world = D.world;
    for (uint32_t t = threadIdx.x; t < world; t += blockDim.x) h[t] = 0;
    __syncthreads();
    for (uint64_t i = dgid(); i < n; i += dstride())
        if (rec[2 * i + 1].x) atomicAdd(&h[rec_owner(rec[2 * i], D)], 1u);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < world; t += blockDim.x)
        if (h[t]) atomicAdd(&hist[t], h[t]);
}
// records grouped by destination (cursor[r] = r's first slot, advanced); the sender's proxy of
// each sent record, in send order, for the returns
__global__ __launch_bounds__(DBLK) void k_dest_scatter(const uint4 *rec, uint32_t n, Dest D, uint32_t *cursor,
                                                       uint32_t *out, uint32_t *sent_px) {
    __shared__ uint32_t h[LDS_W], base[LDS_W];
    const uint32_t world = D.world;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += dstride()) {
        for (uint32_t t = threadIdx.x; t < world; t += blockDim.x) h[t] = 0;
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        uint4 r0 = make_uint4(0, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
        uint32_t dst = 0, at = 0;
        const bool live = i < n && (r1 = rec[2 * i + 1]).x != 0;
        if (live) {
            r0 = rec[2 * i];
            dst = rec_owner(r0, D);
            at = atomicAdd(&h[dst], 1u);
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < world; t += blockDim.x)
            if (h[t]) base[t] = atomicAdd(&cursor[t], h[t]);
        __syncthreads();
        if (live) {
            const uint32_t p = base[dst] + at;
            uint32_t *o = out + (size_t)WIRE_WORDS * p;
            o[0] = r0.x;
            o[1] = r0.y;
            o[2] = r1.x;
            o[3] = r1.y;
            o[4] = r1.z;
            sent_px[p] = r1.w;
        }
        __syncthreads();
    }
}

// Arrival: each received record becomes a goal of generation `gen` at its own position pos0 + i
// (start records resolved against this rank's rows: the root node -- the object is this rank's,
// a phantom when it holds no tuple -- and the subject's membership record).  A block reserves its
// goals in one slice with one atomic; arrived[i] = the goal's arena index (NONE32: the slice was
// full, the position is routed and its return says so).
__global__ __launch_bounds__(DBLK) void k_arrive(FrontierParams P, const uint32_t *rec, uint32_t n, uint32_t pos0, uint32_t gen,
                                                 int32_t max_depth, uint4 *start, uint2 *subj, uint32_t *home, uint32_t *arrived,
                                                 const uint2 *stab, const uint32_t *stab_off) {
    const DevSnapshot &s = P.s;
    const Tables T = global_tables(s);
    __shared__ uint32_t s_base;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += dstride()) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(blockDim.x, n - i0);
        const uint32_t sl = (uint32_t)((i0 / blockDim.x) % FR_SHARDS);
        if (threadIdx.x == 0) s_base = atomicAdd(&P.gcount[sl * GEN_STRIDE + gen], cnt);
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        if (i < n) {
            const uint32_t *wr = rec + (size_t)WIRE_WORDS * i;
            const uint32_t hm = wr[4];
            const uint2 sj = stab[stab_off[hm >> HOME_BITS] + (hm & ((1u << HOME_BITS) - 1u))];  // (the query's subject)
            const uint4 r0 = make_uint4(wr[0], wr[1], sj.x, sj.y), r1 = make_uint4(wr[2], wr[3], hm, 0u);
            const uint32_t pos = pos0 + (uint32_t)i;
            uint4 a, R;
            uint32_t wgt = 0;
            resolve_query(s, T, r0.y & 0x7FFFu, r0.x, r0.y >> 16, (r0.w >> 15) & 1u, r0.z, r0.w & 0x7FFFu, r0.w >> 16,
                          (int32_t)(r1.x & GD_MAX), max_depth, pos, false, a, R, wgt);
            start[2 * (size_t)pos] = a;
            start[2 * (size_t)pos + 1] = R;
            subj[pos] = make_uint2(r0.z, r0.w);
            home[pos] = r1.z;
            P.qspawn[pos] = 0;
            // an IA record shaped here as its sender would have shaped a local sub-check (frontier_goal.inc
            // sub_check): a rewrite with neither a direct check nor an expand-subject to run is its RW
            // goal -- one generation less per remote hop (Drive's parents.traverse(view))
            uint32_t w = r1.x;
            if (((w >> 12) & 7u) == G_IA && !(w & (GF_FOUND | GF_PROBE | GF_ESCHILD | GF_ALIAS)) && (w & GD_MAX) >= 1) {
                const uint32_t sw = sub_check(s, T, subject_of(R), a.x, w & GD_MAX, (w & GF_SKIP) != 0, 0).word;
                if (sw && ((sw >> 12) & 7u) == G_RW) w = sw;
            }
            const uint32_t b = P.gbase[sl * GEN_STRIDE + gen], o = s_base + threadIdx.x;
            if ((uint64_t)b + o < P.scap) {
                const uint32_t idx = sl * P.scap + b + o;
                P.g0[idx] = make_uint4(a.x, pos, w, r1.y);
                arrived[i] = idx;
            } else {
                arrived[i] = NONE32;
                route(P, pos);
            }
        }
        __syncthreads();
    }
}

// a generation's goals on this rank (as fr_expand counts them: each slice clamped)
__global__ void k_gen_total(const uint32_t *gbase, const uint32_t *gcount, uint32_t scap, uint32_t gen, uint32_t *out) {
    if (blockIdx.x || threadIdx.x) return;
    uint32_t t = 0;
    for (uint32_t sl = 0; sl < FR_SHARDS; sl++) {
        const uint32_t b = gbase[sl * GEN_STRIDE + gen], c = gcount[sl * GEN_STRIDE + gen];
        t += std::min(c, scap - std::min(b, scap));
    }
    out[0] = t;
}

// Returns: the values of the goals that arrived at a generation, in receive order: {value, goals
// below | routed << 31}, 8 bytes -- or 4 when the job's values fit (`narrow`: relation name ids
// below 2^15 for the NO_RELATION detail, a goal budget below VAL_GOALS_SAT, which the goal count
// saturates at: any count past the budget routes alike)
constexpr uint32_t VAL_GOALS_SAT = 2047;
__device__ __forceinline__ uint32_t val_pack(uint32_t x, uint32_t y) {
    // membership 2 bits, FOUND_BIT, error code (<= 3) 2 bits, relation name 15 bits, goals 11 bits, routed
    return (x & 3u) | ((x >> 4) & 1u) << 2 | ((x >> 8) & 3u) << 3 | ((x >> 16) & 0x7FFFu) << 5 |
           std::min(y & 0x7FFFFFFFu, VAL_GOALS_SAT) << 20 | (y & (1u << 31));
}
__device__ __forceinline__ uint2 val_unpack(uint32_t p) {
    return make_uint2((p & 3u) | ((p >> 2) & 1u) << 4 | ((p >> 3) & 3u) << 8 | ((p >> 5) & 0x7FFFu) << 16,
                      ((p >> 20) & 0x7FFu) | (p & (1u << 31)));
}
__device__ __forceinline__ uint2 ret_read(const void *ret, uint64_t i, bool narrow) {
    return narrow ? val_unpack(static_cast<const uint32_t *>(ret)[i]) : static_cast<const uint2 *>(ret)[i];
}
__global__ __launch_bounds__(DBLK) void k_ret_gather(FrontierParams P, const uint32_t *arrived, uint32_t n, void *ret, bool narrow) {
    for (uint64_t i = dgid(); i < n; i += dstride()) {
        const uint32_t idx = arrived[i];
        uint2 r = make_uint2(M_UNK, 1u << 31);
        if (idx != NONE32) {
            const uint2 v = P.gvs[idx];
            const uint32_t pos = P.g0[idx].y;
            r = make_uint2(v.x, std::min(v.y, 0x7FFFFFFFu) | (routed(P, pos) ? 1u << 31 : 0u));
        }
        if (narrow) static_cast<uint32_t *>(ret)[i] = val_pack(r.x, r.y);
        else static_cast<uint2 *>(ret)[i] = r;
    }
}
// ... into the proxies that sent them (send order), before the generation above is reduced
__global__ __launch_bounds__(DBLK) void k_ret_apply(FrontierParams P, const uint32_t *sent_px, uint32_t n, const void *ret, bool narrow) {
    for (uint64_t i = dgid(); i < n; i += dstride()) {
        const uint32_t px = sent_px[i];
        const uint2 r = ret_read(ret, i, narrow);
        P.gvs[px] = make_uint2(r.x, r.y & 0x7FFFFFFFu);
        if (r.y >> 31) route(P, P.g0[px].y);
    }
}
// ... or, generation 0, to the queries' homes
__global__ __launch_bounds__(DBLK) void k_ret_home(const uint32_t *sent_px, uint32_t n, const void *ret, bool narrow, uint2 *hv) {
    for (uint64_t i = dgid(); i < n; i += dstride()) hv[sent_px[i]] = ret_read(ret, i, narrow);
}

// Job-wide repeats.  Every rank holds the job's decisive entries {scope, key, home}, grouped by
// source rank; the other ranks' go into this rank's table (dmerge), every local occurrence of a
// decisive key counts itself (dcount, fr_repeat without routing), the per-entry counts are
// gathered (dgather), summed over the ranks (dsum) and a key seen twice routes its query at home.
__global__ __launch_bounds__(DBLK) void k_dmerge(FrontierParams P, const uint4 *ent, uint32_t n, uint32_t skip_lo,
                                                 uint32_t skip_hi) {
    for (uint64_t e = dgid(); e < n; e += dstride()) {
        if (e >= skip_lo && e < skip_hi) continue;  // (this rank's own: inserted by fr_reduce)
        const unsigned long long key = tab_key(P.epoch, ent[e].x, ent[e].y);
        const uint32_t h = tab_hash(key, P.dmask);
        bool rep = false;
        const int64_t at = tab_insert(P.dkeys, P.dmask, P.epoch, key, h, atomicCAS(&P.dkeys[h], 0ull, key), &rep);
        if (at >= 0 && !rep) P.dcnt[at] = 0;
        const uint32_t b = dbit(key);
        atomicOr(&P.dbits[b >> 5], 1u << (b & 31u));
    }
}
__global__ __launch_bounds__(DBLK) void k_dcount(FrontierParams P) {
    for (uint32_t sl = 0; sl < FR_SHARDS; sl++) {
        const uint32_t cnt = std::min(P.occ_count[sl], P.ocap);
        for (uint64_t j = dgid(); j < cnt; j += dstride()) {
            const uint2 o = P.occ[(size_t)sl * P.ocap + j];
            if (o.x == NONE32) continue;
            const unsigned long long key = tab_key(P.epoch, o.x, o.y);
            const uint32_t b = dbit(key);
            if (!((P.dbits[b >> 5] >> (b & 31u)) & 1u)) continue;
            uint32_t h = tab_hash(key, P.dmask);
            for (int probe = 0; probe < TAB_PROBES; probe++) {
                const unsigned long long kk = P.dkeys[h];
                if (kk == key) {
                    atomicAdd(&P.dcnt[h], 1u);
                    break;
                }
                if (tab_free(kk, P.epoch)) break;
                h = (h + 1) & P.dmask;
            }
        }
    }
}
__global__ __launch_bounds__(DBLK) void k_dgather(FrontierParams P, const uint4 *ent, uint32_t n, uint32_t *cnt) {
    for (uint64_t e = dgid(); e < n; e += dstride()) {
        const unsigned long long key = tab_key(P.epoch, ent[e].x, ent[e].y);
        uint32_t h = tab_hash(key, P.dmask), c = 2;  // (not found: the table was crowded -- route)
        for (int probe = 0; probe < TAB_PROBES; probe++) {
            const unsigned long long kk = P.dkeys[h];
            if (kk == key) {
                c = P.dcnt[h];
                break;
            }
            if (tab_free(kk, P.epoch)) break;
            h = (h + 1) & P.dmask;
        }
        cnt[e] = c;
    }
}
__global__ __launch_bounds__(DBLK) void k_dsum(const uint4 *ent, uint32_t n, const uint32_t *cnt, uint32_t world, uint32_t rank,
                                               uint32_t *home_routed) {
    for (uint64_t e = dgid(); e < n; e += dstride()) {
        uint32_t t = 0;
        for (uint32_t r = 0; r < world; r++) t += cnt[(size_t)r * n + e];
        const uint32_t h = ent[e].z;
        if (t >= 2 && (h >> HOME_BITS) == rank) {
            const uint32_t q = h & ((1u << HOME_BITS) - 1u);
            atomicOr(&home_routed[q >> 5], 1u << (q & 31u));
        }
    }
}

// the home's decisions (fr_reduce's generation-0 step): routed -- by a rank on the way, by the
// job-wide repeat count, by the goal budget over the whole subtree, or too deep -- goes to the
// caller's exact path
__global__ __launch_bounds__(DBLK) void k_decide(const uint2 *hv, uint32_t n, const uint32_t *home_routed, const uint32_t *deep,
                                                 uint32_t budget, uint32_t err_detail, uint8_t *allowed, int32_t *err,
                                                 uint32_t *fb_list, uint32_t *fb_count) {
    for (uint64_t i = dgid(); i < n; i += dstride()) {
        const uint2 v = hv[i];
        const bool rt = (v.y >> 31) || ((home_routed[i >> 5] >> (i & 31u)) & 1u) || ((deep[i >> 5] >> (i & 31u)) & 1u) ||
                        1u + (v.y & 0x7FFFFFFFu) > budget;
        if (rt) {
            fb_list[atomicAdd(fb_count, 1u)] = (uint32_t)i;
            allowed[i] = 0;
            err[i] = 0;
            continue;
        }
        const uint32_t e = v.x >> 8;
        allowed[i] = (e == 0 && (v.x & 3u) == M_IS) ? 1 : 0;
        err[i] = (int32_t)(err_detail ? e : e & 0xFFu);
    }
}

// ------------------------------------------------------------------------------ host

// a device buffer that grows, keeping its first `keep` bytes
struct Grow {
    void *p = nullptr;
    size_t cap = 0;
    Grow() = default;
    Grow(const Grow &) = delete;
    Grow &operator=(const Grow &) = delete;
    ~Grow() {
        if (p) (void)hipFree(p);
    }
    void reserve(size_t bytes, size_t keep, hipStream_t s) {
        if (p && cap >= bytes) return;
        size_t c = std::max<size_t>({bytes, cap + cap / 2, 4096});
        void *q = nullptr;
        KETO_HIP(hipMalloc(&q, c + 16));
        if (p && keep) KETO_HIP(hipMemcpyAsync(q, p, std::min(keep, cap), hipMemcpyDeviceToDevice, s));
        KETO_HIP(hipStreamSynchronize(s));
        if (p) KETO_HIP(hipFree(p));
        p = q;
        cap = c;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
};

struct Level {  // one generation's exchange (records that arrive as goals of this generation)
    std::vector<uint64_t> sent, recv;  // records per destination / per source
    uint64_t sent_off = 0, recv_off = 0, n_sent = 0, n_recv = 0;
    bool any = false;                  // some rank sent records at this level
    keto_partition_level stat{};
};

}  // namespace

struct DistEngine {
    int device = 0;
    uint32_t rank = 0, world = 1;
    Placement place{};  // which objects each rank owns (keto_placement; zeros: the hash)
    keto_collective coll{};
    keto_limits limits{5, 100};
    std::unique_ptr<Snapshot> snap;
    hipStream_t hs = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    uint32_t budget = 1024, cus = 1, per_cu = 4;
    bool verbose = false;
    bool staged = false, agreed = false;
    // per batch (grown, reused)
    Grow dq, rec, sbuf, rbuf, sent_px, arrived, ret, rret, hv, deep, hrouted, outv, fbl, ssend, stab, stab_off;
    Grow arena, occ, dtab, dbits, ctrl, start, subj, home, qrouted, qspawn, ob, dlist, dent, dcnt, dsend;
    uint64_t cap = 0, ocap = 0, dcap = 0, pos_cap = 0, ob_cap = 0;
    uint32_t epoch = 1;
    uint64_t last_goals = 0, last_pos = 0, last_ob = 0;
    uint32_t *hpin = nullptr;  // pinned control read-backs
    std::vector<Level> levels;
    std::vector<keto_partition_level> level_acc;  // the last batch's generations, its chunks summed
    ~DistEngine() {
        if (hpin) (void)hipHostFree(hpin);
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
        if (hs) {
            scratch_forget_stream(hs);
            (void)hipStreamDestroy(hs);
        }
    }
};

namespace {

void dcoll_check(int rc, const char *what) {
    if (rc != 0) throw Error(KETO_E_DEVICE, std::string("collective ") + what + " failed with " + std::to_string(rc));
}

// every rank's u64 for this rank (send[r] goes to rank r)
std::vector<uint64_t> d_alltoall(DistEngine &E, const std::vector<uint64_t> &send, double &wait_s) {
    std::vector<uint64_t> recv(E.world, 0);
    const auto t0 = std::chrono::steady_clock::now();
    dcoll_check(E.coll.alltoall_u64(E.coll.ctx, send.data(), recv.data()), "alltoall_u64");
    wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return recv;
}
// all-to-all-v of device bytes on the engine's stream (RCCL device to device when the collective
// takes device buffers; else staged through host memory)
void d_alltoallv(DistEngine &E, const void *src, const std::vector<uint64_t> &sb, void *dst, const std::vector<uint64_t> &rb,
                 double &wait_s) {
    uint64_t ns = 0, nr = 0;
    for (uint32_t r = 0; r < E.world; r++) {
        ns += sb[r];
        nr += rb[r];
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (E.coll.alltoallv_device) {
        dcoll_check(E.coll.alltoallv_device(E.coll.ctx, src, sb.data(), dst, rb.data(), E.hs), "alltoallv_device");
    } else {
        std::vector<uint8_t> hsend(std::max<uint64_t>(1, ns)), hrecv(std::max<uint64_t>(1, nr));
        if (ns) KETO_HIP(hipMemcpyAsync(hsend.data(), src, ns, hipMemcpyDeviceToHost, E.hs));
        KETO_HIP(hipStreamSynchronize(E.hs));
        dcoll_check(E.coll.alltoallv(E.coll.ctx, hsend.data(), sb.data(), hrecv.data(), rb.data()), "alltoallv");
        if (nr) KETO_HIP(hipMemcpyAsync(dst, hrecv.data(), nr, hipMemcpyHostToDevice, E.hs));
        KETO_HIP(hipStreamSynchronize(E.hs));
    }
    wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
// host bytes: every rank's array OR-ed into `v` (all ranks pass equally long arrays)
void or_across(DistEngine &E, std::vector<uint8_t> &v) {
    if (E.world == 1 || v.empty()) return;
    const uint32_t W = E.world;
    std::vector<uint8_t> send((size_t)W * v.size()), recv((size_t)W * v.size());
    for (uint32_t r = 0; r < W; r++) std::memcpy(&send[(size_t)r * v.size()], v.data(), v.size());
    std::vector<uint64_t> b(W, v.size());
    dcoll_check(E.coll.alltoallv(E.coll.ctx, send.data(), b.data(), recv.data(), b.data()), "alltoallv");
    for (uint32_t r = 0; r < W; r++)
        for (size_t i = 0; i < v.size(); i++) v[i] |= recv[(size_t)r * v.size() + i];
}

// The relation flags of the whole graph: a flag only this rank's tuples would clear must not
// decide another rank's node here (collective).  Staged partitions first check that every rank
// laid out the same relation slots.
void agree_flags(DistEngine &D) {
    Snapshot &s = *D.snap;
    if (D.staged) {
        uint64_t h = 0xcbf29ce484222325ull;
        auto mix = [&](uint64_t x) {
            h ^= x;
            h *= 0x100000001b3ull;
        };
        for (uint32_t ns = 0; ns < s.n_ns; ns++) mix(s.ns[ns].n_slots);
        for (uint32_t r : s.slot_rel) mix(r);
        double w = 0;
        const std::vector<uint64_t> all = d_alltoall(D, std::vector<uint64_t>(D.world, h), w);
        for (uint64_t x : all)
            if (x != h)
                throw Error(KETO_E_INVALID, "staged partitions disagree on their relation slots: create them together "
                                            "(without KETO_PART_STAGED)");
    }
    std::vector<uint8_t> fl(s.relinfo.size());
    for (size_t g = 0; g < fl.size(); g++)
        fl[g] = (uint8_t)((ri_setrows(s.relinfo[g]) ? 1u : 0u) | (ri_idrows(s.relinfo[g]) ? 2u : 0u));
    or_across(D, fl);
    for (size_t g = 0; g < fl.size(); g++) {
        if (fl[g] & 1u) s.relinfo[g] |= RI_SETROWS;
        if (fl[g] & 2u) s.relinfo[g] |= RI_IDROWS;
    }
    if (!s.relinfo.empty())
        KETO_HIP(hipMemcpy(const_cast<uint32_t *>(s.dev.relinfo), s.relinfo.data(), 4 * s.relinfo.size(), hipMemcpyHostToDevice));
    D.agreed = true;
}
}  // namespace

DistEngine *dist_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, bool device_ptrs,
                        const keto_collective &coll, const keto_limits &limits, const Placement &place) {
    auto E = std::make_unique<DistEngine>();
    E->device = cfg->device;
    E->place = place;
    E->coll = coll;
    E->rank = (uint32_t)coll.rank;
    E->world = (uint32_t)coll.world;
    E->limits = limits;
    if (E->world > DIST_MAX_WORLD) throw Error(KETO_E_LIMIT, "the distributed frontier holds at most 2048 ranks");
    KETO_HIP(hipSetDevice(E->device));
    KETO_HIP(hipStreamCreateWithFlags(&E->hs, hipStreamNonBlocking));
    KETO_HIP(hipEventCreate(&E->ev[0]));
    KETO_HIP(hipEventCreate(&E->ev[1]));
    KETO_HIP(hipHostMalloc(reinterpret_cast<void **>(&E->hpin), 4096, 0));
    E->verbose = getenv("KETO_PART_VERBOSE") != nullptr;
    if (const char *be = getenv("KETO_FR_BUDGET")) E->budget = (uint32_t)std::max(1, atoi(be));
    E->cus = (uint32_t)std::max(1, num_cus(E->device));
    DistEngine &D = *E;
    BuildOpts o;
    o.no_leaf = true;
    o.no_weights = true;
    o.part_rank = E->rank;  // ghost namespaces for other ranks' subject sets
    o.part_world = E->world;
    o.place = E->place;
    // KETO_PART_STAGED (ranks that share one device and so create their partitions one after
    // another, tests/test_gpu_c5.py): no collective here -- each rank lays out the slots its own
    // tuples use, and the first batch checks that every rank's layout is the same (an error
    // otherwise: such partitions must be created together) and agrees on the relation flags
    E->staged = getenv("KETO_PART_STAGED") != nullptr;
    if (!E->staged) o.agree_used = [&D](std::vector<uint8_t> &used) { or_across(D, used); };
    E->snap.reset(build_snapshot(cfg, tuples, n, device_ptrs, false, &o));
    Snapshot &s = *E->snap;
    DevSnapshot &V = s.dev;
    if (V.n_nodes >= (1u << 30)) throw Error(KETO_E_LIMIT, "a partition's snapshot holds at most 2^30 nodes (EDGE_REMOTE)");
    if (!E->staged) agree_flags(D);
    // visited classes: slots whose ns+"-"+rel strings are equal share one (definitions.go:114-116)
    {
        std::vector<uint32_t> vc(std::max<size_t>(1, s.slot_rel.size()), 0);
        std::unordered_map<std::string, uint32_t> cls;
        for (uint32_t ns = 0; ns < s.n_ns; ns++)
            for (uint32_t k = 0; k < s.ns[ns].n_slots; k++) {
                const uint32_t g = s.ns[ns].slot_base + k;
                const std::string key = s.ns_names[ns] + "-" + s.rel_names[s.slot_rel[g]];
                auto it = cls.emplace(key, (uint32_t)cls.size()).first;
                vc[g] = it->second;
            }
        uint32_t *d = static_cast<uint32_t *>(s.alloc(4 * vc.size() + 16));
        KETO_HIP(hipMemcpy(d, vc.data(), 4 * vc.size(), hipMemcpyHostToDevice));
        V.vclass = d;
    }
    build::remote_mark(const_cast<uint32_t *>(V.set_dst), s.info.n_set_edges, const_cast<uint4 *>(V.set_row), V.n_owned, V.n_owned);
    V.edge_mask = ~(EDGE_ALIAS | EDGE_REMOTE);
    V.edge_leaf = 0;
    const bool lds_tables = V.lds_bytes <= LDS_TABLE_LIMIT;
    int per_cu = 0;
    const void *kx = lds_tables ? reinterpret_cast<const void *>(&fr_expand<true, true>) : reinterpret_cast<const void *>(&fr_expand<false, true>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kx, XBLOCK, lds_tables ? V.lds_bytes : 0) != hipSuccess || per_cu <= 0)
        per_cu = 4;
    E->per_cu = (uint32_t)std::min(per_cu, (int)(2048 / XBLOCK));
    if (E->verbose)
        fprintf(stderr, "[keto dist %u/%u] partition: %llu tuples, %llu nodes, %.2f GiB on the device, %.2f s\n", E->rank, E->world,
                (unsigned long long)n, (unsigned long long)V.n_nodes, s.info.device_bytes / 1073741824.0, s.info.build_seconds);
    return E.release();
}

void dist_free(DistEngine *E) { delete E; }
DistView dist_view(DistEngine &E) {
    if (!E.agreed) agree_flags(E);  // (collective: every dist_view caller is)
    return DistView{E.device, E.rank, E.world, &E.coll, E.hs, E.snap.get(), E.limits, E.place};
}
std::vector<uint64_t> dist_alltoall(const DistView &V, const std::vector<uint64_t> &send, double &wait_s) {
    std::vector<uint64_t> recv(V.world, 0);
    const auto t0 = std::chrono::steady_clock::now();
    dcoll_check(V.coll->alltoall_u64(V.coll->ctx, send.data(), recv.data()), "alltoall_u64");
    wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return recv;
}
void dist_alltoallv(const DistView &V, const void *src, const std::vector<uint64_t> &sb, void *dst,
                    const std::vector<uint64_t> &rb, double &wait_s) {
    uint64_t ns = 0, nr = 0;
    for (uint32_t r = 0; r < V.world; r++) {
        ns += sb[r];
        nr += rb[r];
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (V.coll->alltoallv_device) {
        dcoll_check(V.coll->alltoallv_device(V.coll->ctx, src, sb.data(), dst, rb.data(), V.hs), "alltoallv_device");
    } else {
        std::vector<uint8_t> hsend(std::max<uint64_t>(1, ns)), hrecv(std::max<uint64_t>(1, nr));
        if (ns) KETO_HIP(hipMemcpyAsync(hsend.data(), src, ns, hipMemcpyDeviceToHost, V.hs));
        KETO_HIP(hipStreamSynchronize(V.hs));
        dcoll_check(V.coll->alltoallv(V.coll->ctx, hsend.data(), sb.data(), hrecv.data(), rb.data()), "alltoallv");
        if (nr) KETO_HIP(hipMemcpyAsync(dst, hrecv.data(), nr, hipMemcpyHostToDevice, V.hs));
        KETO_HIP(hipStreamSynchronize(V.hs));
    }
    wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
const Snapshot &dist_snapshot(const DistEngine &E) { return *E.snap; }
std::vector<keto_partition_level> dist_levels(const DistEngine &E) {
    return E.level_acc;
}

namespace {
#ifndef KETO_FR_GOALS_PER_QUERY
#define KETO_FR_GOALS_PER_QUERY 64
#endif
constexpr size_t DCTRL_WORDS = 2 * FR_SHARDS * GEN_STRIDE + 16 + FR_SHARDS;  // gbase | gcount | misc | occ counts
enum Misc : uint32_t { M_ANY_ROUTED = 0, M_OB = 1, M_DLIST = 2, M_FB = 3, M_GEN = 4 };

void ensure_batch(DistEngine &E, uint64_t n) {
    static const uint64_t per_query = [] {
        const char *e = getenv("KETO_FR_GOALS_PER_QUERY");
        return e ? std::max<uint64_t>(1, strtoull(e, nullptr, 10)) : (uint64_t)KETO_FR_GOALS_PER_QUERY;
    }();
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>({n * per_query, E.last_goals + E.last_goals / 2, 1u << 20}), 1ull << 29) /
                          FR_SHARDS * FR_SHARDS;
    hipStream_t s = E.hs;
    if (want > E.cap) {
        E.cap = want;
        E.ocap = E.cap * 2 / FR_SHARDS;
        E.arena.reserve(E.cap * 32, 0, s);
        E.occ.reserve(E.ocap * FR_SHARDS * 8, 0, s);
    }
    uint64_t dcap = 1u << 16;
    while (dcap < 4 * std::max<uint64_t>(n, 1)) dcap <<= 1;
    if (dcap > E.dcap) {
        E.dcap = dcap;
        E.dtab.reserve(dcap * 12, 0, s);
        KETO_HIP(hipMemsetAsync(E.dtab.p, 0, dcap * 12, s));
        E.epoch = 1;
    }
    E.dbits.reserve((1u << DBITS_LOG2) / 8, 0, s);
    E.ctrl.reserve(DCTRL_WORDS * 4, 0, s);
    E.ob_cap = std::max<uint64_t>({E.ob_cap, 1u << 20, 4 * n, E.last_ob + E.last_ob / 2});
    E.ob.reserve(E.ob_cap * 32, 0, s);
    E.sbuf.reserve(std::max<uint64_t>(E.ob_cap, n) * 32, 0, s);
    E.dq.reserve(std::max<uint64_t>(1, n) * sizeof(keto_query), 0, s);
    E.rec.reserve(std::max<uint64_t>(1, n) * 32, 0, s);
    E.hv.reserve(std::max<uint64_t>(1, n) * 8, 0, s);
    const uint64_t bits = (std::max<uint64_t>(1, n) + 31) / 32 * 4;
    E.deep.reserve(bits, 0, s);
    E.hrouted.reserve(bits, 0, s);
    E.outv.reserve(std::max<uint64_t>(1, n) * 5 + 16, 0, s);
    E.fbl.reserve(std::max<uint64_t>(1, n) * 4, 0, s);
    const uint64_t dl = std::max<uint64_t>(1u << 16, n);
    E.dlist.reserve(dl * 16, 0, s);
}

// positions (the goals other ranks send, each with its start records) for `need` in all
void ensure_pos(DistEngine &E, uint64_t need, uint64_t used) {
    if (need <= E.pos_cap) return;
    uint64_t c = std::max<uint64_t>({need, E.pos_cap + E.pos_cap / 2, 1u << 20});
    c = (c + 31) / 32 * 32;
    hipStream_t s = E.hs;
    E.start.reserve(c * 32, used * 32, s);
    E.subj.reserve(c * 8, used * 8, s);
    E.home.reserve(c * 4, used * 4, s);
    E.qspawn.reserve(c * 4, used * 4, s);
    const size_t old_bits = E.qrouted.p ? E.pos_cap / 8 : 0;
    E.qrouted.reserve(c / 8 + 16, old_bits, s);
    KETO_HIP(hipMemsetAsync(static_cast<char *>(E.qrouted.p) + old_bits, 0, c / 8 + 16 - old_bits, s));
    E.pos_cap = c;
}

FrontierParams params(DistEngine &E) {
    FrontierParams P{};
    P.s = E.snap->dev;
    P.start = E.start.as<uint4>();
    P.n = (uint32_t)E.pos_cap;
    uint8_t *a = E.arena.as<uint8_t>();
    P.g0 = reinterpret_cast<uint4 *>(a);
    P.gfn = reinterpret_cast<uint2 *>(a + E.cap * 16);
    P.gvs = reinterpret_cast<uint2 *>(a + E.cap * 24);
    P.cap = (uint32_t)E.cap;
    P.scap = (uint32_t)(E.cap / FR_SHARDS);
    uint32_t *c = E.ctrl.as<uint32_t>();
    P.gbase = c;
    P.gcount = c + FR_SHARDS * GEN_STRIDE;
    uint32_t *misc = c + 2 * FR_SHARDS * GEN_STRIDE;
    P.any_routed = misc + M_ANY_ROUTED;
    P.ob_count = misc + M_OB;
    P.dlist_count = misc + M_DLIST;
    P.fb_count = misc + M_FB;
    P.occ_count = misc + 16;
    P.qrouted = E.qrouted.as<uint32_t>();
    P.qspawn = E.qspawn.as<uint32_t>();
    P.budget = E.budget;
    P.dkeys = E.dtab.as<unsigned long long>();
    P.dcnt = reinterpret_cast<uint32_t *>(P.dkeys + E.dcap);
    P.dbits = E.dbits.as<uint32_t>();
    P.dmask = (uint32_t)(E.dcap - 1);
    P.epoch = E.epoch;
    P.occ = E.occ.as<uint2>();
    P.ocap = (uint32_t)E.ocap;
    P.max_width = (uint32_t)E.limits.max_read_width;
    P.gen_cap = MAX_GEN;
    P.rank = E.rank;
    P.world = E.world;
    P.subj = E.subj.as<uint2>();
    P.home = E.home.as<uint32_t>();
    P.ob = E.ob.as<uint4>();
    P.ob_cap = (uint32_t)E.ob_cap;
    P.dlist = E.dlist.as<uint4>();
    P.dlist_cap = (uint32_t)std::max<uint64_t>(1u << 16, E.dlist.cap / 16);
    return P;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// `n` records in `src` (two uint4 each; word 0 = null) to their owners as level `L`: grouped by
// destination into sbuf (their proxies into sent_px), counts exchanged (with the termination
// flags), the records into rbuf.  Returns the records received.
uint64_t send_level(DistEngine &E, const uint4 *src, uint64_t n, Level &L, bool local_next, bool &any_local, bool &any_sent,
                    double &wait_s) {
    const uint32_t W = E.world;
    hipStream_t s = E.hs;
    E.dsend.reserve((size_t)W * 8 + 64, 0, s);
    uint32_t *h = E.dsend.as<uint32_t>();
    KETO_HIP(hipMemsetAsync(h, 0, (size_t)W * 4, s));
    if (n) hipLaunchKernelGGL(k_dest_count, dgrid(n, 4096), dim3(DBLK), 0, s, src, (uint32_t)n, Dest{W, E.rank, E.place}, h);
    KETO_HIP(hipGetLastError());
    std::vector<uint32_t> cnt(W);
    KETO_HIP(hipMemcpyAsync(cnt.data(), h, (size_t)W * 4, hipMemcpyDeviceToHost, s));
    KETO_HIP(hipStreamSynchronize(s));
    L.sent.assign(W, 0);
    uint64_t tot = 0;
    for (uint32_t r = 0; r < W; r++) {
        L.sent[r] = cnt[r];
        tot += cnt[r];
    }
    L.n_sent = tot;
    E.sent_px.reserve((L.sent_off + tot) * 4 + 16, L.sent_off * 4, s);
    if (tot) {
        std::vector<uint32_t> cur(W, 0);
        for (uint32_t r = 1; r < W; r++) cur[r] = cur[r - 1] + cnt[r - 1];
        KETO_HIP(hipMemcpyAsync(h, cur.data(), (size_t)W * 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_dest_scatter, dgrid(n, 4096), dim3(DBLK), 0, s, src, (uint32_t)n, Dest{W, E.rank, E.place}, h, E.sbuf.as<uint32_t>(),
                           E.sent_px.as<uint32_t>() + L.sent_off);
        KETO_HIP(hipGetLastError());
    }
    // counts, with the termination flags: bit 63 = this rank has goals of its own in the next
    // generation, bit 62 = it sends records
    std::vector<uint64_t> sendc(W);
    for (uint32_t r = 0; r < W; r++) sendc[r] = L.sent[r] | (local_next ? 1ull << 63 : 0ull) | (tot ? 1ull << 62 : 0ull);
    const std::vector<uint64_t> rc = d_alltoall(E, sendc, wait_s);
    L.recv.assign(W, 0);
    any_local = false;
    any_sent = false;
    uint64_t nr = 0;
    for (uint32_t r = 0; r < W; r++) {
        any_local |= (rc[r] >> 63) & 1u;
        any_sent |= (rc[r] >> 62) & 1u;
        L.recv[r] = rc[r] & ((1ull << 62) - 1);
        nr += L.recv[r];
    }
    L.n_recv = nr;
    L.any = any_sent;
    uint64_t bytes_out = 0;
    for (uint32_t r = 0; r < W; r++)
        if (r != E.rank) bytes_out += L.sent[r] * WIRE_BYTES;
    L.stat.request_bytes = bytes_out;
    L.stat.tuples = nr;
    if (any_sent) {
        std::vector<uint64_t> sb(W), rb(W);
        for (uint32_t r = 0; r < W; r++) {
            sb[r] = L.sent[r] * WIRE_BYTES;
            rb[r] = L.recv[r] * WIRE_BYTES;
        }
        E.rbuf.reserve(std::max<uint64_t>(1, nr) * WIRE_BYTES, 0, s);
        d_alltoallv(E, E.sbuf.p, sb, E.rbuf.p, rb, wait_s);
    }
    return nr;
}

}  // namespace

namespace {
void check_chunk(DistEngine &E, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, bool err_detail,
                 std::vector<uint32_t> &routed, DistStats &st) {
    ScratchStream on_hs(E.hs);
    const auto t_all = std::chrono::steady_clock::now();
    hipStream_t s = E.hs;
    const uint32_t W = E.world;
    double wait_s = 0, dev_ms = 0;
    ensure_batch(E, n);
    ensure_pos(E, std::max<uint64_t>(2 * n, E.last_pos + E.last_pos / 4), 0);
    KETO_HIP(hipMemsetAsync(E.ctrl.p, 0, DCTRL_WORDS * 4, s));
    KETO_HIP(hipMemsetAsync(E.dbits.p, 0, (1u << DBITS_LOG2) / 8, s));
    KETO_HIP(hipMemsetAsync(E.qrouted.p, 0, E.pos_cap / 8 + 16, s));
    const uint64_t bits = (std::max<uint64_t>(1, n) + 31) / 32 * 4;
    KETO_HIP(hipMemsetAsync(E.deep.p, 0, bits, s));
    KETO_HIP(hipMemsetAsync(E.hrouted.p, 0, bits, s));
    if (n) KETO_HIP(hipMemcpyAsync(E.dq.p, q, n * sizeof(keto_query), hipMemcpyHostToDevice, s));
    if (n)
        hipLaunchKernelGGL(k_root_records, dgrid(n), dim3(DBLK), 0, s, E.dq.as<keto_query>(), (uint32_t)n, E.limits.max_read_depth,
                           E.rank, E.rec.as<uint4>(), E.deep.as<uint32_t>());
    KETO_HIP(hipGetLastError());
    const bool lds_tables = E.snap->dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? E.snap->dev.lds_bytes : 0;
    const dim3 eg(E.cus * E.per_cu), xb(XBLOCK), eb(256);
    E.levels.clear();
    E.levels.reserve(GEN_STRIDE + 2);  // (references into it stay valid)
    E.levels.emplace_back();
    uint64_t npos = 0, total_goals = 0, sent_total = 0;
    // level 0: the queries' roots to their objects' owners
    bool any_local = false, any_sent = false;
    // the chunk's query subjects to every rank, once: the goal records carry only their home
    uint64_t subj_bytes = 0;
    {
        const std::vector<uint64_t> nq = d_alltoall(E, std::vector<uint64_t>(W, n), wait_s);
        std::vector<uint32_t> off(W + 1, 0);
        for (uint32_t r = 0; r < W; r++) off[r + 1] = off[r] + (uint32_t)nq[r];
        E.ssend.reserve(std::max<uint64_t>(1, n) * 8 * W + 16, 0, s);
        if (n) {
            hipLaunchKernelGGL(k_subjects, dgrid(n), dim3(DBLK), 0, s, E.rec.as<uint4>(), (uint32_t)n, E.ssend.as<uint2>());
            KETO_HIP(hipGetLastError());
            for (uint32_t r = 1; r < W; r++)
                KETO_HIP(hipMemcpyAsync(E.ssend.as<uint8_t>() + (size_t)r * n * 8, E.ssend.p, n * 8, hipMemcpyDeviceToDevice, s));
        }
        E.stab.reserve(std::max<uint64_t>(1, off[W]) * 8 + 16, 0, s);
        E.stab_off.reserve(4 * (W + 1) + 16, 0, s);
        KETO_HIP(hipMemcpyAsync(E.stab_off.p, off.data(), 4 * (W + 1), hipMemcpyHostToDevice, s));
        std::vector<uint64_t> sb(W, n * 8), rb(W);
        for (uint32_t r = 0; r < W; r++) rb[r] = nq[r] * 8;
        d_alltoallv(E, E.ssend.p, sb, E.stab.p, rb, wait_s);
        subj_bytes = n * 8 * (W - 1);
    }
    uint64_t nr = send_level(E, E.rec.as<uint4>(), n, E.levels[0], false, any_local, any_sent, wait_s);
    E.levels[0].stat.request_bytes += subj_bytes;  // (counted with the roots' records)
    sent_total += E.levels[0].n_sent;
    uint32_t G = 0;
    if (any_sent) {
        for (uint32_t k = 0;; k++) {
            Level &L = E.levels[k];
            const auto tg = std::chrono::steady_clock::now();
            KETO_HIP(hipEventRecord(E.ev[0], s));
            // this generation's arrivals (positions npos .. npos + nr)
            ensure_pos(E, npos + nr, npos);
            E.arrived.reserve((L.recv_off + nr) * 4 + 16, L.recv_off * 4, s);
            FrontierParams P = params(E);
            if (nr) {
                hipLaunchKernelGGL(k_arrive, dgrid(nr, 8192), dim3(DBLK), 0, s, P, E.rbuf.as<uint32_t>(), (uint32_t)nr, (uint32_t)npos, k,
                                   E.limits.max_read_depth, E.start.as<uint4>(), E.subj.as<uint2>(), E.home.as<uint32_t>(),
                                   E.arrived.as<uint32_t>() + L.recv_off, E.stab.as<uint2>(), E.stab_off.as<uint32_t>());
                KETO_HIP(hipGetLastError());
            }
            npos += nr;
            // the generation
            P.gen = k;
            if (lds_tables) hipLaunchKernelGGL((fr_expand<true, true>), eg, xb, lds, s, P);
            else hipLaunchKernelGGL((fr_expand<false, true>), eg, xb, 0, s, P);
            KETO_HIP(hipGetLastError());
            uint32_t *misc = E.ctrl.as<uint32_t>() + 2 * FR_SHARDS * GEN_STRIDE;
            hipLaunchKernelGGL(k_gen_total, dim3(1), dim3(1), 0, s, P.gbase, P.gcount, P.scap, k, misc + M_GEN);
            hipLaunchKernelGGL(k_gen_total, dim3(1), dim3(1), 0, s, P.gbase, P.gcount, P.scap, k + 1, misc + M_GEN + 1);
            KETO_HIP(hipMemcpyAsync(E.hpin, misc, 8 * 4, hipMemcpyDeviceToHost, s));
            KETO_HIP(hipEventRecord(E.ev[1], s));
            KETO_HIP(hipStreamSynchronize(s));
            float ms = 0;
            KETO_HIP(hipEventElapsedTime(&ms, E.ev[0], E.ev[1]));
            const uint32_t gk = E.hpin[M_GEN], gnext = E.hpin[M_GEN + 1];
            const uint64_t nob = std::min<uint64_t>(E.hpin[M_OB], E.ob_cap);
            E.last_ob = std::max<uint64_t>(E.last_ob, E.hpin[M_OB]);
            KETO_HIP(hipMemsetAsync(misc + M_OB, 0, 4, s));
            total_goals += gk;
            L.stat.objects = gk;
            // the records of this generation's remote children: level k + 1
            E.levels.emplace_back();
            Level &N = E.levels[k + 1];
            N.sent_off = L.sent_off + L.n_sent;
            N.recv_off = L.recv_off + L.n_recv;
            nr = send_level(E, E.ob.as<uint4>(), nob, N, gnext > 0, any_local, any_sent, wait_s);
            sent_total += N.n_sent;
            dev_ms += ms;
            L.stat.ms = ms;
            if (E.verbose)
                fprintf(stderr, "[keto dist %u] gen %u: %u goals (%llu arrived), %llu records out, %.3f ms device, %.3f ms wall\n",
                        E.rank, k, gk, (unsigned long long)L.n_recv, (unsigned long long)N.n_sent, ms, ms_since(tg));
            if (!any_local && !any_sent) {
                G = k + 1;
                E.levels.pop_back();
                break;
            }
            if (k + 2 >= GEN_STRIDE) throw Error(KETO_E_LIMIT, "distributed frontier: generation cap");
        }
    }
    // bottom-up: each generation reduced on every rank, then the values of the goals other ranks
    // sent back to their proxies (generation 0: to the homes) -- 4 bytes each when they fit
    // (KETO_DIST_WIDE_VALUES=1: always 8, A/B)
    static const bool wide_env = getenv("KETO_DIST_WIDE_VALUES") != nullptr;
    const bool narrow = !wide_env && std::max(E.snap->n_rel, E.snap->n_rel_caller) <= 0x8000u && E.budget < VAL_GOALS_SAT;
    const uint64_t vbytes = narrow ? 4 : 8;
    E.hv.reserve(std::max<uint64_t>(1, n) * 8, 0, s);
    KETO_HIP(hipMemsetAsync(E.hv.p, 0, std::max<uint64_t>(1, n) * 8, s));
    for (int32_t j = (int32_t)G - 1; j >= 0; j--) {
        Level &L = E.levels[j];
        FrontierParams P = params(E);
        P.gen = (uint32_t)j;
        KETO_HIP(hipEventRecord(E.ev[0], s));
        hipLaunchKernelGGL(fr_reduce<true>, dim3(E.cus * 8), eb, 0, s, P);
        KETO_HIP(hipGetLastError());
        if (L.n_recv) {
            E.ret.reserve(L.n_recv * 8, 0, s);
            hipLaunchKernelGGL(k_ret_gather, dgrid(L.n_recv), dim3(DBLK), 0, s, P, E.arrived.as<uint32_t>() + L.recv_off,
                               (uint32_t)L.n_recv, E.ret.p, narrow);
            KETO_HIP(hipGetLastError());
        }
        KETO_HIP(hipEventRecord(E.ev[1], s));
        if (L.any) {
            std::vector<uint64_t> sb(W), rb(W);
            uint64_t back = 0;
            for (uint32_t r = 0; r < W; r++) {
                sb[r] = L.recv[r] * vbytes;
                rb[r] = L.sent[r] * vbytes;
                if (r != E.rank) back += sb[r];
            }
            L.stat.tuple_bytes_sent = back;
            E.rret.reserve(std::max<uint64_t>(1, L.n_sent) * 8, 0, s);
            d_alltoallv(E, E.ret.p, sb, E.rret.p, rb, wait_s);
            if (L.n_sent) {
                if (j > 0)
                    hipLaunchKernelGGL(k_ret_apply, dgrid(L.n_sent), dim3(DBLK), 0, s, P, E.sent_px.as<uint32_t>() + L.sent_off,
                                       (uint32_t)L.n_sent, (const void *)E.rret.p, narrow);
                else
                    hipLaunchKernelGGL(k_ret_home, dgrid(L.n_sent), dim3(DBLK), 0, s, E.sent_px.as<uint32_t>() + L.sent_off,
                                       (uint32_t)L.n_sent, (const void *)E.rret.p, narrow, E.hv.as<uint2>());
                KETO_HIP(hipGetLastError());
            }
        }
        KETO_HIP(hipStreamSynchronize(s));
        float ms = 0;
        KETO_HIP(hipEventElapsedTime(&ms, E.ev[0], E.ev[1]));
        dev_ms += ms;
        L.stat.ms += ms;
    }
    // the job-wide repeat count of the decisive (scope, key) entries
    FrontierParams P = params(E);
    {
        uint32_t *misc = E.ctrl.as<uint32_t>() + 2 * FR_SHARDS * GEN_STRIDE;
        KETO_HIP(hipMemcpyAsync(E.hpin, misc, 8 * 4, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipStreamSynchronize(s));
        const uint64_t nd = std::min<uint64_t>(E.hpin[M_DLIST], P.dlist_cap);
        const std::vector<uint64_t> dc = d_alltoall(E, std::vector<uint64_t>(W, nd), wait_s);
        uint64_t ne = 0, mine_lo = 0;
        for (uint32_t r = 0; r < W; r++) {
            if (r == E.rank) mine_lo = ne;
            ne += dc[r];
        }
        if (ne) {
            E.dsend.reserve(std::max<uint64_t>((uint64_t)W * nd * 16, (uint64_t)W * ne * 4) + 64, 0, s);
            E.dent.reserve(ne * 16, 0, s);
            for (uint32_t r = 0; r < W; r++)
                if (nd) KETO_HIP(hipMemcpyAsync(E.dsend.as<uint8_t>() + (size_t)r * nd * 16, E.dlist.p, nd * 16, hipMemcpyDeviceToDevice, s));
            std::vector<uint64_t> sb(W, nd * 16), rb(W);
            for (uint32_t r = 0; r < W; r++) rb[r] = dc[r] * 16;
            d_alltoallv(E, E.dsend.p, sb, E.dent.p, rb, wait_s);
            hipLaunchKernelGGL(k_dmerge, dgrid(ne), dim3(DBLK), 0, s, P, E.dent.as<uint4>(), (uint32_t)ne, (uint32_t)mine_lo,
                               (uint32_t)(mine_lo + nd));
            hipLaunchKernelGGL(k_dcount, dim3(E.cus * 4), dim3(DBLK), 0, s, P);
            E.dcnt.reserve(ne * 4 * (W + 1), 0, s);
            uint32_t *mine = E.dcnt.as<uint32_t>() + (size_t)W * ne;
            hipLaunchKernelGGL(k_dgather, dgrid(ne), dim3(DBLK), 0, s, P, E.dent.as<uint4>(), (uint32_t)ne, mine);
            KETO_HIP(hipGetLastError());
            for (uint32_t r = 0; r < W; r++)
                KETO_HIP(hipMemcpyAsync(E.dsend.as<uint8_t>() + (size_t)r * ne * 4, mine, ne * 4, hipMemcpyDeviceToDevice, s));
            std::vector<uint64_t> cb(W, ne * 4);
            d_alltoallv(E, E.dsend.p, cb, E.dcnt.p, cb, wait_s);
            hipLaunchKernelGGL(k_dsum, dgrid(ne), dim3(DBLK), 0, s, E.dent.as<uint4>(), (uint32_t)ne, E.dcnt.as<uint32_t>(), W, E.rank,
                               E.hrouted.as<uint32_t>());
            KETO_HIP(hipGetLastError());
        }
        st.decisive = ne;
    }
    // the homes decide
    uint8_t *d_allowed = E.outv.as<uint8_t>();
    int32_t *d_err = reinterpret_cast<int32_t *>(E.outv.as<uint8_t>() + (std::max<uint64_t>(1, n) + 15) / 16 * 16);
    uint32_t *misc = E.ctrl.as<uint32_t>() + 2 * FR_SHARDS * GEN_STRIDE;
    if (n)
        hipLaunchKernelGGL(k_decide, dgrid(n), dim3(DBLK), 0, s, E.hv.as<uint2>(), (uint32_t)n, E.hrouted.as<uint32_t>(),
                           E.deep.as<uint32_t>(), E.budget, err_detail ? 1u : 0u, d_allowed, d_err, E.fbl.as<uint32_t>(), misc + M_FB);
    KETO_HIP(hipGetLastError());
    if (n) {
        KETO_HIP(hipMemcpyAsync(allowed, d_allowed, n, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipMemcpyAsync(err, d_err, n * 4, hipMemcpyDeviceToHost, s));
    }
    KETO_HIP(hipMemcpyAsync(E.hpin, misc, 8 * 4, hipMemcpyDeviceToHost, s));
    KETO_HIP(hipStreamSynchronize(s));
    const uint32_t nfb = E.hpin[M_FB];
    routed.resize(nfb);
    if (nfb) KETO_HIP(hipMemcpy(routed.data(), E.fbl.p, nfb * 4, hipMemcpyDeviceToHost));
    std::sort(routed.begin(), routed.end());
    if (++E.epoch > TAB_EPOCHS) {
        KETO_HIP(hipMemsetAsync(E.dtab.p, 0, E.dcap * 12, s));
        E.epoch = 1;
    }
    E.last_goals = total_goals;
    E.last_pos = npos;
    st.generations = G;
    st.goals = total_goals;
    st.positions = npos;
    st.routed = nfb;
    st.records_sent = sent_total;
    uint64_t bytes = 0;
    for (auto &L : E.levels) bytes += L.stat.request_bytes + L.stat.tuple_bytes_sent;
    st.bytes_exchanged = bytes;
    st.device_s = dev_ms / 1e3;
    st.exchange_s = wait_s;
    st.wall_s = ms_since(t_all) / 1e3;
    if (E.verbose)
        fprintf(stderr,
                "[keto dist %u] batch of %llu: %u generations, %llu goals, %llu records sent, %.1f MB exchanged, %u routed, "
                "%llu decisive; device %.2f ms, collective %.2f ms, wall %.2f ms\n",
                E.rank, (unsigned long long)n, G, (unsigned long long)total_goals, (unsigned long long)sent_total, bytes / 1e6, nfb,
                (unsigned long long)st.decisive, dev_ms, wait_s * 1e3, st.wall_s * 1e3);
}
}  // namespace

// A batch runs in chunks of at most KETO_PART_CHUNK queries (default: one chunk of up to 2^21):
// the arena, the positions and the per-generation exchange buffers scale with a chunk, which
// bounds a rank's memory beside its resident partition (ranks that share a device).  Every rank
// runs the job-wide chunk count -- the largest batch's -- so the collectives stay in step; a rank
// whose batch ran out takes part with empty chunks.
void dist_check(DistEngine &E, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, bool err_detail,
                std::vector<uint32_t> &routed, DistStats &st) {
    KETO_HIP(hipSetDevice(E.device));
    if (!E.agreed) agree_flags(E);
    if (n > FR_MAX_BATCH) throw Error(KETO_E_LIMIT, "a partitioned batch holds at most 2^21 queries");
    static const uint64_t chunk = [] {
        const char *e = getenv("KETO_PART_CHUNK");
        const uint64_t c = e ? strtoull(e, nullptr, 10) : 0;
        return c ? std::min<uint64_t>(c, FR_MAX_BATCH) : (uint64_t)FR_MAX_BATCH;
    }();
    const auto t_all = std::chrono::steady_clock::now();
    double wait_s = 0;
    uint64_t chunks = (n + chunk - 1) / chunk;
    if (chunk < FR_MAX_BATCH)
        for (uint64_t c : d_alltoall(E, std::vector<uint64_t>(E.world, chunks), wait_s)) chunks = std::max(chunks, c);
    chunks = std::max<uint64_t>(chunks, 1);
    st = DistStats{};
    st.exchange_s = wait_s;
    routed.clear();
    std::vector<keto_partition_level> acc;
    for (uint64_t c = 0; c < chunks; c++) {
        const uint64_t b = std::min(n, c * chunk), m = std::min(n, b + chunk) - b;
        std::vector<uint32_t> r;
        DistStats cs;
        check_chunk(E, q + b, m, allowed + b, err + b, err_detail, r, cs);
        for (uint32_t i : r) routed.push_back((uint32_t)(b + i));
        st.generations = std::max(st.generations, cs.generations);
        st.goals += cs.goals;
        st.positions += cs.positions;
        st.routed += cs.routed;
        st.records_sent += cs.records_sent;
        st.bytes_exchanged += cs.bytes_exchanged;
        st.decisive += cs.decisive;
        st.device_s += cs.device_s;
        st.exchange_s += cs.exchange_s;
        for (size_t g = 0; g < E.levels.size(); g++) {
            if (acc.size() <= g) acc.push_back(keto_partition_level{});
            const keto_partition_level &l = E.levels[g].stat;
            acc[g].objects += l.objects;
            acc[g].request_bytes += l.request_bytes;
            acc[g].tuples += l.tuples;
            acc[g].tuple_bytes_sent += l.tuple_bytes_sent;
            acc[g].ms += l.ms;
        }
    }
    E.level_acc = std::move(acc);
    st.wall_s = ms_since(t_all) / 1e3;
}

}  // namespace keto
