// Incremental snapshots (keto_store_snapshot_patch): the store's
// content after some transactions, cut by patching the snapshot of an earlier version instead of
// building it again.
//
// The reference's write path touches single rows (persistence/sql/relationtuples.go:104-126
// WriteRelationTuples, :168-189 DeleteRelationTuples, :277-287 TransactRelationTuples); a read
// after it sees exactly the new rows.  Here the touched tuples (every insert and delete since the
// base version, kept by the store) name the rows that can differ:
//   - the rows of their objects' nodes (set rows for expand-subject / tuple-to-userset, all-rows
//     for Expand) and the reverse rows of their subjects (checkDirect, the found-lookahead, the
//     OR shortcut's IN);
//   - those rows are rebuilt from the store's current content -- one streaming pass over the
//     store finds their tuples (a small hash of the touched keys, a bit filter in LDS first) --
//     in shard order (traverser.go:88, relationtuples.go:216), ties by store position as the
//     full build breaks them;
//   - every other row keeps its content: the CSR arrays are copied with each row shifted by the
//     size change of the touched rows before it (one bandwidth-bound pass per array);
//   - the probe hash gets the heavy subjects' new (subject, node) keys and tombstones for the
//     keys that went away (member() walks past a tombstone: it is neither empty nor the key);
//   - the EDGE_LEAF flags of edges into nodes whose set row became empty / non-empty are fixed
//     through the new reverse rows, RI_SETROWS is recounted, RI_IDROWS only grows;
//   - node space, entities, visited keys, scheduling weights and the rewrite program are
//     shared with the base snapshot (same allocations).
// A touched tuple whose object, subject set or relation slot has no node in the base (a new
// object, a new (namespace, relation) pair, a uuid past n_uuids) cannot be placed: the caller
// builds in full.  The base stays untouched (a batch may still be running on it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <memory>
#include <unordered_map>
#include <vector>

#include "device_common.hpp"

namespace keto {
namespace {

constexpr uint32_t BLK = 256;
constexpr uint32_t ITEMS = 16;  // elements per thread of the copy passes
inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, (n + BLK - 1) / BLK)); }
inline dim3 grid_items(uint64_t n) {
    return dim3((uint32_t)std::max<uint64_t>(1, (n + (uint64_t)BLK * ITEMS - 1) / ((uint64_t)BLK * ITEMS)));
}
__device__ __forceinline__ uint64_t gid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
constexpr unsigned long long PROBE_TOMB = ~0ull;  // a removed probe key (never a key: subject < 2^32 - 2)

// ---- keys of the store scan ------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t key4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return mix64(((uint64_t)a << 32 | b) ^ mix64((uint64_t)c << 32 | d) ^ 0x51ED27u);
}
// a row's key (ns, obj, rel) and a subject's (kind, id, ns, rel) -- a subject id matches on
// its id alone, as the delete does (persistence/sql/relationtuples.go:128-150)
__host__ __device__ __forceinline__ void row_key(const keto_tuple &t, uint4 &k) { k = make_uint4(t.ns, t.obj, t.rel, 0xFFFFFFFFu); }
__host__ __device__ __forceinline__ void subj_key(const keto_tuple &t, uint4 &k) {
    k = t.subj_kind == 1 ? make_uint4(1u, t.s_obj, t.s_ns, t.s_rel) : make_uint4(0u, t.s_obj, 0u, 0u);
}
struct KeyTab {  // open addressing over power-of-two slots {key, value}; value NONE32 = empty
    const uint4 *key;
    const uint32_t *val;
    uint32_t mask;
};
__device__ __forceinline__ uint32_t tab_find(const KeyTab &T, const uint4 &k, uint64_t h) {
    for (uint32_t b = (uint32_t)h & T.mask;; b = (b + 1) & T.mask) {
        const uint32_t v = T.val[b];
        if (v == NONE32) return NONE32;
        const uint4 x = T.key[b];
        if (x.x == k.x && x.y == k.y && x.z == k.z && x.w == k.w) return v;
    }
}

// ---- node / subject index of raw ids in the base snapshot --------------------------------------
__device__ __forceinline__ uint32_t node_in(const DevSnapshot &s, uint32_t ns, uint32_t obj, uint32_t rel) {
    if (ns >= s.n_ns || rel >= s.n_rel) return NONE32;
    const uint32_t e = ent_lookup(s, ns, obj);
    if (e == NONE32) return NONE32;
    const uint32_t slot = nr_slot(s.nsrel[(size_t)ns * s.n_rel + rel]);
    if (slot == NO_SLOT) return NONE32;
    const NsDev nd = s.ns[ns];
    return nd.node_base + (e - nd.ent_base) * nd.n_slots + slot;
}
// {row node, subject value (id, or SKEY_SET | node), subject index (rev_off space), 0}
__device__ __forceinline__ uint4 place(const DevSnapshot &s, const keto_tuple &t) {
    const uint32_t node = node_in(s, t.ns, t.obj, t.rel);
    if (t.subj_kind == 1) {
        const uint32_t c = node_in(s, t.s_ns, t.s_obj, t.s_rel);
        if (c == NONE32) return make_uint4(node, NONE32, NONE32, 0);
        return make_uint4(node, c | SKEY_SET, s.n_uuids + c, 0);
    }
    if (t.subj_kind != 0 || t.s_obj >= s.n_uuids) return make_uint4(node, NONE32, NONE32, 0);
    return make_uint4(node, t.s_obj, t.s_obj, 0);
}

__global__ __launch_bounds__(BLK) void k_place(DevSnapshot s, const keto_tuple *t, uint64_t n, uint4 *out) {
    const uint64_t i = gid();
    if (i < n) out[i] = place(s, t[i]);
}

// one pass over the store: the positions of tuples of a touched row / with a touched subject
constexpr uint32_t FILTER_WORDS = 8192;  // 256 Kbit LDS filter of both key sets
__global__ __launch_bounds__(BLK) void k_scan(const keto_tuple *t, uint64_t n, const uint32_t *filter, KeyTab rows,
                                              KeyTab subj, uint32_t *rlist, uint32_t *slist, uint32_t cap,
                                              uint32_t *counts) {
    __shared__ uint32_t f[FILTER_WORDS];
    for (uint32_t i = threadIdx.x; i < FILTER_WORDS; i += blockDim.x) f[i] = filter[i];
    __syncthreads();
    for (uint64_t i = gid(); i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const keto_tuple x = t[i];
        uint4 k;
        row_key(x, k);
        uint64_t h = key4(k.x, k.y, k.z, k.w);
        uint32_t b = (uint32_t)(h >> 40) & (FILTER_WORDS * 32 - 1);
        if ((f[b >> 5] >> (b & 31)) & 1u)
            if (tab_find(rows, k, h) != NONE32) {
                const uint32_t at = atomicAdd(&counts[0], 1u);
                if (at < cap) rlist[at] = (uint32_t)i;
            }
        subj_key(x, k);
        h = key4(k.x, k.y, k.z, k.w);
        b = (uint32_t)(h >> 40) & (FILTER_WORDS * 32 - 1);
        if ((f[b >> 5] >> (b & 31)) & 1u)
            if (tab_find(subj, k, h) != NONE32) {
                const uint32_t at = atomicAdd(&counts[1], 1u);
                if (at < cap) slist[at] = (uint32_t)i;
            }
    }
}

// matched store tuples -> {place, shard hi, shard lo} for the host
struct Match {
    uint4 p;
    uint32_t pos;
    unsigned long long hi, lo;
};
__global__ __launch_bounds__(BLK) void k_matches(DevSnapshot s, const keto_tuple *t, const uint32_t *list, uint32_t n,
                                                 Match *out) {
    const uint64_t i = gid();
    if (i >= n) return;
    const keto_tuple x = t[list[i]];
    unsigned long long hi = 0, lo = 0;
    for (int k = 0; k < 8; k++) hi = (hi << 8) | x.shard_id[k];
    for (int k = 8; k < 16; k++) lo = (lo << 8) | x.shard_id[k];
    out[i] = Match{place(s, x), list[i], hi, lo};
}

// base rows of the touched nodes / subjects: {all begin, all end, set begin, set end}
__global__ __launch_bounds__(BLK) void k_old_rows(DevSnapshot s, const uint32_t *nodes, uint32_t m, uint4 *out) {
    const uint64_t i = gid();
    if (i >= m) return;
    const uint32_t c = nodes[i];
    const uint4 r = s.set_row[c];
    out[i] = make_uint4(s.all_off[c], s.all_off[c + 1], r.x, r.y);
}
__global__ __launch_bounds__(BLK) void k_old_rev(DevSnapshot s, const uint32_t *subj, uint32_t m, uint2 *out) {
    const uint64_t i = gid();
    if (i < m) out[i] = make_uint2(s.rev_off[subj[i]], s.rev_off[subj[i] + 1]);
}
__global__ __launch_bounds__(BLK) void k_gather_ranges(const uint32_t *src, const uint2 *ranges, const uint32_t *dst_off,
                                                       uint32_t m, uint32_t *dst) {
    const uint64_t i = gid();
    if (i >= m) return;
    for (uint32_t k = ranges[i].x, o = dst_off[i]; k < ranges[i].y; k++, o++) dst[o] = src[k];
}

// ---- the shifted copies ---------------------------------------------------------------------
// rows are touched at sorted indices key[0..m); cum[j] = size change of touched rows 0..j
__device__ __forceinline__ uint32_t upper(const uint32_t *a, uint32_t m, uint64_t x) {  // # of a[j] <= x
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// offsets: dst[x] = src[x] + the change of the touched rows before x (x in [0, n])
__global__ __launch_bounds__(BLK) void k_shift_off(uint32_t *dst, const uint32_t *src, uint64_t n, const uint32_t *key,
                                                   const long long *cum, uint32_t m) {
    const uint64_t x0 = (uint64_t)blockIdx.x * blockDim.x * ITEMS + threadIdx.x;
    if (x0 > n) return;
    uint32_t j = x0 ? upper(key, m, x0 - 1) : 0;  // # of key < x0
    for (uint32_t it = 0; it < ITEMS; it++) {
        const uint64_t x = x0 + (uint64_t)it * blockDim.x;
        if (x > n) break;
        while (j < m && key[j] < x) j++;
        dst[x] = (uint32_t)((long long)src[x] + (j ? cum[j - 1] : 0));
    }
}
// values outside the touched rows, moved by the change of the touched rows before them;
// touched row j holds [beg[j], end[j]) in src
__global__ __launch_bounds__(BLK) void k_shift_vals(uint32_t *dst, const uint32_t *src, uint64_t n, const uint32_t *beg,
                                                    const uint32_t *end, const long long *cum, uint32_t m) {
    const uint64_t e0 = (uint64_t)blockIdx.x * blockDim.x * ITEMS + threadIdx.x;
    if (e0 >= n) return;
    uint32_t j = upper(beg, m, e0);  // touched rows starting at or before e0
    for (uint32_t it = 0; it < ITEMS; it++) {
        const uint64_t e = e0 + (uint64_t)it * blockDim.x;
        if (e >= n) break;
        while (j < m && beg[j] <= e) j++;
        if (j && e < end[j - 1]) continue;  // inside touched row j-1: rewritten
        dst[(long long)e + (j ? cum[j - 1] : 0)] = src[e];
    }
}
// set rows of untouched nodes: begin / end moved (inline edges kept)
__global__ __launch_bounds__(BLK) void k_shift_setrow(uint4 *dst, const uint4 *src, uint64_t n, const uint32_t *key,
                                                      const long long *cum, uint32_t m) {
    const uint64_t x0 = (uint64_t)blockIdx.x * blockDim.x * ITEMS + threadIdx.x;
    if (x0 >= n) return;
    uint32_t j = x0 ? upper(key, m, x0 - 1) : 0;  // # of key < x0
    for (uint32_t it = 0; it < ITEMS; it++) {
        const uint64_t x = x0 + (uint64_t)it * blockDim.x;
        if (x >= n) break;
        while (j < m && key[j] < x) j++;
        if (j < m && key[j] == x) continue;  // touched: written from its new row
        uint4 r = src[x];
        const long long d = j ? cum[j - 1] : 0;
        r.x = (uint32_t)((long long)r.x + d);
        r.y = (uint32_t)((long long)r.y + d);
        dst[x] = r;
    }
}
// the touched rows' new content: values [voff[j], voff[j+1]) at dst_off[key[j]]
__global__ __launch_bounds__(BLK) void k_put_rows(uint32_t *dst, const uint32_t *dst_off, const uint32_t *key,
                                                  const uint32_t *vals, const uint32_t *voff, uint32_t m) {
    const uint64_t j = gid();
    if (j >= m) return;
    for (uint32_t k = voff[j], o = dst_off[key[j]]; k < voff[j + 1]; k++, o++) dst[o] = vals[k];
}
// the touched nodes' set rows: begin / end (the edges follow once every row's extent is known)
__global__ __launch_bounds__(BLK) void k_put_setrow_extent(uint4 *set_row, const uint32_t *key, const uint32_t *begin,
                                                           const uint32_t *len, uint32_t m) {
    const uint64_t j = gid();
    if (j < m) set_row[key[j]] = make_uint4(begin[j], begin[j] + len[j], NONE32, NONE32);
}
__device__ __forceinline__ uint32_t edge_flags(const DevSnapshot &s, const uint4 *set_row, uint32_t c) {
    uint32_t f = 0;
    if (s.vkey && s.vkey[c] != c) f |= EDGE_ALIAS;
    if (s.edge_leaf && set_row[c].x == set_row[c].y) f |= EDGE_LEAF;
    return c | f;
}
// the touched rows' edges (alias / leaf flags from the new rows) and their inline copies
__global__ __launch_bounds__(BLK) void k_put_edges(DevSnapshot s, uint4 *set_row, uint32_t *set_dst, const uint32_t *key,
                                                   const uint32_t *vals, const uint32_t *voff, uint32_t m) {
    const uint64_t j = gid();
    if (j >= m) return;
    uint4 r = set_row[key[j]];
    for (uint32_t k = voff[j], o = r.x; k < voff[j + 1]; k++, o++) set_dst[o] = edge_flags(s, set_row, vals[k]);
    r.z = r.y > r.x ? set_dst[r.x] : NONE32;
    r.w = r.y > r.x + 1 ? set_dst[r.x + 1] : NONE32;
    set_row[key[j]] = r;
}
// Edges into a node whose set row became empty / non-empty: its parents are the reverse row of
// the subject set (n_uuids + c).  Two launches, one block per such node each:
//   k_flip_leaf  sets / clears EDGE_LEAF on the set_dst words naming c -- each word names one
//                child, so the blocks write disjoint words (a row listing c twice: the same
//                value twice);
//   k_fix_inline then rewrites the inline copies (set_row .z/.w) of every such parent from the
//                final set_dst.  Two flipped siblings under one parent both rewrite its row, with
//                the same words: the launch boundary orders them after every flip.  (One launch
//                let a block copy a word another block was still changing.)
__global__ __launch_bounds__(BLK) void k_flip_leaf(DevSnapshot s, const uint4 *set_row, uint32_t *set_dst,
                                                   const uint32_t *rev_off, const uint32_t *rev_nodes, const uint32_t *flip,
                                                   uint32_t m) {
    if (blockIdx.x >= m) return;
    const uint32_t c = flip[blockIdx.x];
    const bool leaf = set_row[c].x == set_row[c].y;
    const uint64_t v = (uint64_t)s.n_uuids + c;
    uint32_t rb, re;
    row_span(rev_off, s.reloc, v, rb, re);
    for (uint32_t r = rb + threadIdx.x; r < re; r += blockDim.x) {
        const uint4 row = set_row[rev_nodes[r]];
        for (uint32_t k = row.x; k < row.y; k++) {
            const uint32_t e = set_dst[k];
            if ((e & s.edge_mask) != c) continue;
            set_dst[k] = leaf ? (e | EDGE_LEAF) : (e & ~EDGE_LEAF);
        }
    }
}
__global__ __launch_bounds__(BLK) void k_fix_inline(DevSnapshot s, uint4 *set_row, const uint32_t *set_dst,
                                                    const uint32_t *rev_off, const uint32_t *rev_nodes, const uint32_t *flip,
                                                    uint32_t m) {
    if (blockIdx.x >= m) return;
    const uint64_t v = (uint64_t)s.n_uuids + flip[blockIdx.x];
    uint32_t rb, re;
    row_span(rev_off, s.reloc, v, rb, re);
    for (uint32_t r = rb + threadIdx.x; r < re; r += blockDim.x) {
        const uint32_t p = rev_nodes[r];
        uint4 row = set_row[p];
        row.z = row.y > row.x ? set_dst[row.x] : NONE32;
        row.w = row.y > row.x + 1 ? set_dst[row.x + 1] : NONE32;
        set_row[p] = row;
    }
}
// does any node of a slot still hold a subject-set row: job {slot, first node, nodes, stride};
// every thread walks each job's nodes grid-strided and stops once the job's flag is set
__global__ __launch_bounds__(BLK) void k_slot_any(const uint4 *set_row, const uint4 *job, uint32_t njobs, uint32_t *flag) {
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t j = 0; j < njobs; j++) {
        const uint4 J = job[j];
        volatile uint32_t *f = flag + j;
        uint32_t it = 0;
        for (uint64_t k = gid(); k < J.z; k += T, it++) {
            if ((it & 63) == 0 && *f) break;
            const uint4 r = set_row[J.y + k * J.w];
            if (r.x != r.y) {
                atomicOr(&flag[j], 1u);
                break;
            }
        }
    }
}
// probe keys: inserts into empty slots (or found present), removals to tombstones
__global__ __launch_bounds__(BLK) void k_probe_apply(unsigned long long *probe, uint64_t bmask, const unsigned long long *keys,
                                                     uint32_t n_ins, uint32_t n_del) {
    const uint64_t i = gid();
    if (i >= (uint64_t)n_ins + n_del) return;
    const unsigned long long key = keys[i];
    for (uint64_t b = mix64(key) & bmask;; b = (b + 1) & bmask) {
        for (int k = 0; k < 2; k++) {
            unsigned long long *slot = &probe[2 * b + k];
            if (i < n_ins) {
                const unsigned long long old = atomicCAS(slot, 0ull, key);
                if (old == 0 || old == key) return;
            } else {
                const unsigned long long cur = *slot;
                if (cur == key) {
                    *slot = PROBE_TOMB;
                    return;
                }
                if (cur == 0) return;  // not there
            }
        }
    }
}

// ent_obj of the spare entities new objects were placed on
__global__ __launch_bounds__(BLK) void k_ent_obj_set(uint32_t *ent_obj, const uint2 *set, uint32_t m) {
    const uint64_t i = gid();
    if (i < m) ent_obj[set[i].x] = set[i].y;
}

struct Touched {  // a touched row or subject, keyed for the scan
    uint4 key;
    uint32_t idx;  // node / subject index
};

// The touched tuples placed in the base's node space (step 1 of both the copy patch and the
// advance): pl[i] = place() of tuple i, with the objects the inserts create put on spares first.
struct Placed {
    std::vector<keto_tuple> ht;  // the touched tuples, host copy
    std::vector<uint4> pl;
    DevSnapshot Dp{};            // the base's view, plus the objects this patch creates
    std::vector<uint4> ext;      // the family's ext entries, this patch's included
    std::vector<uint2> ent_set;  // {spare entity, obj} taken here
    std::unique_ptr<void, void (*)(void *)> ext_dev{nullptr, [](void *p) { (void)hipFree(p); }};  // a new ext table
    // spares this patch takes go back if it then falls back to the full build (or throws), as
    // long as no later patch of the family took spares since
    struct Taken {
        std::shared_ptr<Spares> spares;
        std::vector<uint32_t> from, to;
        bool keep = false;
        ~Taken() {
            if (keep || !spares) return;
            std::lock_guard<std::mutex> g(spares->mu);
            for (size_t ns = 0; ns < from.size(); ns++)
                if (spares->used[ns] == to[ns]) spares->used[ns] = from[ns];
        }
    } taken;
};

// false: a new object cannot go on a spare (aliased visited keys, out of spares) -- build in full
bool place_touched(const Snapshot &B, const keto_tuple *touched, const uint8_t *is_ins, uint64_t n_touched, Placed &P) {
    using build::DevBuf;
    const DevSnapshot &D = B.dev;
    std::vector<keto_tuple> &ht = P.ht;
    std::vector<uint4> &pl = P.pl;
    ht.resize(n_touched);
    pl.resize(n_touched);
    P.Dp = D;
    P.ext = B.ext;
    auto place_all = [&] {
        DevBuf d_pl(sizeof(uint4) * n_touched);
        hipLaunchKernelGGL(k_place, grid_for(n_touched), dim3(BLK), 0, 0, P.Dp, touched, n_touched, static_cast<uint4 *>(d_pl.p));
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(pl.data(), d_pl.p, sizeof(uint4) * n_touched, hipMemcpyDeviceToHost));
    };
    if (n_touched) {
        KETO_HIP(hipMemcpy(ht.data(), touched, sizeof(keto_tuple) * n_touched, hipMemcpyDeviceToHost));
        place_all();
    }
    // ---- 0. objects the inserts create: the reference writes a row for any object
    // (relationtuples.go:104-126); an (ns, obj) -- row object or subject-set object -- that has no
    // entity in the base but a slot for the relation and an id inside the base's id space goes on
    // one of the namespace's spare entities (a store snapshot keeps them: BuildOpts), entered in
    // the ext table ent_lookup consults.  A namespace whose visited keys alias across namespaces
    // (relinfo bit 20) or that ran out of spares builds in full.
    std::vector<std::pair<uint32_t, uint32_t>> fresh_objs;  // (ns, obj)
    if (B.spares) {
        auto needs_entity = [&](uint32_t ns, uint32_t obj, uint32_t rel) {
            if (ns >= B.n_ns || rel >= B.n_rel || obj >= B.n_uuids) return false;
            return nr_slot(B.nsrel[(size_t)ns * B.n_rel + rel]) != NO_SLOT;
        };
        for (uint64_t i = 0; i < n_touched; i++) {
            if (!is_ins[i]) continue;
            const keto_tuple &t = ht[i];
            if (pl[i].x == NONE32 && needs_entity(t.ns, t.obj, t.rel)) fresh_objs.emplace_back(t.ns, t.obj);
            if (t.subj_kind == 1 && pl[i].y == NONE32 && needs_entity(t.s_ns, t.s_obj, t.s_rel))
                fresh_objs.emplace_back(t.s_ns, t.s_obj);
        }
        std::sort(fresh_objs.begin(), fresh_objs.end());
        fresh_objs.erase(std::unique(fresh_objs.begin(), fresh_objs.end()), fresh_objs.end());
        // (an object the row object check flagged may have an entity after all -- the tuple failed on
        // its subject; those are filtered by the device lookup below)
    }
    if (!fresh_objs.empty()) {
        std::vector<uint4> probe(fresh_objs.size());
        {   // which of them really lack an entity (ent_lookup, ext included)
            std::vector<keto_tuple> q(fresh_objs.size());
            for (size_t k = 0; k < fresh_objs.size(); k++) {
                q[k] = keto_tuple{};
                q[k].ns = fresh_objs[k].first;
                q[k].obj = fresh_objs[k].second;
                uint32_t rel = 0;  // any relation with a slot in ns
                while (rel < B.n_rel && nr_slot(B.nsrel[(size_t)q[k].ns * B.n_rel + rel]) == NO_SLOT) rel++;
                q[k].rel = rel;
                q[k].subj_kind = 0;
            }
            DevBuf dq(sizeof(keto_tuple) * q.size()), dp(sizeof(uint4) * q.size());
            KETO_HIP(hipMemcpy(dq.p, q.data(), sizeof(keto_tuple) * q.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_place, grid_for(q.size()), dim3(BLK), 0, 0, P.Dp, static_cast<const keto_tuple *>(dq.p), q.size(),
                               static_cast<uint4 *>(dp.p));
            KETO_HIP(hipGetLastError());
            KETO_HIP(hipMemcpy(probe.data(), dp.p, sizeof(uint4) * q.size(), hipMemcpyDeviceToHost));
        }
        std::lock_guard<std::mutex> g(B.spares->mu);
        // every new object's namespace is checked first -- aliased visited keys, room -- so a
        // patch that falls back to the full build takes no spare (they are the family's)
        std::vector<uint32_t> want(B.n_ns, 0);
        for (size_t k = 0; k < fresh_objs.size(); k++) {
            if (probe[k].x != NONE32) continue;  // it has an entity
            const uint32_t ns = fresh_objs[k].first;
            for (uint32_t sl = 0; sl < B.ns[ns].n_slots; sl++)
                if ((B.relinfo[B.ns[ns].slot_base + sl] >> 20) & 1u) return false;  // aliased visited keys
            if (B.spares->used[ns] + ++want[ns] > B.spares->count[ns]) return false;  // out of spares
        }
        for (size_t k = 0; k < fresh_objs.size(); k++) {
            if (probe[k].x != NONE32) continue;
            const uint32_t ns = fresh_objs[k].first, obj = fresh_objs[k].second;
            const uint32_t e = B.spares->first[ns] + B.spares->used[ns]++;
            P.ext.push_back(make_uint4(obj, ns, e, 0));
            P.ent_set.push_back(make_uint2(e, obj));
        }
        P.taken.spares = B.spares;
        P.taken.from.assign(B.n_ns, 0);
        P.taken.to.assign(B.n_ns, 0);
        for (uint32_t ns = 0; ns < B.n_ns; ns++) {
            P.taken.to[ns] = B.spares->used[ns];
            P.taken.from[ns] = P.taken.to[ns] - want[ns];
        }
    }
    if (!P.ent_set.empty()) {
        // the ext table of the new snapshot: every object placed on a spare so far in this family line
        uint32_t size = 64;
        while (size < 2 * P.ext.size()) size <<= 1;
        std::vector<uint4> tab(size, make_uint4(0, 0, NONE32, 0));
        for (const uint4 &x : P.ext) {
            uint32_t h = (uint32_t)mix64((((uint64_t)x.y << 32) | x.x) + 1) & (size - 1);
            while (tab[h].z != NONE32) h = (h + 1) & (size - 1);
            tab[h] = x;
        }
        void *ext_dev = nullptr;
        KETO_HIP(hipMalloc(&ext_dev, 16ull * size));
        P.ext_dev.reset(ext_dev);
        KETO_HIP(hipMemcpy(ext_dev, tab.data(), 16ull * size, hipMemcpyHostToDevice));
        P.Dp.ext = static_cast<const uint4 *>(ext_dev);
        P.Dp.ext_mask = size - 1;
        // the spares' uuid ids for Expand output: words of the shared ent_obj no snapshot of the
        // family reads before this one (a spare is handed out once)
        DevBuf d_set(sizeof(uint2) * P.ent_set.size());
        KETO_HIP(hipMemcpy(d_set.p, P.ent_set.data(), sizeof(uint2) * P.ent_set.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_ent_obj_set, grid_for(P.ent_set.size()), dim3(BLK), 0, 0, const_cast<uint32_t *>(D.ent_obj),
                           static_cast<const uint2 *>(d_set.p), (uint32_t)P.ent_set.size());
        KETO_HIP(hipGetLastError());
        place_all();
    }
    return true;
}

}  // namespace

Snapshot *patch_snapshot(const Snapshot &B, const keto_tuple *rows, uint64_t n_store, const keto_tuple *touched,
                         const uint8_t *is_ins, uint64_t n_touched) {
    using build::DevBuf;
    auto t0 = std::chrono::steady_clock::now();
    KETO_HIP(hipSetDevice(B.device));
    static const bool verbose = getenv("KETO_PATCH_VERBOSE") != nullptr;
    auto tp = t0;
    auto phase = [&](const char *what) {  // KETO_PATCH_VERBOSE: where the time goes
        if (!verbose) return;
        KETO_HIP(hipDeviceSynchronize());
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto patch]   %-10s %.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    const DevSnapshot &D = B.dev;
    const uint32_t N = D.n_nodes;
    const uint64_t M = (uint64_t)D.n_uuids + N;  // subject index space
    if (n_store >= (1ull << 32) || n_touched >= (1ull << 31)) return nullptr;
    // a base advanced in place holds rows outside its CSR extents: the shifted copies below
    // assume none (a full build instead)
    if (B.room.moved) return nullptr;
    // ---- 1. place the touched tuples in the base's node space -----------------------------------
    Placed P;
    if (!place_touched(B, touched, is_ins, n_touched, P)) return nullptr;
    const std::vector<keto_tuple> &ht = P.ht;
    const std::vector<uint4> &pl = P.pl;
    const DevSnapshot &Dp = P.Dp;
    const std::vector<uint4> &ext = P.ext;
    std::unordered_map<uint32_t, size_t> node_at, subj_at;  // node / subject index -> position in the sorted lists
    std::vector<Touched> tn, ts;
    std::vector<uint32_t> idrow_slots;
    for (uint64_t i = 0; i < n_touched; i++) {
        const keto_tuple &t = ht[i];
        if (pl[i].x == NONE32 || pl[i].y == NONE32) {
            if (is_ins[i]) return nullptr;  // an insert with no place in the base: build in full
            continue;                       // a delete naming no node deletes nothing the base holds
        }
        Touched a{}, b{};
        row_key(t, a.key);
        a.idx = pl[i].x;
        subj_key(t, b.key);
        b.idx = pl[i].z;
        if (node_at.emplace(a.idx, 0).second) tn.push_back(a);
        if (subj_at.emplace(b.idx, 0).second) ts.push_back(b);
        if (is_ins[i] && t.subj_kind == 0) idrow_slots.push_back(pl[i].x);
    }
    std::sort(tn.begin(), tn.end(), [](const Touched &x, const Touched &y) { return x.idx < y.idx; });
    std::sort(ts.begin(), ts.end(), [](const Touched &x, const Touched &y) { return x.idx < y.idx; });
    for (size_t j = 0; j < tn.size(); j++) node_at[tn[j].idx] = j;
    for (size_t j = 0; j < ts.size(); j++) subj_at[ts[j].idx] = j;
    const uint32_t m = (uint32_t)tn.size(), ms = (uint32_t)ts.size();

    phase("place");
    // ---- 2. the touched rows' tuples: one pass over the store ------------------------------------
    std::vector<Match> rmatch, smatch;
    if (m) {
        auto tab = [&](const std::vector<Touched> &v, DevBuf &kb, DevBuf &vb, std::vector<uint32_t> &filter) -> KeyTab {
            uint32_t size = 64;
            while (size < 4 * v.size()) size <<= 1;
            std::vector<uint4> keys(size, make_uint4(0, 0, 0, 0));
            std::vector<uint32_t> vals(size, NONE32);
            for (size_t j = 0; j < v.size(); j++) {
                const uint64_t h = key4(v[j].key.x, v[j].key.y, v[j].key.z, v[j].key.w);
                uint32_t b = (uint32_t)h & (size - 1);
                while (vals[b] != NONE32) b = (b + 1) & (size - 1);
                keys[b] = v[j].key;
                vals[b] = (uint32_t)j;
                const uint32_t fb = (uint32_t)(h >> 40) & (FILTER_WORDS * 32 - 1);
                filter[fb >> 5] |= 1u << (fb & 31);
            }
            kb = DevBuf(16ull * size);
            vb = DevBuf(4ull * size);
            KETO_HIP(hipMemcpy(kb.p, keys.data(), 16ull * size, hipMemcpyHostToDevice));
            KETO_HIP(hipMemcpy(vb.p, vals.data(), 4ull * size, hipMemcpyHostToDevice));
            return KeyTab{static_cast<const uint4 *>(kb.p), vb.u32(), size - 1};
        };
        std::vector<uint32_t> filter(FILTER_WORDS, 0);
        DevBuf rk, rv, sk, sv;
        const KeyTab RT = tab(tn, rk, rv, filter), ST = tab(ts, sk, sv, filter);
        DevBuf d_filter(4ull * FILTER_WORDS), counts(16);
        KETO_HIP(hipMemcpy(d_filter.p, filter.data(), 4ull * FILTER_WORDS, hipMemcpyHostToDevice));
        int per_cu = 0;
        KETO_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&k_scan), BLK, 0));
        const uint32_t grid = (uint32_t)std::max(1, num_cus(B.device) * std::max(per_cu, 1));
        uint32_t cap = 1u << 20;
        for (;;) {
            DevBuf rl(4ull * cap), sl(4ull * cap);
            KETO_HIP(hipMemset(counts.p, 0, 16));
            hipLaunchKernelGGL(k_scan, dim3(grid), dim3(BLK), 0, 0, rows, n_store, d_filter.u32(), RT, ST, rl.u32(), sl.u32(),
                               cap, counts.u32());
            KETO_HIP(hipGetLastError());
            uint32_t c[2];
            KETO_HIP(hipMemcpy(c, counts.p, 8, hipMemcpyDeviceToHost));
            if (c[0] > cap || c[1] > cap) {
                cap = std::max(c[0], c[1]);
                continue;
            }
            for (int w = 0; w < 2; w++) {
                std::vector<Match> &out = w ? smatch : rmatch;
                out.resize(c[w]);
                if (!c[w]) continue;
                DevBuf mb(sizeof(Match) * c[w]);
                hipLaunchKernelGGL(k_matches, grid_for(c[w]), dim3(BLK), 0, 0, Dp, rows, w ? sl.u32() : rl.u32(), c[w],
                                   static_cast<Match *>(mb.p));
                KETO_HIP(hipGetLastError());
                KETO_HIP(hipMemcpy(out.data(), mb.p, sizeof(Match) * c[w], hipMemcpyDeviceToHost));
            }
            break;
        }
    }
    for (const Match &x : rmatch)  // (store tuples of touched rows were placed by step 1 or the base build)
        if (x.p.x == NONE32 || x.p.y == NONE32) return nullptr;
    for (const Match &x : smatch)
        if (x.p.x == NONE32 || x.p.z == NONE32) return nullptr;

    phase("scan");
    // ---- 3. the touched rows' new content (host: a few rows) --------------------------------------
    std::vector<std::vector<const Match *>> per_node(m);
    for (const Match &x : rmatch) {
        auto it = node_at.find(x.p.x);
        if (it != node_at.end()) per_node[it->second].push_back(&x);
    }
    std::vector<uint32_t> key_n(m), all_vals, all_voff(m + 1, 0), set_vals, set_voff(m + 1, 0), set_len(m);
    for (uint32_t j = 0; j < m; j++) {
        key_n[j] = tn[j].idx;
        auto &v = per_node[j];
        std::sort(v.begin(), v.end(), [](const Match *a, const Match *b) {
            return a->hi != b->hi ? a->hi < b->hi : (a->lo != b->lo ? a->lo < b->lo : a->pos < b->pos);
        });
        for (const Match *x : v) {
            all_vals.push_back(x->p.y);
            if (x->p.y & SKEY_SET) set_vals.push_back(x->p.y & ~SKEY_SET);
        }
        all_voff[j + 1] = (uint32_t)all_vals.size();
        set_voff[j + 1] = (uint32_t)set_vals.size();
        set_len[j] = set_voff[j + 1] - set_voff[j];
    }
    std::vector<std::vector<uint32_t>> per_subj(ms);
    for (const Match &x : smatch) {
        auto it = subj_at.find(x.p.z);
        if (it != subj_at.end()) per_subj[it->second].push_back(x.p.x);
    }
    std::vector<uint32_t> key_s(ms), rev_vals, rev_voff(ms + 1, 0);
    for (uint32_t j = 0; j < ms; j++) {
        key_s[j] = ts[j].idx;
        std::sort(per_subj[j].begin(), per_subj[j].end());
        rev_vals.insert(rev_vals.end(), per_subj[j].begin(), per_subj[j].end());
        rev_voff[j + 1] = (uint32_t)rev_vals.size();
    }
    // the base's extents of those rows
    std::vector<uint4> old_n(m);
    std::vector<uint2> old_s(ms);
    auto up = [](const auto &v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        DevBuf b(std::max<size_t>(1, v.size()) * sizeof(T));
        if (!v.empty()) KETO_HIP(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        return b;
    };
    DevBuf d_key_n = up(key_n), d_key_s = up(key_s);
    if (m) {
        DevBuf o(sizeof(uint4) * m);
        hipLaunchKernelGGL(k_old_rows, grid_for(m), dim3(BLK), 0, 0, D, d_key_n.u32(), m, static_cast<uint4 *>(o.p));
        KETO_HIP(hipMemcpy(old_n.data(), o.p, sizeof(uint4) * m, hipMemcpyDeviceToHost));
    }
    if (ms) {
        DevBuf o(sizeof(uint2) * ms);
        hipLaunchKernelGGL(k_old_rev, grid_for(ms), dim3(BLK), 0, 0, D, d_key_s.u32(), ms, static_cast<uint2 *>(o.p));
        KETO_HIP(hipMemcpy(old_s.data(), o.p, sizeof(uint2) * ms, hipMemcpyDeviceToHost));
    }
    // the heavy subjects' old reverse rows (their probe keys)
    std::vector<uint2> heavy_rng;
    std::vector<uint32_t> heavy_off(1, 0), heavy_j;
    for (uint32_t j = 0; j < ms; j++)
        if (old_s[j].y - old_s[j].x > PROBE_K) {
            heavy_rng.push_back(old_s[j]);
            heavy_j.push_back(j);
            heavy_off.push_back(heavy_off.back() + (old_s[j].y - old_s[j].x));
        }
    std::vector<uint32_t> heavy_old(heavy_off.back());
    if (!heavy_j.empty()) {
        DevBuf r = up(heavy_rng), o = up(heavy_off), g(4ull * std::max<uint32_t>(1, heavy_off.back()));
        hipLaunchKernelGGL(k_gather_ranges, grid_for(heavy_j.size()), dim3(BLK), 0, 0, D.rev_nodes,
                           static_cast<const uint2 *>(r.p), o.u32(), (uint32_t)heavy_j.size(), g.u32());
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(heavy_old.data(), g.p, 4ull * heavy_off.back(), hipMemcpyDeviceToHost));
    }
    // probe key changes: a heavy subject's keys are exactly the distinct nodes of its reverse row
    std::vector<unsigned long long> ins_keys, del_keys;
    {
        std::vector<int64_t> hj(ms, -1);
        for (size_t h = 0; h < heavy_j.size(); h++) hj[heavy_j[h]] = (int64_t)h;
        for (uint32_t j = 0; j < ms; j++) {
            std::vector<uint32_t> nw(rev_vals.begin() + rev_voff[j], rev_vals.begin() + rev_voff[j + 1]), old;
            const bool new_heavy = nw.size() > PROBE_K;
            if (hj[j] >= 0) old.assign(heavy_old.begin() + heavy_off[hj[j]], heavy_old.begin() + heavy_off[hj[j] + 1]);
            std::sort(old.begin(), old.end());
            old.erase(std::unique(old.begin(), old.end()), old.end());
            nw.erase(std::unique(nw.begin(), nw.end()), nw.end());
            if (!new_heavy) nw.clear();
            const uint64_t v = key_s[j];
            auto key = [&](uint32_t node) { return ((v << 32) | node) + 1; };
            std::vector<uint32_t> d;
            std::set_difference(nw.begin(), nw.end(), old.begin(), old.end(), std::back_inserter(d));
            for (uint32_t x : d) ins_keys.push_back(key(x));
            d.clear();
            std::set_difference(old.begin(), old.end(), nw.begin(), nw.end(), std::back_inserter(d));
            for (uint32_t x : d) del_keys.push_back(key(x));
        }
    }
    const uint64_t probe_slots = 2ull * ((uint64_t)D.probe_mask + 1);
    if (B.probe_used + ins_keys.size() > probe_slots * 3 / 4) return nullptr;  // too full: build in full

    phase("rows");
    // ---- 4. the new snapshot: shifted copies, the touched rows, the probe keys ---------------------
    auto S = std::make_unique<Snapshot>();
    Snapshot &s = *S;
    s.device = B.device;
    s.n_ns = B.n_ns;
    s.n_rel = B.n_rel;
    s.n_rel_caller = B.n_rel_caller;
    s.n_uuids = B.n_uuids;
    s.strict = B.strict;
    s.ns_names = B.ns_names;
    s.rel_names = B.rel_names;
    s.ns = B.ns;
    s.ent_obj = B.ent_obj;
    s.slot_rel = B.slot_rel;
    s.relinfo = B.relinfo;
    s.nsrel = B.nsrel;
    s.ops = B.ops;
    s.op_children = B.op_children;
    s.op_items = B.op_items;
    s.or_items = B.or_items;
    s.info = B.info;
    s.info.device_bytes = 0;
    s.store_id = B.store_id;
    s.cfg_hash = B.cfg_hash;
    s.probe_used = B.probe_used + ins_keys.size();
    s.spares = B.spares;
    s.ext = ext;
    DevSnapshot &X = s.dev;
    X = Dp;  // (the base's arrays, its ext table or this patch's)
    X.reloc = nullptr;  // (a copy patch is not advanced in place: no room kept)
    for (const void *p : {(const void *)D.weight, (const void *)D.ent_obj, (const void *)D.slot_rel, (const void *)D.vkey,
                          (const void *)D.ns, (const void *)D.nsrel, (const void *)D.ops, (const void *)D.op_children,
                          (const void *)D.op_items, (const void *)D.or_items, (const void *)D.ent_rank, (const void *)D.ns_rcp})
        s.share(B, p);
    if (P.ext_dev) {
        s.own(P.ext_dev.release(), 16ull * ((uint64_t)Dp.ext_mask + 1));
    } else if (D.ext) {
        s.share(B, D.ext);
    }
    auto fresh = [&](size_t bytes) -> void * { return s.alloc((bytes + 31) / 16 * 16); };
    // size change per touched row, cumulative
    std::vector<long long> cum_all(m), cum_set(m), cum_rev(ms);
    std::vector<uint32_t> beg_all(m), end_all(m), beg_set(m), end_set(m), beg_rev(ms), end_rev(ms);
    long long ca = 0, cs = 0, cr = 0;
    for (uint32_t j = 0; j < m; j++) {
        beg_all[j] = old_n[j].x;
        end_all[j] = old_n[j].y;
        beg_set[j] = old_n[j].z;
        end_set[j] = old_n[j].w;
        ca += (long long)(all_voff[j + 1] - all_voff[j]) - (old_n[j].y - old_n[j].x);
        cs += (long long)set_len[j] - (old_n[j].w - old_n[j].z);
        cum_all[j] = ca;
        cum_set[j] = cs;
    }
    for (uint32_t j = 0; j < ms; j++) {
        beg_rev[j] = old_s[j].x;
        end_rev[j] = old_s[j].y;
        cr += (long long)(rev_voff[j + 1] - rev_voff[j]) - (old_s[j].y - old_s[j].x);
        cum_rev[j] = cr;
    }
    const uint64_t n_all_old = B.info.n_tuples, n_set_old = B.info.n_set_edges;
    const uint64_t n_all = (uint64_t)((long long)n_all_old + ca), n_set = (uint64_t)((long long)n_set_old + cs);
    if (n_all != n_store || (uint64_t)((long long)n_all_old + cr) != n_store) return nullptr;  // (the log and the store disagree)
    DevBuf d_cum_all = up(cum_all), d_cum_set = up(cum_set), d_cum_rev = up(cum_rev);
    DevBuf d_beg_all = up(beg_all), d_end_all = up(end_all), d_beg_set = up(beg_set), d_end_set = up(end_set);
    DevBuf d_beg_rev = up(beg_rev), d_end_rev = up(end_rev);
    DevBuf d_all_vals = up(all_vals), d_all_voff = up(all_voff), d_set_vals = up(set_vals), d_set_voff = up(set_voff);
    DevBuf d_rev_vals = up(rev_vals), d_rev_voff = up(rev_voff), d_set_len = up(set_len);
    const long long *CA = static_cast<const long long *>(d_cum_all.p), *CS = static_cast<const long long *>(d_cum_set.p),
                    *CR = static_cast<const long long *>(d_cum_rev.p);
    // all-rows (Expand)
    uint32_t *all_off = static_cast<uint32_t *>(fresh(4ull * (N + 1)));
    uint32_t *all_subj = static_cast<uint32_t *>(fresh(4ull * std::max<uint64_t>(1, n_all)));
    hipLaunchKernelGGL(k_shift_off, grid_items(N + 1), dim3(BLK), 0, 0, all_off, D.all_off, (uint64_t)N, d_key_n.u32(), CA, m);
    hipLaunchKernelGGL(k_shift_vals, grid_items(n_all_old), dim3(BLK), 0, 0, all_subj, D.all_subj, n_all_old, d_beg_all.u32(),
                       d_end_all.u32(), CA, m);
    hipLaunchKernelGGL(k_put_rows, grid_for(m), dim3(BLK), 0, 0, all_subj, all_off, d_key_n.u32(), d_all_vals.u32(),
                       d_all_voff.u32(), m);
    KETO_HIP(hipGetLastError());
    phase("all-rows");
    // reverse rows (membership)
    uint32_t *rev_off = static_cast<uint32_t *>(fresh(4ull * (M + 1)));
    uint32_t *rev_nodes = static_cast<uint32_t *>(fresh(4ull * std::max<uint64_t>(1, n_all)));
    hipLaunchKernelGGL(k_shift_off, grid_items(M + 1), dim3(BLK), 0, 0, rev_off, D.rev_off, M, d_key_s.u32(), CR, ms);
    hipLaunchKernelGGL(k_shift_vals, grid_items(n_all_old), dim3(BLK), 0, 0, rev_nodes, D.rev_nodes, n_all_old, d_beg_rev.u32(),
                       d_end_rev.u32(), CR, ms);
    hipLaunchKernelGGL(k_put_rows, grid_for(ms), dim3(BLK), 0, 0, rev_nodes, rev_off, d_key_s.u32(), d_rev_vals.u32(),
                       d_rev_voff.u32(), ms);
    KETO_HIP(hipGetLastError());
    phase("rev-rows");
    // set rows (expand-subject, tuple-to-userset): extents, then the touched rows' edges
    uint4 *set_row = static_cast<uint4 *>(fresh(16ull * N));
    uint32_t *set_dst = static_cast<uint32_t *>(fresh(4ull * n_set + 16));
    hipLaunchKernelGGL(k_shift_setrow, grid_items(N), dim3(BLK), 0, 0, set_row, D.set_row, (uint64_t)N, d_key_n.u32(), CS, m);
    hipLaunchKernelGGL(k_shift_vals, grid_items(n_set_old), dim3(BLK), 0, 0, set_dst, D.set_dst, n_set_old, d_beg_set.u32(),
                       d_end_set.u32(), CS, m);
    {
        std::vector<uint32_t> nb(m);  // new begin of each touched set row: old begin + change before it
        for (uint32_t j = 0; j < m; j++) nb[j] = (uint32_t)((long long)beg_set[j] + (j ? cum_set[j - 1] : 0));
        DevBuf d_nb = up(nb);
        hipLaunchKernelGGL(k_put_setrow_extent, grid_for(m), dim3(BLK), 0, 0, set_row, d_key_n.u32(), d_nb.u32(), d_set_len.u32(), m);
        KETO_HIP(hipGetLastError());
        X.set_row = set_row;
        hipLaunchKernelGGL(k_put_edges, grid_for(m), dim3(BLK), 0, 0, X, set_row, set_dst, d_key_n.u32(), d_set_vals.u32(),
                           d_set_voff.u32(), m);
        KETO_HIP(hipGetLastError());
    }
    phase("set-rows");
    // leaf flags of the edges into nodes whose set row changed between empty and non-empty
    std::vector<uint32_t> flip;
    for (uint32_t j = 0; j < m; j++)
        if ((set_len[j] == 0) != (old_n[j].w == old_n[j].z)) flip.push_back(key_n[j]);
    if (D.edge_leaf && !flip.empty()) {
        DevBuf d_flip = up(flip);
        hipLaunchKernelGGL(k_flip_leaf, dim3((uint32_t)flip.size()), dim3(BLK), 0, 0, X, set_row, set_dst, rev_off, rev_nodes,
                           d_flip.u32(), (uint32_t)flip.size());
        hipLaunchKernelGGL(k_fix_inline, dim3((uint32_t)flip.size()), dim3(BLK), 0, 0, X, set_row, set_dst, rev_off, rev_nodes,
                           d_flip.u32(), (uint32_t)flip.size());
        KETO_HIP(hipGetLastError());
    }
    phase("leaf");
    // probe hash: a copy with the heavy subjects' key changes
    // (exactly the base's size, no tail pad -- a probe never reads past its last bucket -- so the
    // pool's block of an earlier version of the family fits it: a fresh 16 GB block at C4 is
    // cleared by the driver at first touch, 0.2-0.7 s)
    void *probe = s.alloc(16ull * ((uint64_t)D.probe_mask + 1));
    phase("probe-get");
    KETO_HIP(hipMemcpyAsync(probe, D.probe, 16ull * ((uint64_t)D.probe_mask + 1), hipMemcpyDeviceToDevice, 0));
    phase("probe-copy");
    if (!ins_keys.empty() || !del_keys.empty()) {
        std::vector<unsigned long long> keys(ins_keys);
        keys.insert(keys.end(), del_keys.begin(), del_keys.end());
        DevBuf d_keys = up(keys);
        hipLaunchKernelGGL(k_probe_apply, grid_for(keys.size()), dim3(BLK), 0, 0, static_cast<unsigned long long *>(probe),
                           (uint64_t)D.probe_mask, static_cast<const unsigned long long *>(d_keys.p), (uint32_t)ins_keys.size(),
                           (uint32_t)del_keys.size());
        KETO_HIP(hipGetLastError());
    }
    phase("probe");
    // relation info: RI_SETROWS can only change on the slots of the touched nodes whose set row
    // flipped -- set where one became non-empty; where one became empty, kept only if another row
    // of the slot still holds a subject set (a scan of that slot's nodes, stopping at the first);
    // RI_IDROWS grows by the inserts (a stale bit only costs a probe)
    {
        auto slot_of = [&](uint32_t node) {
            const uint32_t ns = B.ns_of(node);
            return s.ns[ns].slot_base + (node - s.ns[ns].node_base) % s.ns[ns].n_slots;
        };
        std::vector<uint32_t> emptied;
        for (uint32_t j = 0; j < m; j++) {
            if ((set_len[j] == 0) == (old_n[j].w == old_n[j].z)) continue;
            const uint32_t gs = slot_of(key_n[j]);
            if (set_len[j]) s.relinfo[gs] |= RI_SETROWS;
            else emptied.push_back(gs);
        }
        std::sort(emptied.begin(), emptied.end());
        emptied.erase(std::unique(emptied.begin(), emptied.end()), emptied.end());
        if (!emptied.empty()) {
            std::vector<uint4> job;  // {global slot, first node, nodes, stride}
            for (uint32_t gs : emptied) {
                uint32_t ns = 0;
                while (ns + 1 < s.n_ns && s.ns[ns + 1].slot_base <= gs) ns++;
                const NsDev &nd = s.ns[ns];
                const uint32_t ents = (s.ns[ns + 1].node_base - nd.node_base) / std::max(1u, nd.n_slots);
                job.push_back(make_uint4(gs, nd.node_base + (gs - nd.slot_base), ents, nd.n_slots));
            }
            DevBuf d_job = up(job), flag(4ull * job.size());
            KETO_HIP(hipMemset(flag.p, 0, 4ull * job.size()));
            hipLaunchKernelGGL(k_slot_any, dim3((uint32_t)num_cus(B.device) * 4), dim3(BLK), 0, 0, set_row,
                               static_cast<const uint4 *>(d_job.p), (uint32_t)job.size(), flag.u32());
            KETO_HIP(hipGetLastError());
            std::vector<uint32_t> hf(job.size());
            KETO_HIP(hipMemcpy(hf.data(), flag.p, 4ull * job.size(), hipMemcpyDeviceToHost));
            for (size_t k = 0; k < job.size(); k++)
                s.relinfo[job[k].x] = (s.relinfo[job[k].x] & ~RI_SETROWS) | (hf[k] ? RI_SETROWS : 0u);
        }
        for (uint32_t node : idrow_slots) s.relinfo[slot_of(node)] |= RI_IDROWS;
        uint32_t *ri = static_cast<uint32_t *>(fresh(std::max<size_t>(1, s.relinfo.size()) * 4));
        if (!s.relinfo.empty()) KETO_HIP(hipMemcpy(ri, s.relinfo.data(), 4 * s.relinfo.size(), hipMemcpyHostToDevice));
        X.relinfo = ri;
    }
    KETO_HIP(hipDeviceSynchronize());
    phase("relinfo");
    X.all_off = all_off;
    X.all_subj = all_subj;
    X.rev_off = rev_off;
    X.rev_nodes = rev_nodes;
    X.set_row = set_row;
    X.set_dst = set_dst;
    X.probe = static_cast<const uint4 *>(probe);
    s.info.n_tuples = n_all;
    s.info.n_set_edges = n_set;
    s.info.n_rev_entries = n_all;
    // the reachability tables: the rows this patch changed move the reaches of their ancestors
    {
        std::vector<uint32_t> tnodes(tn.size());
        for (size_t j = 0; j < tn.size(); j++) tnodes[j] = tn[j].idx;
        patch_reach(s, B, tnodes);
    }
    phase("reach");
    s.info.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (verbose)
        fprintf(stderr, "[keto patch] %llu touched tuples: %u rows, %u subjects, %llu store matches, %zu leaf flips, "
                        "probe +%zu -%zu keys, %.2f ms\n", (unsigned long long)n_touched, m, ms,
                (unsigned long long)(rmatch.size() + smatch.size()), flip.size(), ins_keys.size(), del_keys.size(),
                s.info.build_seconds * 1e3);
    P.taken.keep = true;
    return S.release();
}

// ---- the in-place advance ---------------------------------------------------------------------
// keto_store_snapshot_advance: the transactions since a store snapshot's version applied to its own
// rows, work proportional to the rows they name -- the reference's write path touches only its
// rows (persistence/sql/relationtuples.go:104-126 WriteRelationTuples, :168-189 DeleteRelationTuples,
// :277-287 TransactRelationTuples).  A store snapshot keeps room for it (snapshot.cpp, BuildOpts::room):
//   - every all-row entry's shard key (the high 64 bits of its shard_id): a row is kept in shard
//     order (traverser.go:88, relationtuples.go:216) by inserting a new tuple before the first key
//     above its own; a key equal to its own cannot be ordered without the low half and the store
//     position -- the advance declines (a full build orders it);
//   - slack past the value arrays (all_subj, rev_nodes, set_dst): a row that grows is rewritten at
//     the tail, one that does not where it lies;
//   - a relocation table for the offset arrays (all_off, rev_off): a moved row's word becomes
//     ROW_MOVED | its entry {begin, end, the word's original offset} (layout.hpp row_span), set_row
//     is an extent already.
// The probe hash, EDGE_LEAF flags, relation info and reachability tables follow as in the copy
// patch, where they lie.  Nothing in flight may read the snapshot: the caller serves from another
// one meanwhile.  Every way to decline (placement, spares, a key tie, slack, relocation entries,
// probe load) is decided before the first write, so a declined advance leaves it as it was.
namespace {
// old rows of the touched nodes: {offset word, begin, end, original offset of a moved row}, set row
__global__ __launch_bounds__(BLK) void k_adv_old_nodes(DevSnapshot s, const uint32_t *nodes, uint32_t m, uint4 *all, uint4 *set) {
    const uint64_t j = gid();
    if (j >= m) return;
    const uint32_t c = nodes[j], w = s.all_off[c];
    uint32_t b, e;
    row_span(s.all_off, s.reloc, c, b, e);
    all[j] = make_uint4(w, b, e, (w & ROW_MOVED) ? s.reloc[w & ~ROW_MOVED].z : 0u);
    set[j] = s.set_row[c];
}
__global__ __launch_bounds__(BLK) void k_adv_old_subjects(DevSnapshot s, const uint32_t *subj, uint32_t m, uint4 *out) {
    const uint64_t j = gid();
    if (j >= m) return;
    const uint32_t v = subj[j], w = s.rev_off[v];
    uint32_t b, e;
    row_span(s.rev_off, s.reloc, v, b, e);
    out[j] = make_uint4(w, b, e, (w & ROW_MOVED) ? s.reloc[w & ~ROW_MOVED].z : 0u);
}
__global__ __launch_bounds__(BLK) void k_gather_ranges64(const unsigned long long *src, const uint2 *ranges, const uint32_t *dst_off,
                                                         uint32_t m, unsigned long long *dst) {
    const uint64_t i = gid();
    if (i >= m) return;
    for (uint32_t k = ranges[i].x, o = dst_off[i]; k < ranges[i].y; k++, o++) dst[o] = src[k];
}
// new row contents: row j = {destination, source offset in vals, length, 0}
template <class T>
__global__ __launch_bounds__(BLK) void k_put_vals(T *dst, const uint4 *rows, uint32_t m, const T *vals) {
    const uint64_t j = gid();
    if (j >= m) return;
    const uint4 r = rows[j];
    for (uint32_t k = 0; k < r.z; k++) dst[r.x + k] = vals[r.y + k];
}
__global__ __launch_bounds__(BLK) void k_put_words(uint32_t *dst, const uint2 *iv, uint32_t m) {
    const uint64_t j = gid();
    if (j < m) dst[iv[j].x] = iv[j].y;
}
__global__ __launch_bounds__(BLK) void k_put_reloc(uint4 *reloc, const uint32_t *at, const uint4 *val, uint32_t m) {
    const uint64_t j = gid();
    if (j < m) reloc[at[j]] = val[j];
}
// per slot: set edges into its nodes, its nodes with a non-empty set row (block counters in LDS)
constexpr uint32_t SLOT_LDS = 1024;
__global__ __launch_bounds__(BLK) void k_slot_counts(DevSnapshot s, uint64_t n_rows, uint32_t n_slots, unsigned long long *in_cnt,
                                                     unsigned long long *row_cnt) {
    __shared__ uint32_t lin[SLOT_LDS], lrow[SLOT_LDS];
    const bool lds = n_slots <= SLOT_LDS;
    for (uint32_t i = threadIdx.x; i < SLOT_LDS; i += blockDim.x) lin[i] = lrow[i] = 0;
    __syncthreads();
    auto slot = [&](uint32_t node) {
        uint32_t lo = 0, hi = s.n_ns;  // last namespace whose node_base <= node
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (s.ns[m].node_base <= node) lo = m;
            else hi = m;
        }
        return s.ns[lo].slot_base + (node - s.ns[lo].node_base) % s.ns[lo].n_slots;
    };
    for (uint64_t v = gid(); v < n_rows; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = s.set_row[v];
        if (r.x == r.y) continue;
        const uint32_t g = slot((uint32_t)v);
        if (lds) atomicAdd(&lrow[g], 1u);
        else atomicAdd(&row_cnt[g], 1ull);
        for (uint32_t k = r.x; k < r.y; k++) {
            const uint32_t h = slot(s.set_dst[k] & s.edge_mask);
            if (lds) atomicAdd(&lin[h], 1u);
            else atomicAdd(&in_cnt[h], 1ull);
        }
    }
    __syncthreads();
    if (lds)
        for (uint32_t i = threadIdx.x; i < n_slots; i += blockDim.x) {
            if (lin[i]) atomicAdd(&in_cnt[i], (unsigned long long)lin[i]);
            if (lrow[i]) atomicAdd(&row_cnt[i], (unsigned long long)lrow[i]);
        }
}
uint64_t shard_hi_host(const keto_tuple &t) {
    uint64_t h = 0;
    for (int k = 0; k < 8; k++) h = (h << 8) | t.shard_id[k];
    return h;
}
}  // namespace

void room_slot_counts(Snapshot &s) {
    using build::DevBuf;
    const uint32_t n_slots = (uint32_t)s.relinfo.size();
    s.slot_in.assign(n_slots, 0);
    s.slot_rows.assign(n_slots, 0);
    if (!n_slots || !s.dev.n_owned) return;
    DevBuf c(16ull * n_slots);
    KETO_HIP(hipMemset(c.p, 0, 16ull * n_slots));
    auto *in_cnt = static_cast<unsigned long long *>(c.p);
    hipLaunchKernelGGL(k_slot_counts, dim3((uint32_t)std::min<uint64_t>(4096, (s.dev.n_owned + BLK - 1) / BLK)), dim3(BLK), 0, 0, s.dev,
                       (uint64_t)s.dev.n_owned, n_slots, in_cnt, in_cnt + n_slots);
    KETO_HIP(hipGetLastError());
    KETO_HIP(hipMemcpy(s.slot_in.data(), in_cnt, 8ull * n_slots, hipMemcpyDeviceToHost));
    KETO_HIP(hipMemcpy(s.slot_rows.data(), in_cnt + n_slots, 8ull * n_slots, hipMemcpyDeviceToHost));
}

bool advance_snapshot(Snapshot &S, const keto_tuple *touched, const uint8_t *is_ins, uint64_t n_touched, uint64_t n_store) {
    using build::DevBuf;
    const auto t0 = std::chrono::steady_clock::now();
    KETO_HIP(hipSetDevice(S.device));
    static const bool verbose = getenv("KETO_PATCH_VERBOSE") != nullptr;
    auto tp = t0;
    auto phase = [&](const char *what) {
        if (!verbose) return;
        KETO_HIP(hipDeviceSynchronize());
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto advance] %-10s %.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    Snapshot::Room &R = S.room;
    DevSnapshot &D = S.dev;
    if (!R.all_shard || !D.reloc || n_touched >= (1ull << 31) || n_store >= ROW_MOVED) return false;
    if (S.slot_in.size() != S.relinfo.size() || S.slot_rows.size() != S.relinfo.size()) return false;
    for (const void *p : {(const void *)D.all_off, (const void *)D.all_subj, (const void *)D.rev_off, (const void *)D.rev_nodes,
                          (const void *)D.set_row, (const void *)D.set_dst, (const void *)D.probe, (const void *)D.reloc,
                          (const void *)R.all_shard})
        if (!S.sole(p)) return false;  // an array another snapshot shares is not this one's to rewrite
    // ---- 1. placement (new objects on spares), as the copy patch ---------------------------------
    Placed P;
    if (!place_touched(S, touched, is_ins, n_touched, P)) return false;
    const std::vector<keto_tuple> &ht = P.ht;
    const std::vector<uint4> &pl = P.pl;
    // the log entries naming each touched row / subject, in log order
    std::unordered_map<uint32_t, uint32_t> node_at, subj_at;
    std::vector<uint32_t> key_n, key_s, idrow_nodes;
    std::vector<std::vector<uint32_t>> ops_n, ops_s;
    for (uint64_t i = 0; i < n_touched; i++) {
        if (pl[i].x == NONE32 || pl[i].y == NONE32) {
            if (is_ins[i]) return false;  // an insert with no place: build in full
            continue;                     // a delete naming no node deletes nothing the snapshot holds
        }
        auto a = node_at.emplace(pl[i].x, (uint32_t)key_n.size());
        if (a.second) {
            key_n.push_back(pl[i].x);
            ops_n.emplace_back();
        }
        ops_n[a.first->second].push_back((uint32_t)i);
        auto b = subj_at.emplace(pl[i].z, (uint32_t)key_s.size());
        if (b.second) {
            key_s.push_back(pl[i].z);
            ops_s.emplace_back();
        }
        ops_s[b.first->second].push_back((uint32_t)i);
        if (is_ins[i] && ht[i].subj_kind == 0) idrow_nodes.push_back(pl[i].x);
    }
    const uint32_t m = (uint32_t)key_n.size(), ms = (uint32_t)key_s.size();
    auto up = [](const auto &v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        DevBuf b(std::max<size_t>(1, v.size()) * sizeof(T));
        if (!v.empty()) KETO_HIP(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        return b;
    };
    phase("place");
    // ---- 2. the touched rows as they are ----------------------------------------------------------
    std::vector<uint4> old_all(m), old_set(m), old_rev(ms);
    DevBuf d_key_n = up(key_n), d_key_s = up(key_s);
    if (m) {
        DevBuf a(16ull * m), b(16ull * m);
        hipLaunchKernelGGL(k_adv_old_nodes, grid_for(m), dim3(BLK), 0, 0, D, d_key_n.u32(), m, static_cast<uint4 *>(a.p),
                           static_cast<uint4 *>(b.p));
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(old_all.data(), a.p, 16ull * m, hipMemcpyDeviceToHost));
        KETO_HIP(hipMemcpy(old_set.data(), b.p, 16ull * m, hipMemcpyDeviceToHost));
    }
    if (ms) {
        DevBuf a(16ull * ms);
        hipLaunchKernelGGL(k_adv_old_subjects, grid_for(ms), dim3(BLK), 0, 0, D, d_key_s.u32(), ms, static_cast<uint4 *>(a.p));
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(old_rev.data(), a.p, 16ull * ms, hipMemcpyDeviceToHost));
    }
    auto gather = [&](const std::vector<uint4> &old, const uint32_t *src32, const unsigned long long *src64, std::vector<uint32_t> &off,
                      std::vector<uint32_t> &v32, std::vector<unsigned long long> &v64) {
        const uint32_t k = (uint32_t)old.size();
        std::vector<uint2> rng(k);
        off.assign(k + 1, 0);
        for (uint32_t j = 0; j < k; j++) {
            rng[j] = make_uint2(old[j].y, old[j].z);
            off[j + 1] = off[j] + (old[j].z - old[j].y);
        }
        v32.resize(off[k]);
        if (!k || !off[k]) return;
        DevBuf d_rng = up(rng), d_off = up(off), g(4ull * off[k]);
        hipLaunchKernelGGL(k_gather_ranges, grid_for(k), dim3(BLK), 0, 0, src32, static_cast<const uint2 *>(d_rng.p), d_off.u32(), k,
                           g.u32());
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(v32.data(), g.p, 4ull * off[k], hipMemcpyDeviceToHost));
        if (src64) {
            v64.resize(off[k]);
            DevBuf g64(8ull * off[k]);
            hipLaunchKernelGGL(k_gather_ranges64, grid_for(k), dim3(BLK), 0, 0, src64, static_cast<const uint2 *>(d_rng.p), d_off.u32(),
                               k, static_cast<unsigned long long *>(g64.p));
            KETO_HIP(hipGetLastError());
            KETO_HIP(hipMemcpy(v64.data(), g64.p, 8ull * off[k], hipMemcpyDeviceToHost));
        }
    };
    std::vector<uint32_t> all_off0, all_v0, rev_off0, rev_v0;
    std::vector<unsigned long long> shard_v0, unused;
    gather(old_all, D.all_subj, R.all_shard, all_off0, all_v0, shard_v0);
    gather(old_rev, D.rev_nodes, nullptr, rev_off0, rev_v0, unused);
    phase("gather");
    // ---- 3. the new rows: the log applied in order (inserts then deletes of each transaction) ------
    std::vector<uint32_t> all_v, set_v, rev_v, all_len(m), set_len(m), rev_len(ms);
    std::vector<unsigned long long> shard_v;
    long long d_all = 0, d_set = 0, d_rev = 0;
    auto slot_of = [&](uint32_t node) {
        const uint32_t ns = S.ns_of(node);
        return S.ns[ns].slot_base + (node - S.ns[ns].node_base) % S.ns[ns].n_slots;
    };
    std::unordered_map<uint32_t, long long> d_in;  // per slot: the change of its incoming set edges
    for (uint32_t j = 0; j < m; j++) {
        std::vector<std::pair<unsigned long long, uint32_t>> row;
        for (uint32_t k = all_off0[j]; k < all_off0[j + 1]; k++) {
            row.emplace_back(shard_v0[k], all_v0[k]);
            if (all_v0[k] & SKEY_SET) d_in[slot_of(all_v0[k] & ~SKEY_SET)]--;
        }
        for (uint32_t i : ops_n[j]) {
            const uint32_t v = pl[i].y;
            if (is_ins[i]) {
                const unsigned long long h = shard_hi_host(ht[i]);
                auto it = std::lower_bound(row.begin(), row.end(), h,
                                           [](const std::pair<unsigned long long, uint32_t> &x, unsigned long long k) { return x.first < k; });
                if (it != row.end() && it->first == h) return false;  // a key tie: only the full build orders it
                row.insert(it, std::make_pair(h, v));
            } else {  // every tuple of the row with this subject (relationtuples.go:168-189)
                row.erase(std::remove_if(row.begin(), row.end(), [v](const std::pair<unsigned long long, uint32_t> &x) { return x.second == v; }),
                          row.end());
            }
        }
        all_len[j] = (uint32_t)row.size();
        uint32_t ns = 0;
        for (const auto &x : row) {
            all_v.push_back(x.second);
            shard_v.push_back(x.first);
            if (x.second & SKEY_SET) {
                set_v.push_back(x.second & ~SKEY_SET);
                d_in[slot_of(x.second & ~SKEY_SET)]++;
                ns++;
            }
        }
        set_len[j] = ns;
        d_all += (long long)all_len[j] - (old_all[j].z - old_all[j].y);
        d_set += (long long)ns - (old_set[j].y - old_set[j].x);
    }
    std::vector<unsigned long long> ins_keys, del_keys;  // probe keys: a heavy subject's distinct nodes
    for (uint32_t j = 0; j < ms; j++) {
        std::vector<uint32_t> row(rev_v0.begin() + rev_off0[j], rev_v0.begin() + rev_off0[j + 1]), old = row;
        for (uint32_t i : ops_s[j]) {
            const uint32_t node = pl[i].x;
            if (is_ins[i]) row.push_back(node);
            else row.erase(std::remove(row.begin(), row.end(), node), row.end());
        }
        std::sort(row.begin(), row.end());
        rev_len[j] = (uint32_t)row.size();
        rev_v.insert(rev_v.end(), row.begin(), row.end());
        d_rev += (long long)rev_len[j] - (long long)old.size();
        const bool was_heavy = old.size() > PROBE_K, heavy = row.size() > PROBE_K;
        std::sort(old.begin(), old.end());
        old.erase(std::unique(old.begin(), old.end()), old.end());
        row.erase(std::unique(row.begin(), row.end()), row.end());
        if (!was_heavy) old.clear();
        if (!heavy) row.clear();
        const uint64_t v = key_s[j];
        std::vector<uint32_t> d;
        std::set_difference(row.begin(), row.end(), old.begin(), old.end(), std::back_inserter(d));
        for (uint32_t x : d) ins_keys.push_back(((v << 32) | x) + 1);
        d.clear();
        std::set_difference(old.begin(), old.end(), row.begin(), row.end(), std::back_inserter(d));
        for (uint32_t x : d) del_keys.push_back(((v << 32) | x) + 1);
    }
    if ((long long)S.info.n_tuples + d_all != (long long)n_store || d_rev != d_all) return false;  // (the log and the store disagree)
    const uint64_t probe_slots = 2ull * ((uint64_t)D.probe_mask + 1);
    if (S.probe_used + ins_keys.size() > probe_slots * 3 / 4) return false;  // too full: build in full
    // ---- 4. where each row goes: where it lies if it fits, else the tail; moved offset rows get a
    // relocation entry -------------------------------------------------------------------------------
    uint64_t at_all = R.all_tail, at_rev = R.rev_tail, at_set = R.set_tail;
    uint32_t n_reloc = R.reloc_used;
    std::vector<uint4> put_all, put_rev;  // {destination, source, length, 0}
    std::vector<uint2> all_words, rev_words;
    std::vector<uint32_t> reloc_at;
    std::vector<uint4> reloc_val;
    auto place_row = [&](const uint4 &old, uint32_t len, uint32_t src, uint32_t key, uint64_t &tail, std::vector<uint4> &put,
                         std::vector<uint2> &words) {
        const uint32_t ob = old.y, oe = old.z;
        uint32_t nb = ob;
        if (len > oe - ob) {
            nb = (uint32_t)tail;
            tail += len;
        }
        if (len) put.push_back(make_uint4(nb, src, len, 0));
        if (nb == ob && len == oe - ob) return;  // the same extent
        if (old.x & ROW_MOVED) {
            reloc_at.push_back(old.x & ~ROW_MOVED);
            reloc_val.push_back(make_uint4(nb, nb + len, old.w, 0));
        } else {
            reloc_at.push_back(n_reloc);
            reloc_val.push_back(make_uint4(nb, nb + len, old.x, 0));
            words.push_back(make_uint2(key, ROW_MOVED | n_reloc));
            n_reloc++;
        }
    };
    std::vector<uint32_t> set_begin(m), set_voff(m + 1, 0);
    for (uint32_t j = 0, src = 0; j < m; j++) {
        place_row(old_all[j], all_len[j], src, key_n[j], at_all, put_all, all_words);
        src += all_len[j];
        const uint32_t ob = old_set[j].x, oe = old_set[j].y;
        set_begin[j] = ob;
        if (set_len[j] > oe - ob) {
            set_begin[j] = (uint32_t)at_set;
            at_set += set_len[j];
        }
        set_voff[j + 1] = set_voff[j] + set_len[j];
    }
    for (uint32_t j = 0, src = 0; j < ms; j++) {
        place_row(old_rev[j], rev_len[j], src, key_s[j], at_rev, put_rev, rev_words);
        src += rev_len[j];
    }
    if (at_all > R.all_cap || at_rev > R.rev_cap || at_set > R.set_cap || n_reloc > R.reloc_cap) return false;  // no room left
    // the reachability pool: every advance appends its re-walked records and never reclaims the
    // ones they supersede, so past twice the build's entries (+ 1Mi) the advance declines and the
    // full build the caller falls back to compacts it
    if (S.reach_pool_n > 2 * S.reach_pool_built + (1u << 20)) return false;
    phase("rows");
    // every staging buffer of the writes, allocated (and filled) before the first write: an
    // allocation that fails here declines with the snapshot untouched
    std::vector<uint32_t> flip;  // set rows that changed between empty and not: their parents' EDGE_LEAF
    for (uint32_t j = 0; j < m; j++)
        if ((set_len[j] == 0) != (old_set[j].x == old_set[j].y)) flip.push_back(key_n[j]);
    std::vector<unsigned long long> keys(ins_keys);
    keys.insert(keys.end(), del_keys.begin(), del_keys.end());
    DevBuf d_all_v = up(all_v), d_shard_v = up(shard_v), d_rev_v = up(rev_v), d_put_all = up(put_all), d_put_rev = up(put_rev);
    DevBuf d_at = up(reloc_at), d_val = up(reloc_val), d_words[2] = {up(all_words), up(rev_words)};
    DevBuf d_sb = up(set_begin), d_sl = up(set_len), d_sv = up(set_v), d_svo = up(set_voff), d_flip = up(flip), d_keys = up(keys);
    uint32_t *ri_own = S.sole(D.relinfo) ? nullptr : static_cast<uint32_t *>(S.alloc(std::max<size_t>(1, S.relinfo.size()) * 4 + 16));
    // ---- 5. the writes (committed from here on) -----------------------------------------------------
    // A failure past this point (a launch, a copy, the reachability pool's growth) leaves rows
    // half-advanced: the snapshot is marked broken and every later call on it is refused
    // (capi.cpp) until the caller replaces it with a fresh cut.
    try {
    P.taken.keep = true;
    if (P.ext_dev) {  // the objects this advance created: the new ext table replaces the old one
        const void *old_ext = D.ext;
        S.own(P.ext_dev.release(), 16ull * ((uint64_t)P.Dp.ext_mask + 1));
        D.ext = P.Dp.ext;
        D.ext_mask = P.Dp.ext_mask;
        if (old_ext) S.drop(old_ext);
        S.ext = P.ext;
    }
    uint32_t *all_off = const_cast<uint32_t *>(D.all_off), *rev_off = const_cast<uint32_t *>(D.rev_off);
    uint32_t *all_subj = const_cast<uint32_t *>(D.all_subj), *rev_nodes = const_cast<uint32_t *>(D.rev_nodes);
    uint32_t *set_dst = const_cast<uint32_t *>(D.set_dst);
    uint4 *set_row = const_cast<uint4 *>(D.set_row), *reloc = const_cast<uint4 *>(D.reloc);
    if (!put_all.empty()) {
        hipLaunchKernelGGL(k_put_vals<uint32_t>, grid_for(put_all.size()), dim3(BLK), 0, 0, all_subj, static_cast<const uint4 *>(d_put_all.p),
                           (uint32_t)put_all.size(), d_all_v.u32());
        hipLaunchKernelGGL(k_put_vals<unsigned long long>, grid_for(put_all.size()), dim3(BLK), 0, 0, R.all_shard,
                           static_cast<const uint4 *>(d_put_all.p), (uint32_t)put_all.size(),
                           static_cast<const unsigned long long *>(d_shard_v.p));
    }
    if (getenv("KETO_FAULT_ADVANCE"))  // (tests only: a failure after the first write)
        throw Error(KETO_E_DEVICE, "injected fault after the advance's first write (KETO_FAULT_ADVANCE)");
    if (!put_rev.empty())
        hipLaunchKernelGGL(k_put_vals<uint32_t>, grid_for(put_rev.size()), dim3(BLK), 0, 0, rev_nodes, static_cast<const uint4 *>(d_put_rev.p),
                           (uint32_t)put_rev.size(), d_rev_v.u32());
    KETO_HIP(hipGetLastError());
    if (!reloc_at.empty()) {
        hipLaunchKernelGGL(k_put_reloc, grid_for(reloc_at.size()), dim3(BLK), 0, 0, reloc, d_at.u32(), static_cast<const uint4 *>(d_val.p),
                           (uint32_t)reloc_at.size());
        KETO_HIP(hipGetLastError());
    }
    for (int w = 0; w < 2; w++) {
        const std::vector<uint2> &words = w ? rev_words : all_words;
        if (words.empty()) continue;
        hipLaunchKernelGGL(k_put_words, grid_for(words.size()), dim3(BLK), 0, 0, w ? rev_off : all_off, static_cast<const uint2 *>(d_words[w].p),
                           (uint32_t)words.size());
        KETO_HIP(hipGetLastError());
    }
    // set rows: extents, then edges (flags from the new rows) and their inline copies
    if (m) {
        hipLaunchKernelGGL(k_put_setrow_extent, grid_for(m), dim3(BLK), 0, 0, set_row, d_key_n.u32(), d_sb.u32(), d_sl.u32(), m);
        hipLaunchKernelGGL(k_put_edges, grid_for(m), dim3(BLK), 0, 0, D, set_row, set_dst, d_key_n.u32(), d_sv.u32(), d_svo.u32(), m);
        KETO_HIP(hipGetLastError());
    }
    if (D.edge_leaf && !flip.empty()) {
        hipLaunchKernelGGL(k_flip_leaf, dim3((uint32_t)flip.size()), dim3(BLK), 0, 0, D, set_row, set_dst, rev_off, rev_nodes,
                           d_flip.u32(), (uint32_t)flip.size());
        hipLaunchKernelGGL(k_fix_inline, dim3((uint32_t)flip.size()), dim3(BLK), 0, 0, D, set_row, set_dst, rev_off, rev_nodes,
                           d_flip.u32(), (uint32_t)flip.size());
        KETO_HIP(hipGetLastError());
    }
    if (!keys.empty()) {
        hipLaunchKernelGGL(k_probe_apply, grid_for(keys.size()), dim3(BLK), 0, 0,
                           reinterpret_cast<unsigned long long *>(const_cast<uint4 *>(D.probe)), (uint64_t)D.probe_mask,
                           static_cast<const unsigned long long *>(d_keys.p), (uint32_t)ins_keys.size(), (uint32_t)del_keys.size());
        KETO_HIP(hipGetLastError());
    }
    phase("write");
    // relation info: RI_SETROWS of the slots whose rows flipped -- the slot's count of non-empty
    // set rows, kept from the rows themselves --, RI_IDROWS grows by the inserts; the per-slot
    // edge counts the reachability tables read (tabled_slots)
    {
        for (const auto &kv : d_in) S.slot_in[kv.first] = (uint64_t)((long long)S.slot_in[kv.first] + kv.second);
        for (uint32_t j = 0; j < m; j++) {
            if ((set_len[j] == 0) == (old_set[j].x == old_set[j].y)) continue;
            const uint32_t gs = slot_of(key_n[j]);
            S.slot_rows[gs] = set_len[j] ? S.slot_rows[gs] + 1 : S.slot_rows[gs] - 1;
            S.relinfo[gs] = (S.relinfo[gs] & ~RI_SETROWS) | (S.slot_rows[gs] ? RI_SETROWS : 0u);
        }
        for (uint32_t node : idrow_nodes) S.relinfo[slot_of(node)] |= RI_IDROWS;
        uint32_t *ri = ri_own ? ri_own : const_cast<uint32_t *>(D.relinfo);
        if (!S.relinfo.empty()) KETO_HIP(hipMemcpy(ri, S.relinfo.data(), 4 * S.relinfo.size(), hipMemcpyHostToDevice));
        D.relinfo = ri;
    }
    R.all_tail = at_all;
    R.rev_tail = at_rev;
    R.set_tail = at_set;
    R.reloc_used = n_reloc;
    R.moved = true;
    S.probe_used += ins_keys.size();
    S.info.n_tuples = n_store;
    S.info.n_rev_entries = n_store;
    S.info.n_set_edges = (uint64_t)((long long)S.info.n_set_edges + d_set);
    KETO_HIP(hipDeviceSynchronize());
    phase("relinfo");
    patch_reach(S, S, key_n);  // the reaches the changed rows move, where they lie
    phase("reach");
    } catch (...) {
        S.broken = true;
        throw;
    }
    S.info.build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (verbose)
        fprintf(stderr, "[keto advance] %llu touched tuples: %u rows, %u subjects, %zu moved, %zu leaf flips, probe +%zu -%zu keys, "
                        "%.2f ms\n", (unsigned long long)n_touched, m, ms, reloc_at.size(), flip.size(), ins_keys.size(),
                del_keys.size(), S.info.build_seconds * 1e3);
    return true;
}

}  // namespace keto
