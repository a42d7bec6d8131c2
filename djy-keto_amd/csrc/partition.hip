// Graphs larger than one GPU (BASELINE config 5): the relation-tuple graph
// is partitioned by object over the ranks of a job -- every tuple of (ns, obj) lives on rank
// keto_object_owner(ns, obj, world) -- so all relation slots of an object (its direct rows, the
// rows its computed usersets reach, its tuple-to-userset row) are on one rank and crossing to
// another object only happens along a subject-set edge.
//
// A batch (collective: every rank calls keto_partition_check / _expand together, each with its
// own queries) runs in three steps, all on the device except the caller's collective:
//  1. closure exchange.  The reference reads rows only of objects reachable from the query's
//     object along subject-set edges, and only while the depth ledger allows (engine.go:214-249
//     returns before any read at rest depth <= 0; the found-lookahead of traverser.go:73-80
//     reads one level further), so max_read_depth + 1 levels of a level-synchronous object BFS
//     collect every row any query of the batch can read.  Per level: the new objects (a device
//     hash set drops the ones fetched before) are routed to their owners (counting scatter,
//     one all-to-all of object keys), the owners gather those objects' tuples from their
//     key-sorted partition (binary search + two-pass compaction) and send them back (second
//     all-to-all).  The next frontier is the subject sets of the tuples received.
//     Check batches also send every owner the batch's subject ids once: a subject-id tuple is
//     only ever read by an EXISTS probe against the query's own subject (checkDirect
//     engine.go:167-208, the found-lookahead traverser.go:73-80, the OR shortcut :143-172);
//     expand-subject rows select subject sets only (traverser.go:87) and tuple-to-userset
//     skips subject ids (rewrites.go:280).  So owners ship subject-set tuples plus only the
//     subject-id tuples naming one of the batch's subjects -- the same decisions, a fraction
//     of the bytes.  Expand batches ship every tuple (leaves are part of the tree).
//  2. the closure (in shard order after the build's own sort) becomes an ordinary device
//     snapshot (build_snapshot, the replicated path's builder);
//  3. the unmodified Check / Expand kernels run on it.
// A job of one rank holds the whole graph: its partition is built once, at creation, into a
// resident snapshot (the replicated path's), and every batch runs on it directly -- no closure,
// no per-batch build (KETO_PART_CLOSURE=1 keeps the closure path, for tests of it on one GPU).
// The closure holds every row the reference engine could read for these queries, so the
// kernels take exactly the decisions (and build exactly the trees) they would on the whole
// graph; exactness needs no distributed version of the sequential walk.
//
// The collective is the caller's (keto_collective): a Go host passes its RCCL communicator's
// all-to-all, the tests pass gloo.  coll == NULL runs one rank with no exchange.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "device_common.hpp"
#include "frontier_dist.hpp"

namespace keto {
namespace {

using build::DevBuf;
constexpr uint32_t BLK = 256;
constexpr uint32_t MAX_WORLD = 4096;

inline dim3 grid_for(uint64_t n) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + BLK - 1) / BLK, 1u << 16)));
}
__device__ __forceinline__ uint64_t gid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }
__device__ __forceinline__ uint64_t okey(uint32_t ns, uint32_t obj) { return ((uint64_t)ns << 32) | obj; }
// keto_object_owner (include/keto_mi355x.h) on the device -- or the job's keto_placement
__host__ __device__ __forceinline__ uint32_t owner_of(uint64_t key, const Dest &D) {
    return D.owner((uint32_t)(key >> 32), (uint32_t)key);
}

// ------------------------------------------------------------------ kernels

// Appends to one counter: a block reserves its range with one atomic (per-wave atomics on a
// single counter serialise at its L2 channel: k_next spent 3.3 ms of a C3 x10 batch on them).
// Each thread offers up to K values (bit k of `mask`); every thread of the block calls it.
constexpr uint32_t TILE_K = 8;  // values per thread per call: one atomic per BLK * TILE_K items
__device__ __forceinline__ unsigned long long block_reserve(uint32_t cnt, unsigned long long *n_out,
                                                            unsigned long long *s_base, uint32_t *s_wsum) {
    const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    uint32_t x = cnt;  // inclusive scan over the wave
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_wsum[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < nw; w++) {
            const uint32_t v = s_wsum[w];
            s_wsum[w] = (uint32_t)t;
            t += v;
        }
        *s_base = t ? atomicAdd(n_out, t) : 0ull;
    }
    __syncthreads();
    const unsigned long long o = *s_base + s_wsum[wv] + x - cnt;
    __syncthreads();  // (the shared words are reused by the next call)
    return o;
}
template <class T>
__device__ __forceinline__ void block_append(const T (&v)[TILE_K], uint32_t mask, T *out, unsigned long long *n_out) {
    __shared__ unsigned long long s_base;
    __shared__ uint32_t s_wsum[BLK / 64];
    unsigned long long o = block_reserve((uint32_t)__popc(mask), n_out, &s_base, s_wsum);
    for (uint32_t k = 0; k < TILE_K; k++)
        if ((mask >> k) & 1u) out[o++] = v[k];
}
// grid-stride over tiles of blockDim * TILE_K items, uniform per block; item k of a thread's
// tile is i = tile + k * blockDim + threadIdx (coalesced)
#define FOR_TILES(t0, n)                                                                                  \
    for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x * TILE_K; t0 < (n);                          \
         t0 += (uint64_t)gridDim.x * blockDim.x * TILE_K)
inline dim3 grid_tiles(uint64_t n) { return grid_for((n + TILE_K - 1) / TILE_K); }

// sort key of a store tuple: its object key, then subject sets before subject ids
__global__ __launch_bounds__(BLK) void k_tuple_keys(const keto_tuple *t, uint64_t n, uint64_t *keys, uint32_t *idx) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        keys[i] = (okey(t[i].ns, t[i].obj) << 1) | (t[i].subj_kind == 1 ? 0u : 1u);
        idx[i] = (uint32_t)i;
    }
}
// The partition's store, grouped by object: a run's (ns, obj) is its key, so a tuple keeps only
// its subject and relations -- 24 bytes instead of keto_tuple's 48 (a config-5 partition is
// billions of tuples): meta = {s_obj, rel | s_rel << 10 | s_ns << 20 | subj_kind << 31} and
// the shard_id (16 B, it orders every row).  partition_create checks that the name tables fit.
constexpr uint32_t ST_REL_BITS = 10, ST_NS_BITS = 11;
__device__ __forceinline__ uint2 st_meta(const keto_tuple &t) {
    return make_uint2(t.s_obj, t.rel | (t.s_rel << ST_REL_BITS) | (t.s_ns << (2 * ST_REL_BITS)) | (t.subj_kind << 31));
}
__device__ __forceinline__ keto_tuple st_tuple(uint64_t key, uint2 m, uint4 shard) {
    keto_tuple t;
    t.ns = (uint32_t)(key >> 32);
    t.obj = (uint32_t)key;
    t.rel = m.y & ((1u << ST_REL_BITS) - 1u);
    t.subj_kind = m.y >> 31;
    t.s_obj = m.x;
    t.s_ns = (m.y >> (2 * ST_REL_BITS)) & ((1u << ST_NS_BITS) - 1u);
    t.s_rel = (m.y >> ST_REL_BITS) & ((1u << ST_REL_BITS) - 1u);
    t.reserved = 0;
    *reinterpret_cast<uint4 *>(t.shard_id) = shard;
    return t;
}
__global__ __launch_bounds__(BLK) void k_gather_store(const keto_tuple *t, const uint32_t *idx, uint64_t n, uint2 *meta,
                                                      uint4 *shard, unsigned long long *bad) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        const keto_tuple &x = t[idx[i]];
        if (x.rel >> ST_REL_BITS || x.s_rel >> ST_REL_BITS || x.s_ns >> ST_NS_BITS || x.subj_kind > 1) atomicOr(bad, 1ull);
        meta[i] = st_meta(x);
        shard[i] = *reinterpret_cast<const uint4 *>(x.shard_id);
    }
}
// run starts of the sorted keys: flag[i] = key[i] != key[i-1]
__global__ __launch_bounds__(BLK) void k_run_flags(const uint64_t *k, uint64_t n, uint32_t *flag) {
    for (uint64_t i = gid(); i < n; i += gstride()) flag[i] = (i == 0 || (k[i] >> 1) != (k[i - 1] >> 1)) ? 1u : 0u;
}
// compacted runs: run r starts at the i with flag[i] and exclusive-scan pos[i] == r
__global__ __launch_bounds__(BLK) void k_run_starts(const uint64_t *k, const uint32_t *flag, const uint32_t *pos,
                                                     uint64_t n, uint64_t *ukeys, uint64_t *beg) {
    for (uint64_t i = gid(); i < n; i += gstride())
        if (flag[i]) {
            ukeys[pos[i]] = k[i] >> 1;
            beg[pos[i]] = i;
        }
}
__global__ __launch_bounds__(BLK) void k_query_keys(const keto_query *q, uint64_t n, uint64_t *keys, uint32_t *subj,
                                                     unsigned long long *n_subj) {
    FOR_TILES(t0, n) {
        uint32_t v[TILE_K], mask = 0;
        for (uint32_t k = 0; k < TILE_K; k++) {
            const uint64_t i = t0 + (uint64_t)k * blockDim.x + threadIdx.x;
            v[k] = 0;
            if (i >= n) continue;
            keys[i] = okey(q[i].ns, q[i].obj);
            if (q[i].subj_kind == 0) {
                v[k] = q[i].s_obj;
                mask |= 1u << k;
            }
        }
        block_append<uint32_t>(v, mask, subj, n_subj);
    }
}
__global__ __launch_bounds__(BLK) void k_root_keys(const keto_subject_set *r, uint64_t n, uint64_t *keys) {
    for (uint64_t i = gid(); i < n; i += gstride()) keys[i] = okey(r[i].ns, r[i].obj);
}
// seen-set insert: keys never asked for before go to `out` (each once)
__global__ __launch_bounds__(BLK) void k_insert(const uint64_t *cand, uint64_t n, const unsigned long long *n_dev,
                                                 unsigned long long *table, uint64_t mask, uint64_t *out,
                                                 unsigned long long *n_out) {
    if (n_dev) n = *n_dev;  // (a level launched before its count reached the host)
    FOR_TILES(t0, n) {
        uint64_t v[TILE_K];
        uint32_t fresh = 0;
        for (uint32_t k = 0; k < TILE_K; k++) {
            const uint64_t i = t0 + (uint64_t)k * blockDim.x + threadIdx.x;
            v[k] = 0;
            if (i >= n) continue;
            const unsigned long long key = cand[i] + 1;  // 0 = empty slot
            v[k] = cand[i];
            uint64_t h = mix64(key) & mask;
            for (;;) {
                // most candidates were seen before (popular groups, shared ancestors): a plain load
                // answers them, the atomic is only for an empty slot
                unsigned long long prev = __atomic_load_n(&table[h], __ATOMIC_RELAXED);
                if (prev == 0ull) prev = atomicCAS(&table[h], 0ull, key);
                if (prev == 0ull) {
                    fresh |= 1u << k;
                    break;
                }
                if (prev == key) break;
                h = (h + 1) & mask;
            }
        }
        block_append<uint64_t>(v, fresh, out, n_out);
    }
}
__global__ __launch_bounds__(BLK) void k_rehash(const uint64_t *keys, uint64_t n, unsigned long long *table,
                                                 uint64_t mask) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        const unsigned long long k = keys[i] + 1;
        uint64_t h = mix64(k) & mask;
        while (atomicCAS(&table[h], 0ull, k) != 0ull) h = (h + 1) & mask;
    }
}
// routing: destination histogram, then a counting scatter (order within a destination is free)
__global__ __launch_bounds__(BLK) void k_dest_hist(const uint64_t *keys, uint64_t n, Dest D, unsigned long long *hist) {
    for (uint64_t i = gid(); i < n; i += gstride()) atomicAdd(&hist[owner_of(keys[i], D)], 1ull);
}
__global__ __launch_bounds__(BLK) void k_dest_scatter(const uint64_t *keys, uint64_t n, Dest D, unsigned long long *cursor,
                                                       uint64_t *out) {
    for (uint64_t i = gid(); i < n; i += gstride()) out[atomicAdd(&cursor[owner_of(keys[i], D)], 1ull)] = keys[i];
}
// object-key index of the partition: open addressing, {key lo, key hi, run, 0} per slot
__global__ __launch_bounds__(BLK) void k_index_fill(const uint64_t *ukeys, uint64_t m, uint4 *slots, uint64_t mask) {
    for (uint64_t r = gid(); r < m; r += gstride()) {
        const uint64_t k = ukeys[r];
        uint64_t h = mix64(k + 1) & mask;
        // claim a slot by its run word (NONE32 = empty), then publish the key
        while (atomicCAS(&slots[h].z, NONE32, (uint32_t)r) != NONE32) h = (h + 1) & mask;
        slots[h].x = (uint32_t)k;
        slots[h].y = (uint32_t)(k >> 32);
    }
}

// owner side: tuples to ship for each requested key (all of them for Expand; subject sets plus
// subject ids in the requester's subject list for Check)
struct Lookup {
    const uint64_t *ukeys, *beg;  // partition runs: ukeys[m], beg[m+1]
    uint64_t m;
    const uint4 *index;           // k_index_fill table
    uint64_t index_mask;
    const uint2 *meta;            // the store (k_gather_store): subject + relations, and shard ids
    const uint4 *shard;
    const uint64_t *req;          // requested keys, grouped by source rank
    const uint64_t *req_off;      // [world+1] request offsets per source
    const unsigned long long *subj_set;  // (source, subject id) hash set (k_subj_fill)
    uint64_t subj_mask;
    const uint32_t *subj_bits;    // 2^SUBJ_BITS-bit filter of the set: most subject-id tuples miss it
    uint32_t world;
    int filter;
    // a job over resident partitions (frontier_dist.hip): the rows of the rank's own snapshot stand
    // for the store -- an object's tuples are its nodes' Expand rows (all_off / all_subj: one
    // contiguous range per entity, slot after slot, each in shard order)
    bool use_snap = false;
    DevSnapshot S{};
};
__device__ __forceinline__ unsigned long long subj_key(uint32_t src, uint32_t sid) {
    return (((unsigned long long)src << 32) | sid) + 1ull;  // 0 = empty slot
}
constexpr uint32_t SUBJ_BITS = 24;  // 2 MB: the batch's subjects set a few percent of the bits
__device__ __forceinline__ uint32_t subj_bit(unsigned long long k) {
    return (uint32_t)(mix64(k) >> 40) & ((1u << SUBJ_BITS) - 1u);
}
// the subject lists every source sent (concatenated, soff[world+1]) into one hash set
__global__ __launch_bounds__(BLK) void k_subj_fill(const uint32_t *subj, const uint64_t *soff, uint32_t world,
                                                    uint64_t n, unsigned long long *set, uint64_t mask, uint32_t *bits) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        uint32_t lo = 0, hi = world;  // last source whose offset <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (soff[mid] <= i) lo = mid;
            else hi = mid;
        }
        const unsigned long long k = subj_key(lo, subj[i]);
        const uint32_t b = subj_bit(k);
        atomicOr(&bits[b >> 5], 1u << (b & 31u));
        uint64_t h = mix64(k) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&set[h], 0ull, k);
            if (prev == 0ull || prev == k) break;
            h = (h + 1) & mask;
        }
    }
}
// a key's range in a k_index_fill table over runs (beg[run], beg[run + 1])
__device__ __forceinline__ bool index_range(const uint4 *index, uint64_t mask, const uint64_t *beg, uint64_t key, uint64_t &b,
                                            uint64_t &e, uint32_t &run) {
    uint64_t h = mix64(key + 1) & mask;
    for (;;) {  // one 16-byte probe per step; the table is at most half full
        const uint4 sl = index[h];
        if (sl.z == NONE32) return false;
        if (sl.x == (uint32_t)key && sl.y == (uint32_t)(key >> 32)) {
            run = sl.z;
            b = beg[sl.z];
            e = beg[sl.z + 1];
            return true;
        }
        h = (h + 1) & mask;
    }
}
__device__ __forceinline__ bool run_of(const Lookup &L, uint64_t key, uint64_t &b, uint64_t &e) {
    if (L.use_snap) {
        const uint32_t ns = (uint32_t)(key >> 32), en = ent_lookup(L.S, ns, (uint32_t)key);
        if (en == NONE32) return false;
        const NsDev nd = L.S.ns[ns];
        const uint32_t node0 = nd.node_base + (en - nd.ent_base) * nd.n_slots;
        b = L.S.all_off[node0];
        e = L.S.all_off[node0 + nd.n_slots];
        return true;
    }
    uint32_t r;
    return index_range(L.index, L.index_mask, L.beg, key, b, e, r);
}
// the store record at position j: {subject, kind bit 31} (st_meta's fields the filter reads)
__device__ __forceinline__ uint2 meta_at(const Lookup &L, uint64_t j) {
    if (L.use_snap) {
        const uint32_t sub = L.S.all_subj[j];
        return make_uint2(sub & ~SKEY_SET, (sub & SKEY_SET) ? 1u << 31 : 0u);
    }
    return L.meta[j];
}
// the tuple at position j of key's run.  Resident snapshots: its node is the slot whose all-row
// holds j, and its shard_id the position in that row (big-endian), which is all the closure
// snapshot's sort by shard_id needs to rebuild every row in order
__device__ __forceinline__ keto_tuple tuple_at(const Lookup &L, uint64_t key, uint64_t j) {
    if (!L.use_snap) return st_tuple(key, L.meta[j], L.shard[j]);
    const DevSnapshot &S = L.S;
    const uint32_t ns = (uint32_t)(key >> 32), obj = (uint32_t)key;
    const NsDev nd = S.ns[ns];
    const uint32_t node0 = nd.node_base + (ent_lookup(S, ns, obj) - nd.ent_base) * nd.n_slots;
    uint32_t k = 0;
    while (k + 1 < nd.n_slots && S.all_off[node0 + k + 1] <= j) k++;
    keto_tuple t;
    t.ns = ns;
    t.obj = obj;
    t.rel = S.slot_rel[nd.slot_base + k];
    t.reserved = 0;
    const uint32_t sub = S.all_subj[j];
    if (sub & SKEY_SET) {
        const uint32_t c = sub & ~SKEY_SET;
        uint32_t lo = 0, hi = ns_entries(S);  // last ns table entry whose node_base <= c (ghosts included)
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (S.ns[m].node_base <= c) lo = m;
            else hi = m;
        }
        const NsDev n2 = S.ns[lo];
        t.subj_kind = 1;
        t.s_ns = lo >= S.n_ns ? lo - S.n_ns : lo;
        t.s_obj = S.ent_obj[n2.ent_base + (c - n2.node_base) / n2.n_slots];
        t.s_rel = S.slot_rel[n2.slot_base + (c - n2.node_base) % n2.n_slots];
    } else {
        t.subj_kind = 0;
        t.s_obj = sub;
        t.s_ns = 0;
        t.s_rel = 0;
    }
    const uint32_t p = (uint32_t)(j - S.all_off[node0 + k]);  // shard_id bytes 0-3 = p, big-endian
    *reinterpret_cast<uint4 *>(t.shard_id) =
        make_uint4(((p >> 24) & 0xFFu) | (((p >> 16) & 0xFFu) << 8) | (((p >> 8) & 0xFFu) << 16) | ((p & 0xFFu) << 24), 0, 0, 0);
    return t;
}
__device__ __forceinline__ uint32_t source_of(const Lookup &L, uint64_t i) {
    uint32_t lo = 0, hi = L.world;  // last source whose offset <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.req_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ bool keep(const Lookup &L, uint2 m, uint32_t src) {
    if (!L.filter || (m.y >> 31)) return true;
    const unsigned long long k = subj_key(src, m.x);
    const uint32_t b = subj_bit(k);
    if (!((L.subj_bits[b >> 5] >> (b & 31u)) & 1u)) return false;
    uint64_t h = mix64(k) & L.subj_mask;
    for (;;) {  // at most half full: every probe sequence ends at an empty slot
        const unsigned long long v = L.subj_set[h];
        if (v == k) return true;
        if (v == 0ull) return false;
        h = (h + 1) & L.subj_mask;
    }
}
__global__ __launch_bounds__(BLK) void k_lookup_count(Lookup L, uint64_t n, uint32_t *cnt) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        uint64_t b, e;
        uint32_t c = 0;
        if (run_of(L, L.req[i], b, e)) {
            const uint32_t src = source_of(L, i);
            for (uint64_t j = b; j < e; j++) c += keep(L, meta_at(L, j), src) ? 1 : 0;
        }
        cnt[i] = c;
    }
}
__global__ __launch_bounds__(BLK) void k_lookup_fill(Lookup L, uint64_t n, const uint32_t *pos, keto_tuple *out) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        uint64_t b, e;
        if (!run_of(L, L.req[i], b, e)) continue;
        const uint32_t src = source_of(L, i);
        uint64_t o = pos[i];
        for (uint64_t j = b; j < e; j++)
            if (keep(L, meta_at(L, j), src)) out[o++] = tuple_at(L, L.req[i], j);
    }
}
// Block exclusive scan of one u32 per thread (wave scans + the waves' sums); *tot = the sum.
__device__ __forceinline__ uint32_t block_excl_u32(uint32_t v, uint32_t *s_wsum, uint32_t *tot) {
    const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    uint32_t x = v;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_wsum[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < nw; w++) {
            const uint32_t y = s_wsum[w];
            s_wsum[w] = t;
            t += y;
        }
        s_wsum[nw] = t;
    }
    __syncthreads();
    const uint32_t r = s_wsum[wv] + x - v;
    *tot = s_wsum[nw];
    __syncthreads();
    return r;
}
// One pass for a rank gathering for itself (no grouping by source needed; the closure's order
// is free: the builder sorts every row by shard_id).  A block takes BLK requests and lays their
// runs end to end, a virtual list of tuples that all its threads then walk in segments of GSEG
// items: a lane's work no longer depends on how long its own object's run is (folder runs of
// hundreds of viewer tuples next to runs of one).  Per segment the kept tuples are marked in an
// LDS bitmap, one range is reserved for them, and they are written in list order.  An item
// past `cap` sets *overflow; the host then reruns the level with the two passes.
constexpr uint32_t GSEG = BLK * 32;  // items per segment: one 32-bit bitmap word per thread
__global__ __launch_bounds__(BLK) void k_lookup_gather(Lookup L, uint64_t n, const unsigned long long *n_dev, keto_tuple *out,
                                                        uint64_t cap, unsigned long long *total,
                                                        unsigned long long *overflow) {
    if (n_dev) n = *n_dev;
    __shared__ uint64_t s_b[BLK], s_key[BLK];
    __shared__ uint32_t s_off[BLK + 1], s_bits[GSEG / 32], s_wsum[BLK / 64 + 1];
    __shared__ unsigned long long s_wpos[GSEG / 32], s_base;
    const uint32_t t = threadIdx.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * BLK; i0 < n; i0 += (uint64_t)gridDim.x * BLK) {
        const uint64_t i = i0 + t;
        uint64_t b = 0, e = 0;
        const uint64_t key = i < n ? L.req[i] : 0ull;
        if (i < n) run_of(L, key, b, e);
        uint32_t T = 0;
        const uint32_t off = block_excl_u32((uint32_t)(e - b), s_wsum, &T);
        s_off[t] = off;
        s_b[t] = b;
        s_key[t] = key;
        if (t == 0) s_off[BLK] = T;
        __syncthreads();
        for (uint32_t S0 = 0; S0 < T; S0 += GSEG) {
            const uint32_t segn = min(GSEG, T - S0);
            // marking pass: item v = k * BLK + t (consecutive lanes, consecutive tuples of a run);
            // a wave's 64 answers are two bitmap words
            for (uint32_t k = 0; k < GSEG / BLK; k++) {
                const uint32_t v = k * BLK + t, x = S0 + v;
                bool kp = false;
                if (v < segn) {
                    uint32_t lo = 0, hi = BLK;  // the request whose range holds x
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_off[mid] <= x) lo = mid;
                        else hi = mid;
                    }
                    kp = keep(L, meta_at(L, s_b[lo] + (x - s_off[lo])), 0);
                }
                const unsigned long long m = __ballot(kp);
                const uint32_t lane = __lane_id();
                if (lane == 0) s_bits[v >> 5] = (uint32_t)m;
                if (lane == 32) s_bits[v >> 5] = (uint32_t)(m >> 32);
            }
            __syncthreads();
            const uint32_t word = s_bits[t];
            const unsigned long long o = block_reserve((uint32_t)__popc(word), total, &s_base, s_wsum);
            s_wpos[t] = o;
            __syncthreads();
            // write pass: consecutive threads take consecutive items (coalesced stores)
            for (uint32_t v = t; v < segn; v += BLK) {
                const uint32_t wd = s_bits[v >> 5], bit = v & 31u;
                if (!((wd >> bit) & 1u)) continue;
                const unsigned long long pos = s_wpos[v >> 5] + (uint32_t)__popc(wd & ((1u << bit) - 1u));
                if (pos >= cap) {
                    atomicOr(overflow, 1ull);
                    continue;
                }
                const uint32_t x = S0 + v;
                uint32_t lo = 0, hi = BLK;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_off[mid] <= x) lo = mid;
                    else hi = mid;
                }
                const uint64_t j = s_b[lo] + (x - s_off[lo]);
                out[pos] = tuple_at(L, s_key[lo], j);
            }
            __syncthreads();
        }
    }
}

// next frontier: the subject-set objects of the tuples received
__global__ __launch_bounds__(BLK) void k_next(const keto_tuple *t, uint64_t n, const unsigned long long *range_dev,
                                               uint64_t *cand, unsigned long long *n_cand) {
    if (range_dev) {  // the level's tuples: [range_dev[0], range_dev[1]) of the closure
        t += range_dev[0];
        n = range_dev[1] - range_dev[0];
    }
    FOR_TILES(t0, n) {
        uint64_t v[TILE_K];
        uint32_t mask = 0;
        for (uint32_t k = 0; k < TILE_K; k++) {
            const uint64_t i = t0 + (uint64_t)k * blockDim.x + threadIdx.x;
            v[k] = 0;
            if (i < n && t[i].subj_kind == 1) {
                v[k] = okey(t[i].s_ns, t[i].s_obj);
                mask |= 1u << k;
            }
        }
        block_append<uint64_t>(v, mask, cand, n_cand);
    }
}

// *any = 1 when some query of the batch has an error code
__global__ __launch_bounds__(BLK) void k_any_nonzero(const int32_t *err, uint64_t n, unsigned long long *any) {
    for (uint64_t i = gid(); i < n; i += gstride())
        if (err[i] && !*any) atomicOr(any, 1ull);
}
// a device-side level boundary: *dst = min(*total, cap)
__global__ void k_mark(const unsigned long long *total, unsigned long long *dst, unsigned long long cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *dst = *total < cap ? *total : cap;
}

// Compact id space of a closure (remap_ids): the uuid ids its tuples and the batch's queries /
// roots name, ranked in global order.  The builder sizes its entity table and reverse offsets
// by the id space, so a closure snapshot over local ids costs its tuples, not the whole graph's
// uuid range.  Decisions and trees do not depend on the ids' values, only on equality.
__global__ __launch_bounds__(BLK) void k_ids_tuples(const keto_tuple *t, uint64_t n, uint32_t *ids, uint32_t *pos) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        ids[2 * i] = t[i].obj;
        ids[2 * i + 1] = t[i].s_obj;
        pos[2 * i] = (uint32_t)(2 * i);
        pos[2 * i + 1] = (uint32_t)(2 * i + 1);
    }
}
__global__ __launch_bounds__(BLK) void k_ids_queries(const keto_query *q, uint64_t n, uint64_t base, uint32_t *ids,
                                                      uint32_t *pos) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        ids[base + 2 * i] = q[i].obj;
        ids[base + 2 * i + 1] = q[i].s_obj;
        pos[base + 2 * i] = (uint32_t)(base + 2 * i);
        pos[base + 2 * i + 1] = (uint32_t)(base + 2 * i + 1);
    }
}
__global__ __launch_bounds__(BLK) void k_ids_roots(const keto_subject_set *r, uint64_t n, uint64_t base, uint32_t *ids,
                                                    uint32_t *pos) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        ids[base + i] = r[i].obj;
        pos[base + i] = (uint32_t)(base + i);
    }
}
// sorted entry i: local id = (distinct ids before it, the exclusive scan of the run flags)
// + its own flag - 1
__global__ __launch_bounds__(BLK) void k_ids_assign(const uint32_t *sk, const uint32_t *spos, const uint32_t *excl,
                                                     uint64_t n, uint32_t *lid, uint32_t *uniq) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        const bool head = i == 0 || sk[i] != sk[i - 1];
        const uint32_t l = excl[i] + (head ? 1u : 0u) - 1u;
        lid[spos[i]] = l;
        if (head) uniq[l] = sk[i];
    }
}
__global__ __launch_bounds__(BLK) void k_apply_tuples(keto_tuple *t, uint64_t n, const uint32_t *lid) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        t[i].obj = lid[2 * i];
        t[i].s_obj = lid[2 * i + 1];
    }
}
__global__ __launch_bounds__(BLK) void k_apply_queries(keto_query *q, uint64_t n, uint64_t base, const uint32_t *lid) {
    for (uint64_t i = gid(); i < n; i += gstride()) {
        q[i].obj = lid[base + 2 * i];
        q[i].s_obj = lid[base + 2 * i + 1];
    }
}
__global__ __launch_bounds__(BLK) void k_apply_roots(keto_subject_set *r, uint64_t n, uint64_t base, const uint32_t *lid) {
    for (uint64_t i = gid(); i < n; i += gstride()) r[i].obj = lid[base + i];
}

// ------------------------------------------------------------------ host side

template <class T>
T *dptr(const DevBuf &b) { return static_cast<T *>(b.p); }

void ensure(DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return;
    b = DevBuf(std::max<size_t>(bytes, 256));
}

struct Partition {
    int device = 0;
    bool have_coll = false;
    keto_collective coll{};
    uint32_t rank = 0, world = 1;
    Placement place{};  // which objects each rank owns (keto_placement; zeros: keto_object_owner's hash)
    keto_limits limits{5, 100};
    // snapshot configuration for the per-batch closure builds
    std::vector<std::string> ns_names, rel_names;
    std::vector<const char *> ns_ptr, rel_ptr;
    std::string json;
    keto_snapshot_config cfg{};
    // this rank's partition, sorted by object key: store meta[n] + shard[n] (k_gather_store), run
    // keys ukeys[m], beg[m+1]
    DevBuf meta, shard, ukeys, beg, index;
    uint64_t n = 0, m = 0, index_mask = 0;
    // a job of one rank: the whole graph as one resident snapshot, built at creation (null: the
    // per-batch closure path)
    std::unique_ptr<Snapshot> home;
    // a job of several ranks: this rank's partition as a resident snapshot and the distributed
    // frontier engine over it (frontier_dist.hip); the closure path answers its routed queries and
    // Expand, reading that snapshot's rows (no separate store)
    DistEngine *dist = nullptr;
    DistStats dstats{};
    hipStream_t hs = nullptr;
    keto_stream *kstream = nullptr;
    // per-batch workspace (grown on demand, reused)
    DevBuf table, seen, cand, fresh, routed, req, req_off, subj, subj_off, subj_set, subj_bits, cnt, pos, out, got, scratch, ctr,
        closure, lctr;
    uint64_t subj_mask = 0;
    // compact id space of the last closure (remap_ids): local id -> global uuid id
    DevBuf rm_ids, rm_pos, rm_ids2, rm_pos2, rm_flag, rm_lid, uniq, bout;
    uint64_t n_local = 0;
    void *hpin = nullptr;  // pinned staging for a batch's decisions
    size_t hpin_bytes = 0;
    // batches in flight (partition_check_many): the closure of batch k+1 (stage 1: hs, the
    // members above) runs while batch k is remapped, built and checked (stage 2: hs2,
    // ctr2, the remap buffers, kstream); each batch's closure and queries live in its slot
    struct Slot {
        DevBuf closure, bq;
        uint64_t nt = 0;
        keto_partition_stats st{};
        std::vector<keto_partition_level> levels;
    };
    Slot slots[2];
    hipStream_t hs2 = nullptr;
    DevBuf ctr2;
    DevBuf bq, braw, bsorted, braw_v, bsorted_v, bkeys, bsubj, bsubj_src, bhist;  // per-batch inputs, reused
    bool verbose = false;
    bool trim = false;  // KETO_PART_TRIM: the engine stream's scratch is released after every batch
    uint64_t table_mask = 0, n_seen = 0;
    keto_partition_stats last{};
    std::vector<keto_partition_level> cur_levels, last_levels;  // the closure running / the last batch's
    std::vector<keto_partition_generation> last_gens;           // the last distributed-frontier batch's generations
    // Expand results between keto_partition_expand and keto_partition_expand_result
    std::vector<keto_tree_node> xnodes;
    std::vector<uint64_t> xoffs;
    std::vector<int32_t> xerr;
    ~Partition() {
        if (dist) dist_free(dist);
        if (hpin) (void)hipHostFree(hpin);
        if (kstream) keto_stream_destroy(kstream);
        scratch_forget_stream(hs);
        scratch_forget_stream(hs2);
        if (hs) (void)hipStreamDestroy(hs);
        if (hs2) (void)hipStreamDestroy(hs2);
    }
};

void sync(Partition &P) { KETO_HIP(hipStreamSynchronize(P.hs)); }

// the closure's owner-side reads from the resident partition (a job of several ranks)
void snap_source(Partition &P, Lookup &L) {
    if (!P.dist) return;
    const Snapshot &S = dist_snapshot(*P.dist);
    // run_of / tuple_at read all_off[node0 .. node0 + n_slots] as one CSR run, without row_span:
    // only a snapshot no advance ever relocated rows in (partition builds take no room)
    if (S.dev.reloc || S.room.moved || S.room.reloc_cap)
        throw Error(KETO_E_DEVICE, "partition snapshot has advance room: its CSR runs are not contiguous");
    L.use_snap = true;
    L.S = S.dev;
}

uint64_t d2h_u64(Partition &P, const void *d) {
    uint64_t v = 0;
    KETO_HIP(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, P.hs));
    sync(P);
    return v;
}

void coll_check(int rc, const char *what) {
    if (rc != 0) throw Error(KETO_E_DEVICE, std::string("collective ") + what + " failed with " + std::to_string(rc));
}

uint64_t allreduce_max(Partition &P, uint64_t v) {
    if (!P.have_coll || P.world == 1) return v;
    coll_check(P.coll.allreduce_max_u64(P.coll.ctx, &v), "allreduce_max_u64");
    return v;
}

// all-to-all-v of device records grouped by destination (send_cnt[r] records of `rec` bytes
// for rank r): received records land in `dst` (grown), grouped by source; returns per-source
// counts.  With the collective's alltoallv_device the bytes go device to device on the
// partition's stream (RCCL over xGMI); otherwise host-staged, so any collective (gloo, MPI) can
// carry it.
std::vector<uint64_t> exchange(Partition &P, const void *src, const std::vector<uint64_t> &send_cnt, size_t rec,
                               DevBuf &dst, uint64_t &bytes_sent) {
    const uint32_t W = P.world;
    if (!P.have_coll || W == 1) {
        ensure(dst, send_cnt[0] * rec);
        if (send_cnt[0]) KETO_HIP(hipMemcpyAsync(dst.p, src, send_cnt[0] * rec, hipMemcpyDeviceToDevice, P.hs));
        return send_cnt;
    }
    std::vector<uint64_t> recv_cnt(W, 0), sb(W), rb(W);
    coll_check(P.coll.alltoall_u64(P.coll.ctx, send_cnt.data(), recv_cnt.data()), "alltoall_u64");
    uint64_t ns = 0, nr = 0;
    for (uint32_t r = 0; r < W; r++) {
        sb[r] = send_cnt[r] * rec;
        rb[r] = recv_cnt[r] * rec;
        ns += sb[r];
        nr += rb[r];
        if (r != P.rank) bytes_sent += sb[r];
    }
    if (P.coll.alltoallv_device) {
        ensure(dst, nr);
        coll_check(P.coll.alltoallv_device(P.coll.ctx, src, sb.data(), dst.p, rb.data(), P.hs), "alltoallv_device");
        return recv_cnt;
    }
    std::vector<uint8_t> hsend(ns), hrecv(nr);
    if (ns) KETO_HIP(hipMemcpyAsync(hsend.data(), src, ns, hipMemcpyDeviceToHost, P.hs));
    sync(P);
    coll_check(P.coll.alltoallv(P.coll.ctx, hsend.data(), sb.data(), hrecv.data(), rb.data()), "alltoallv");
    ensure(dst, nr);
    if (nr) KETO_HIP(hipMemcpyAsync(dst.p, hrecv.data(), nr, hipMemcpyHostToDevice, P.hs));
    sync(P);
    return recv_cnt;
}

// grow the closure buffer keeping its content (capacity doubles: few copies per batch)
void reserve_closure(Partition &P, uint64_t keep, uint64_t n) {
    const size_t need = std::max<uint64_t>(1, n) * sizeof(keto_tuple);
    if (P.closure.p && P.closure.bytes >= need) return;
    // (KETO_PART_MIN_CLOSURE, tuples: a smaller floor than 64 MB, so tests reach the overflow path)
    static const size_t floor_bytes = getenv("KETO_PART_MIN_CLOSURE")
                                          ? std::max<size_t>(1, strtoull(getenv("KETO_PART_MIN_CLOSURE"), nullptr, 10)) * sizeof(keto_tuple)
                                          : (size_t)64 << 20;
    DevBuf b(std::max<size_t>(need * 2, floor_bytes));
    if (keep) KETO_HIP(hipMemcpyAsync(b.p, P.closure.p, keep * sizeof(keto_tuple), hipMemcpyDeviceToDevice, P.hs));
    P.closure = std::move(b);
}

void ensure_table(Partition &P, uint64_t add) {
    uint64_t cap = P.table_mask + 1;
    if (P.table.p && 2 * (P.n_seen + add) <= cap) return;
    while (2 * (P.n_seen + add) > cap || cap < (1u << 20)) cap *= 2;
    if (cap < 2) cap = 1u << 20;
    ensure(P.table, cap * 8);
    P.table_mask = cap - 1;
    KETO_HIP(hipMemsetAsync(P.table.p, 0, cap * 8, P.hs));
    if (P.n_seen)
        hipLaunchKernelGGL(k_rehash, grid_for(P.n_seen), dim3(BLK), 0, P.hs, dptr<uint64_t>(P.seen), P.n_seen,
                           dptr<unsigned long long>(P.table), P.table_mask);
}

// One rank with a closure buffer from an earlier batch: every level is enqueued at once, its
// kernels reading their counts from the device (no host round trip per level: 3 per level on the
// synchronous path).  Buffers are sized for the worst case the buffer allows -- every candidate
// is a batch key or the subject set of a gathered tuple -- and a closure that outgrows the
// buffer returns UINT64_MAX (the caller reruns the batch's closure on the synchronous path).
uint64_t closure_self(Partition &P, const uint64_t *keys, uint64_t n_keys, bool filter, uint64_t n_subj, int levels,
                      keto_partition_stats &st) {
    using ull = unsigned long long;
    const uint64_t cap = P.closure.bytes / sizeof(keto_tuple);
    P.n_seen = 0;
    ensure_table(P, n_keys + cap);
    KETO_HIP(hipMemsetAsync(P.table.p, 0, (P.table_mask + 1) * 8, P.hs));
    const uint64_t cc = std::max<uint64_t>(1, std::max(n_keys, cap));
    ensure(P.cand, cc * 8);
    ensure(P.fresh, cc * 8);
    // [0] closure total, [1] overflow, [2] level 0's candidates; level L: {new, start, end, next}
    const size_t nb = (3 + 4 * (size_t)levels) * 8;
    ensure(P.lctr, nb);
    ull *c = dptr<ull>(P.lctr), *lv = c + 3;
    KETO_HIP(hipMemsetAsync(c, 0, nb, P.hs));
    const ull nk = n_keys;
    KETO_HIP(hipMemcpyAsync(c + 2, &nk, 8, hipMemcpyHostToDevice, P.hs));
    if (n_keys) KETO_HIP(hipMemcpyAsync(P.cand.p, keys, n_keys * 8, hipMemcpyDeviceToDevice, P.hs));
    Lookup L{dptr<uint64_t>(P.ukeys), dptr<uint64_t>(P.beg), P.m, dptr<uint4>(P.index), P.index_mask,
             dptr<uint2>(P.meta), dptr<uint4>(P.shard), dptr<uint64_t>(P.fresh), dptr<uint64_t>(P.req_off),
             dptr<ull>(P.subj_set), P.subj_mask, dptr<uint32_t>(P.subj_bits), 1u, filter ? 1 : 0};
    snap_source(P, L);
    const dim3 G(std::max(1, num_cus(P.device)) * 8u);
    keto_tuple *cl = dptr<keto_tuple>(P.closure);
    for (int l = 0; l < levels; l++) {
        ull *m = lv + 4 * l;
        const ull *n_cand = l ? lv + 4 * (l - 1) + 3 : c + 2;
        hipLaunchKernelGGL(k_insert, G, dim3(BLK), 0, P.hs, dptr<uint64_t>(P.cand), 0, n_cand, dptr<ull>(P.table),
                           P.table_mask, dptr<uint64_t>(P.fresh), m);
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, P.hs, c, m + 1, (ull)cap);
        hipLaunchKernelGGL(k_lookup_gather, G, dim3(BLK), 0, P.hs, L, 0, m, cl, cap, c, c + 1);
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, P.hs, c, m + 2, (ull)cap);
        hipLaunchKernelGGL(k_next, G, dim3(BLK), 0, P.hs, cl, 0, m + 1, dptr<uint64_t>(P.cand), m + 3);
    }
    KETO_HIP(hipGetLastError());
    std::vector<ull> h(3 + 4 * (size_t)levels);
    KETO_HIP(hipMemcpyAsync(h.data(), c, nb, hipMemcpyDeviceToHost, P.hs));
    sync(P);
    if (h[1]) return UINT64_MAX;
    for (int l = 0; l < levels; l++) {
        const ull nn = h[3 + 4 * l];
        if (!nn) break;
        st.levels++;
        st.objects += nn;
        P.cur_levels.push_back(keto_partition_level{nn, 0, h[3 + 4 * l + 2] - h[3 + 4 * l + 1], 0, 0.0});
    }
    if (P.verbose)
        fprintf(stderr, "[keto partition] one-rank closure: %llu tuples, %llu levels, %llu objects (no per-level sync)\n",
                (ull)h[0], (ull)st.levels, (ull)st.objects);
    return h[0];
}

// Closure of the objects keyed in `keys` (device, n_keys): appended into P.closure, count returned.
// subj (device, sorted unique, n_subj) filters subject-id tuples (Check); null ships everything.
uint64_t closure(Partition &P, const uint64_t *keys, uint64_t n_keys, const uint32_t *subj, uint64_t n_subj,
                 bool filter, keto_partition_stats &st) {
    const uint32_t W = P.world;
    P.cur_levels.clear();
    // every owner gets this rank's subject list once per batch
    std::vector<uint64_t> subj_cnt(W, filter ? n_subj : 0);
    DevBuf &subj_src = P.bsubj_src;
    const void *subj_send = subj;
    if (W > 1) {
        ensure(subj_src, std::max<uint64_t>(1, n_subj) * W * 4);
        if (filter)
            for (uint32_t r = 0; r < W; r++)
                if (n_subj)
                    KETO_HIP(hipMemcpyAsync(dptr<uint32_t>(subj_src) + (uint64_t)r * n_subj, subj, n_subj * 4,
                                            hipMemcpyDeviceToDevice, P.hs));
        subj_send = subj_src.p;
    }
    std::vector<uint64_t> subj_from = exchange(P, subj_send, subj_cnt, 4, P.subj, st.bytes_sent);
    std::vector<uint64_t> soff(W + 1, 0);
    for (uint32_t r = 0; r < W; r++) soff[r + 1] = soff[r] + subj_from[r];
    ensure(P.subj_off, (W + 1) * 8);
    KETO_HIP(hipMemcpyAsync(P.subj_off.p, soff.data(), (W + 1) * 8, hipMemcpyHostToDevice, P.hs));
    // (source, subject) hash set: an owner's filter is one probe per subject-id tuple
    uint64_t scap = 1u << 10;
    while (scap < 2 * std::max<uint64_t>(1, soff[W])) scap *= 2;
    ensure(P.subj_set, scap * 8);
    P.subj_mask = scap - 1;
    KETO_HIP(hipMemsetAsync(P.subj_set.p, 0, scap * 8, P.hs));
    ensure(P.subj_bits, (1u << SUBJ_BITS) / 8);
    KETO_HIP(hipMemsetAsync(P.subj_bits.p, 0, (1u << SUBJ_BITS) / 8, P.hs));
    if (filter && soff[W])
        hipLaunchKernelGGL(k_subj_fill, grid_for(soff[W]), dim3(BLK), 0, P.hs, dptr<uint32_t>(P.subj),
                           dptr<uint64_t>(P.subj_off), W, soff[W], dptr<unsigned long long>(P.subj_set), P.subj_mask,
                           dptr<uint32_t>(P.subj_bits));

    const int levels = P.limits.max_read_depth + 1;
    if (W == 1 && P.closure.p && !getenv("KETO_PART_SYNC_LEVELS")) {
        const uint64_t got = closure_self(P, keys, n_keys, filter, filter ? soff[W] : 0, levels, st);
        if (got != UINT64_MAX) {
            st.tuples = got;
            return got;
        }
        st.levels = 0;  // the buffer was too small: the synchronous levels below grow it
        st.objects = 0;
        P.cur_levels.clear();
    }
    // seen set: fresh per batch
    P.n_seen = 0;
    ensure_table(P, n_keys);
    KETO_HIP(hipMemsetAsync(P.table.p, 0, (P.table_mask + 1) * 8, P.hs));
    ensure(P.ctr, 64);
    ensure(P.cand, std::max<uint64_t>(1, n_keys) * 8);
    KETO_HIP(hipMemcpyAsync(P.cand.p, keys, n_keys * 8, hipMemcpyDeviceToDevice, P.hs));
    uint64_t n_cand = n_keys, total = 0;
    auto tl = std::chrono::steady_clock::now();
    double step_ms[6] = {0, 0, 0, 0, 0, 0};  // verbose: insert, route+exchange, count+scan, fill, next, (spare)
    auto ts = std::chrono::steady_clock::now();
    auto mark = [&](int k) {
        if (!P.verbose) return;
        sync(P);
        const auto now = std::chrono::steady_clock::now();
        step_ms[k] += std::chrono::duration<double, std::milli>(now - ts).count();
        ts = now;
    };
    for (int level = 0; level < levels; level++) {
        const auto lv_t0 = std::chrono::steady_clock::now();
        const uint64_t lv_b0 = st.bytes_sent;
        uint64_t lv_req = 0, lv_new = 0;
        auto end_level = [&](uint64_t n_got) {  // keto_partition_level of this level
            P.cur_levels.push_back(keto_partition_level{
                lv_new, lv_req, n_got, st.bytes_sent - lv_b0 - lv_req,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - lv_t0).count()});
        };
        if (P.verbose) {
            sync(P);
            fprintf(stderr, "[keto partition] level %d: %llu candidates, prev level %.3f ms\n", level,
                    (unsigned long long)n_cand,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count());
            tl = std::chrono::steady_clock::now();
        }
        // new objects of this level: never asked for before (seen-set insert)
        ensure_table(P, n_cand);
        ensure(P.fresh, std::max<uint64_t>(1, n_cand) * 8);
        unsigned long long *c = dptr<unsigned long long>(P.ctr);
        KETO_HIP(hipMemsetAsync(c, 0, 8, P.hs));
        if (n_cand)
            hipLaunchKernelGGL(k_insert, grid_tiles(n_cand), dim3(BLK), 0, P.hs, dptr<uint64_t>(P.cand), n_cand, nullptr,
                               dptr<unsigned long long>(P.table), P.table_mask, dptr<uint64_t>(P.fresh), c);
        const uint64_t n_new = d2h_u64(P, c);
        mark(0);
        if (allreduce_max(P, n_new) == 0) break;
        lv_new = n_new;
        st.levels++;
        st.objects += n_new;
        if (!P.seen.p || P.seen.bytes < (P.n_seen + n_new) * 8) {  // remembered for rehashing
            DevBuf bigger(std::max<uint64_t>(1u << 20, (P.n_seen + n_new) * 16));
            if (P.n_seen) KETO_HIP(hipMemcpyAsync(bigger.p, P.seen.p, P.n_seen * 8, hipMemcpyDeviceToDevice, P.hs));
            P.seen = std::move(bigger);
        }
        if (n_new)
            KETO_HIP(hipMemcpyAsync(dptr<uint64_t>(P.seen) + P.n_seen, P.fresh.p, n_new * 8, hipMemcpyDeviceToDevice,
                                    P.hs));
        P.n_seen += n_new;
        // route the requests to their owners
        std::vector<uint64_t> send(W, 0);
        ensure(P.routed, std::max<uint64_t>(1, n_new) * 8);
        if (W == 1) {
            send[0] = n_new;
            if (n_new) KETO_HIP(hipMemcpyAsync(P.routed.p, P.fresh.p, n_new * 8, hipMemcpyDeviceToDevice, P.hs));
        } else {
            DevBuf &hist = P.bhist;
            ensure(hist, W * 8);
            KETO_HIP(hipMemsetAsync(hist.p, 0, W * 8, P.hs));
            if (n_new)
                hipLaunchKernelGGL(k_dest_hist, grid_for(n_new), dim3(BLK), 0, P.hs, dptr<uint64_t>(P.fresh), n_new,
                                   Dest{W, P.rank, P.place}, dptr<unsigned long long>(hist));
            KETO_HIP(hipMemcpyAsync(send.data(), hist.p, W * 8, hipMemcpyDeviceToHost, P.hs));
            sync(P);
            std::vector<uint64_t> cur(W, 0);
            for (uint32_t r = 1; r < W; r++) cur[r] = cur[r - 1] + send[r - 1];
            KETO_HIP(hipMemcpyAsync(hist.p, cur.data(), W * 8, hipMemcpyHostToDevice, P.hs));
            if (n_new)
                hipLaunchKernelGGL(k_dest_scatter, grid_for(n_new), dim3(BLK), 0, P.hs, dptr<uint64_t>(P.fresh), n_new,
                                   Dest{W, P.rank, P.place}, dptr<unsigned long long>(hist), dptr<uint64_t>(P.routed));
        }
        std::vector<uint64_t> from = exchange(P, P.routed.p, send, 8, P.req, st.bytes_sent);
        lv_req = st.bytes_sent - lv_b0;
        mark(1);
        std::vector<uint64_t> roff(W + 1, 0);
        for (uint32_t r = 0; r < W; r++) roff[r + 1] = roff[r] + from[r];
        const uint64_t n_req = roff[W];
        // owner side: count, scan, fill
        ensure(P.req_off, (W + 1) * 8);
        KETO_HIP(hipMemcpyAsync(P.req_off.p, roff.data(), (W + 1) * 8, hipMemcpyHostToDevice, P.hs));
        Lookup L{dptr<uint64_t>(P.ukeys), dptr<uint64_t>(P.beg), P.m, dptr<uint4>(P.index), P.index_mask,
                 dptr<uint2>(P.meta), dptr<uint4>(P.shard),
                 dptr<uint64_t>(P.req), dptr<uint64_t>(P.req_off), dptr<unsigned long long>(P.subj_set), P.subj_mask,
                 dptr<uint32_t>(P.subj_bits), W, filter ? 1 : 0};
        snap_source(P, L);
        if (W == 1 && P.closure.p) {  // one rank: a single gathering pass into the closure (k_lookup_gather)
            const uint64_t cap = P.closure.bytes / sizeof(keto_tuple) - total;
            unsigned long long *g = dptr<unsigned long long>(P.ctr) + 2;  // [2] total, [3] overflow
            KETO_HIP(hipMemsetAsync(g, 0, 16, P.hs));
            if (n_req)
                hipLaunchKernelGGL(k_lookup_gather, grid_for(n_req), dim3(BLK), 0, P.hs, L, n_req, nullptr,
                                   dptr<keto_tuple>(P.closure) + total, cap, g, g + 1);
            unsigned long long gv[2] = {0, 0};
            KETO_HIP(hipMemcpyAsync(gv, g, 16, hipMemcpyDeviceToHost, P.hs));
            sync(P);
            mark(3);
            if (!gv[1]) {
                const uint64_t n_got = gv[0];
                ensure(P.cand, std::max<uint64_t>(1, n_got) * 8);
                KETO_HIP(hipMemsetAsync(c, 0, 8, P.hs));
                if (n_got)
                    hipLaunchKernelGGL(k_next, grid_tiles(n_got), dim3(BLK), 0, P.hs, dptr<keto_tuple>(P.closure) + total, n_got,
                                       nullptr, dptr<uint64_t>(P.cand), c);
                n_cand = d2h_u64(P, c);
                mark(4);
                total += n_got;
                end_level(n_got);
                continue;
            }
            // overflow: the level again with the two passes (the closure grows to fit)
        }
        // counts, scanned in place into each request's first output position (u32: a level ships
        // fewer than 2^32 tuples -- the compact id pass takes at most 2^31)
        ensure(P.pos, (n_req + 1) * 4);
        uint32_t *posp = dptr<uint32_t>(P.pos);
        KETO_HIP(hipMemsetAsync(posp, 0, (n_req + 1) * 4, P.hs));
        if (n_req) hipLaunchKernelGGL(k_lookup_count, grid_for(n_req), dim3(BLK), 0, P.hs, L, n_req, posp);
        build::scan_excl(posp, n_req, P.hs);
        // tuples per source = pos at the source boundaries
        std::vector<uint32_t> pbv(W + 1, 0);
        for (uint32_t r = 0; r <= W; r++)
            KETO_HIP(hipMemcpyAsync(&pbv[r], posp + roff[r], 4, hipMemcpyDeviceToHost, P.hs));
        sync(P);
        std::vector<uint64_t> pb(pbv.begin(), pbv.end());
        mark(2);
        const uint64_t n_out = pb[W];
        uint64_t n_got = 0;
        if (W == 1) {  // one rank: the owner's gather lands in the closure directly
            reserve_closure(P, total, total + n_out);
            if (n_req)
                hipLaunchKernelGGL(k_lookup_fill, grid_for(n_req), dim3(BLK), 0, P.hs, L, n_req, posp,
                                   dptr<keto_tuple>(P.closure) + total);
            n_got = n_out;
        } else {
            ensure(P.out, std::max<uint64_t>(1, n_out) * sizeof(keto_tuple));
            if (n_req)
                hipLaunchKernelGGL(k_lookup_fill, grid_for(n_req), dim3(BLK), 0, P.hs, L, n_req, posp,
                                   dptr<keto_tuple>(P.out));
            std::vector<uint64_t> back(W);
            for (uint32_t r = 0; r < W; r++) back[r] = pb[r + 1] - pb[r];
            std::vector<uint64_t> recv = exchange(P, P.out.p, back, sizeof(keto_tuple), P.got, st.bytes_sent);
            for (uint64_t v : recv) n_got += v;
            reserve_closure(P, total, total + n_got);
            if (n_got)
                KETO_HIP(hipMemcpyAsync(dptr<keto_tuple>(P.closure) + total, P.got.p, n_got * sizeof(keto_tuple),
                                        hipMemcpyDeviceToDevice, P.hs));
        }
        mark(3);
        // next frontier: the subject sets of the tuples received
        ensure(P.cand, std::max<uint64_t>(1, n_got) * 8);
        KETO_HIP(hipMemsetAsync(c, 0, 8, P.hs));
        if (n_got)
            hipLaunchKernelGGL(k_next, grid_tiles(n_got), dim3(BLK), 0, P.hs, dptr<keto_tuple>(P.closure) + total, n_got, nullptr,
                               dptr<uint64_t>(P.cand), c);
        n_cand = d2h_u64(P, c);
        mark(4);
        total += n_got;
        end_level(n_got);
    }
    sync(P);
    if (P.verbose)
        fprintf(stderr, "[keto partition] steps (ms): insert %.2f, route+exchange %.2f, count+scan %.2f, fill %.2f, next %.2f\n",
                step_ms[0], step_ms[1], step_ms[2], step_ms[3], step_ms[4]);
    st.tuples = total;
    return total;
}

double secs(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
}

}  // namespace

struct PartitionHandle : Partition {};

PartitionHandle *partition_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n,
                                  bool device_ptrs, const keto_collective *coll, const keto_limits *limits, bool force_dist,
                                  const Placement &place) {
    if (!cfg) throw Error(KETO_E_INVALID, "null config");
    if (n && !tuples) throw Error(KETO_E_INVALID, "null tuples");
    if (n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "a partition holds at most 2^31 - 1 tuples");
    if (cfg->n_relations > (1u << ST_REL_BITS) || cfg->n_namespaces > (1u << ST_NS_BITS))
        throw Error(KETO_E_LIMIT, "a partitioned snapshot holds at most 1024 relation names and 2048 namespaces");
    auto P = std::make_unique<PartitionHandle>();
    P->device = cfg->device;
    P->place = place;
    KETO_HIP(hipSetDevice(P->device));
    if (coll) {
        if (coll->world < 1 || (uint32_t)coll->world > MAX_WORLD || coll->rank < 0 || coll->rank >= coll->world)
            throw Error(KETO_E_INVALID, "collective rank / world out of range");
        if ((coll->world > 1 || force_dist) && (!coll->alltoall_u64 || !coll->alltoallv || !coll->allreduce_max_u64))
            throw Error(KETO_E_INVALID, "collective callbacks missing");
        P->have_coll = true;
        P->coll = *coll;
        P->rank = (uint32_t)coll->rank;
        P->world = (uint32_t)coll->world;
    }
    if (limits) P->limits = *limits;
    if (P->limits.max_read_depth < 1 || P->limits.max_read_depth > 65535 || P->limits.max_read_width < 1)
        throw Error(KETO_E_INVALID, "limits out of range");
    for (uint32_t i = 0; i < cfg->n_namespaces; i++)
        P->ns_names.emplace_back(cfg->namespace_names && cfg->namespace_names[i] ? cfg->namespace_names[i] : "");
    for (uint32_t i = 0; i < cfg->n_relations; i++)
        P->rel_names.emplace_back(cfg->relation_names && cfg->relation_names[i] ? cfg->relation_names[i] : "");
    for (auto &s : P->ns_names) P->ns_ptr.push_back(s.c_str());
    for (auto &s : P->rel_names) P->rel_ptr.push_back(s.c_str());
    P->json = cfg->namespaces_json ? cfg->namespaces_json : "";
    P->cfg = *cfg;
    P->cfg.namespace_names = P->ns_ptr.data();
    P->cfg.relation_names = P->rel_ptr.data();
    P->cfg.namespaces_json = P->json.c_str();
    KETO_HIP(hipStreamCreateWithFlags(&P->hs, hipStreamNonBlocking));
    KETO_HIP(hipStreamCreateWithFlags(&P->hs2, hipStreamNonBlocking));
    P->verbose = getenv("KETO_PART_VERBOSE") != nullptr;
    P->trim = getenv("KETO_PART_TRIM") != nullptr;
    if (keto_stream_create(P->device, &P->kstream) != KETO_OK) throw Error(KETO_E_DEVICE, "stream creation failed");
    P->n = n;
    if (force_dist && !P->have_coll) throw Error(KETO_E_INVALID, "KETO_F_PART_DIST needs a collective");
    if ((P->world > 1 || force_dist) && !getenv("KETO_PART_CLOSURE")) {
        // several ranks (or KETO_F_PART_DIST): the partition resident, the distributed frontier over it
        auto t0 = std::chrono::steady_clock::now();
        P->dist = dist_create(&P->cfg, tuples, n, device_ptrs, P->coll, P->limits, P->place);
        if (P->verbose)
            fprintf(stderr, "[keto partition] rank %u: %llu tuples as a resident partition, %.2f s\n", P->rank,
                    (unsigned long long)n, secs(t0));
        return P.release();
    }
    if (P->world == 1 && !getenv("KETO_PART_CLOSURE")) {
        // one rank owns every object: its partition is the whole graph, built once into a
        // resident snapshot (scheduling weights included, as a replica's) that every batch reads
        auto t0 = std::chrono::steady_clock::now();
        P->home.reset(build_snapshot(&P->cfg, tuples, n, device_ptrs));
        if (P->verbose)
            fprintf(stderr, "[keto partition] one rank: %llu tuples as a resident snapshot, %.2f s\n", (unsigned long long)n,
                    secs(t0));
        return P.release();
    }
    ScratchStream on_hs(P->hs);  // (the store is built on P->hs)
    // the partition, grouped by object key (stable radix sort of (key, index), then a gather)
    DevBuf raw;
    const keto_tuple *src = tuples;
    if (!device_ptrs) {
        raw = DevBuf(std::max<uint64_t>(1, n) * sizeof(keto_tuple));
        if (n) KETO_HIP(hipMemcpyAsync(raw.p, tuples, n * sizeof(keto_tuple), hipMemcpyHostToDevice, P->hs));
        src = static_cast<const keto_tuple *>(raw.p);
    }
    Partition &Q = *P;
    DevBuf k0(std::max<uint64_t>(1, n) * 8), k1(std::max<uint64_t>(1, n) * 8), i0(std::max<uint64_t>(1, n) * 4),
        i1(std::max<uint64_t>(1, n) * 4);
    if (n) hipLaunchKernelGGL(k_tuple_keys, grid_for(n), dim3(BLK), 0, Q.hs, src, n, dptr<uint64_t>(k0), dptr<uint32_t>(i0));
    // key = (ns << 32 | obj) << 1 | kind: 33 bits plus the namespace's
    uint32_t ns_bits = 1;
    while ((1u << ns_bits) < cfg->n_namespaces) ns_bits++;
    const bool in1 = prim::sort_pairs(dptr<uint64_t>(k0), dptr<uint32_t>(i0), dptr<uint64_t>(k1), dptr<uint32_t>(i1), n,
                                      33 + ns_bits, Q.hs);
    const uint64_t *kout = in1 ? dptr<uint64_t>(k1) : dptr<uint64_t>(k0);
    const uint32_t *vout = in1 ? dptr<uint32_t>(i1) : dptr<uint32_t>(i0);
    Q.meta = DevBuf(std::max<uint64_t>(1, n) * sizeof(uint2));
    Q.shard = DevBuf(std::max<uint64_t>(1, n) * sizeof(uint4));
    ensure(Q.ctr, 64);
    KETO_HIP(hipMemsetAsync(Q.ctr.p, 0, 8, Q.hs));
    if (n)
        hipLaunchKernelGGL(k_gather_store, grid_for(n), dim3(BLK), 0, Q.hs, src, vout, n, dptr<uint2>(Q.meta),
                           dptr<uint4>(Q.shard), dptr<unsigned long long>(Q.ctr));
    if (d2h_u64(Q, Q.ctr.p)) throw Error(KETO_E_INVALID, "partition tuple with a relation / namespace id past the store's fields");
    raw.reset();
    // runs: one entry per object key (run flags scanned in place into run positions)
    DevBuf fpos(std::max<uint64_t>(1, n + 1) * 4), flag(std::max<uint64_t>(1, n + 1) * 4);
    uint32_t *fl = dptr<uint32_t>(flag), *fp = dptr<uint32_t>(fpos);
    if (n) hipLaunchKernelGGL(k_run_flags, grid_for(n), dim3(BLK), 0, Q.hs, kout, n, fl);
    KETO_HIP(hipMemcpyAsync(fp, fl, n * 4, hipMemcpyDeviceToDevice, Q.hs));
    build::scan_excl(fp, n, Q.hs);
    uint32_t m32 = 0;
    KETO_HIP(hipMemcpyAsync(&m32, fp + n, 4, hipMemcpyDeviceToHost, Q.hs));
    sync(Q);
    Q.m = n ? m32 : 0;
    Q.ukeys = DevBuf(std::max<uint64_t>(1, Q.m) * 8);
    Q.beg = DevBuf((Q.m + 1) * 8);
    if (n)
        hipLaunchKernelGGL(k_run_starts, grid_for(n), dim3(BLK), 0, Q.hs, kout, fl, fp, n, dptr<uint64_t>(Q.ukeys),
                           dptr<uint64_t>(Q.beg));
    KETO_HIP(hipMemcpyAsync(dptr<uint64_t>(Q.beg) + Q.m, &Q.n, 8, hipMemcpyHostToDevice, Q.hs));
    uint64_t cap = 1u << 10;
    while (cap < 2 * Q.m) cap *= 2;
    Q.index = DevBuf(cap * 16);
    Q.index_mask = cap - 1;
    KETO_HIP(hipMemsetAsync(Q.index.p, 0xFF, cap * 16, Q.hs));
    if (Q.m)
        hipLaunchKernelGGL(k_index_fill, grid_for(Q.m), dim3(BLK), 0, Q.hs, dptr<uint64_t>(Q.ukeys), Q.m,
                           dptr<uint4>(Q.index), Q.index_mask);
    KETO_HIP(hipGetLastError());
    sync(Q);
    return P.release();
}

namespace {
// the batch's subject ids (kind 0), sorted and unique, into P.cand-independent storage
uint64_t batch_keys(Partition &P, const keto_query *q, uint64_t n, DevBuf &keys, DevBuf &subj) {
    DevBuf &dq = P.bq, &raw = P.braw, &sorted = P.bsorted;
    ensure(dq, std::max<uint64_t>(1, n) * sizeof(keto_query));
    if (n) KETO_HIP(hipMemcpyAsync(dq.p, q, n * sizeof(keto_query), hipMemcpyHostToDevice, P.hs));
    ensure(keys, std::max<uint64_t>(1, n) * 8);
    ensure(raw, std::max<uint64_t>(1, n) * 4);
    ensure(sorted, std::max<uint64_t>(1, n) * 4);
    ensure(P.braw_v, std::max<uint64_t>(1, n) * 4);
    ensure(P.bsorted_v, std::max<uint64_t>(1, n) * 4);
    ensure(subj, std::max<uint64_t>(1, n) * 4 + 8);
    ensure(P.ctr, 64);
    unsigned long long *c = dptr<unsigned long long>(P.ctr);
    KETO_HIP(hipMemsetAsync(c, 0, 16, P.hs));
    if (n)
        hipLaunchKernelGGL(k_query_keys, grid_tiles(n), dim3(BLK), 0, P.hs, dptr<keto_query>(dq), n, dptr<uint64_t>(keys),
                           dptr<uint32_t>(raw), c);
    const uint64_t ns = d2h_u64(P, c);
    if (!ns) return 0;
    // (the sort carries a payload it ignores: only the keys matter here)
    const bool in1 = prim::sort_pairs(dptr<uint32_t>(raw), dptr<uint32_t>(P.braw_v), dptr<uint32_t>(sorted),
                                      dptr<uint32_t>(P.bsorted_v), ns, 32, P.hs);
    return prim::unique_sorted(in1 ? dptr<uint32_t>(sorted) : dptr<uint32_t>(raw), ns, dptr<uint32_t>(subj), P.hs);
}

// The closure's tuples plus the batch's queries (q, device) or Expand roots (r, device) over the
// compact id space: rewritten in place, P.uniq[local] = global, P.n_local ids.
void remap_ids(Partition &P, keto_tuple *t, uint64_t nt, keto_query *q, keto_subject_set *r, uint64_t n, hipStream_t hs) {
    const uint64_t E = 2 * nt + (q ? 2 * n : n);
    if (E >= (1ull << 31)) throw Error(KETO_E_LIMIT, "closure too large for the compact id pass (2^31 ids)");
    for (DevBuf *b : {&P.rm_ids, &P.rm_pos, &P.rm_ids2, &P.rm_pos2, &P.rm_lid, &P.uniq})
        ensure(*b, std::max<uint64_t>(1, E) * 4);
    ensure(P.rm_flag, (std::max<uint64_t>(1, E) + 1) * 4);
    uint32_t *ids = dptr<uint32_t>(P.rm_ids), *pos = dptr<uint32_t>(P.rm_pos), *ids2 = dptr<uint32_t>(P.rm_ids2),
             *pos2 = dptr<uint32_t>(P.rm_pos2), *fl = dptr<uint32_t>(P.rm_flag), *lid = dptr<uint32_t>(P.rm_lid);
    if (nt) hipLaunchKernelGGL(k_ids_tuples, grid_for(nt), dim3(BLK), 0, hs, t, nt, ids, pos);
    if (n && q) hipLaunchKernelGGL(k_ids_queries, grid_for(n), dim3(BLK), 0, hs, q, n, 2 * nt, ids, pos);
    if (n && r) hipLaunchKernelGGL(k_ids_roots, grid_for(n), dim3(BLK), 0, hs, r, n, 2 * nt, ids, pos);
    P.n_local = 0;
    if (E) {
        uint32_t bits = 1;  // ids are < n_uuids: only their digits are sorted
        while (bits < 32 && (1ull << bits) < (uint64_t)std::max<uint32_t>(2, P.cfg.n_uuids)) bits++;
        const bool in1 = prim::sort_pairs(ids, pos, ids2, pos2, E, bits, hs);
        const uint32_t *sk = in1 ? ids2 : ids, *sp = in1 ? pos2 : pos;
        prim::run_flags(sk, E, fl, hs);
        build::scan_excl(fl, E, hs);
        hipLaunchKernelGGL(k_ids_assign, grid_for(E), dim3(BLK), 0, hs, sk, sp, fl, E, lid, dptr<uint32_t>(P.uniq));
        uint32_t m = 0;
        KETO_HIP(hipMemcpyAsync(&m, fl + E, 4, hipMemcpyDeviceToHost, hs));
        if (nt) hipLaunchKernelGGL(k_apply_tuples, grid_for(nt), dim3(BLK), 0, hs, t, nt, lid);
        if (n && q) hipLaunchKernelGGL(k_apply_queries, grid_for(n), dim3(BLK), 0, hs, q, n, 2 * nt, lid);
        if (n && r) hipLaunchKernelGGL(k_apply_roots, grid_for(n), dim3(BLK), 0, hs, r, n, 2 * nt, lid);
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipStreamSynchronize(hs));
        P.n_local = m;
    }
}

// Processes sharing one device (tests/test_gpu_c5.py: eight ranks on the box's GPU) cannot each keep
// a 2^20-query stream's scratch (frontier arena, DFS tiers: ~7 GB) between batches: with
// KETO_PART_TRIM the stream is recreated after a batch, its scratch allocated again by the next.
void trim_stream(Partition &P) {
    if (!P.trim) return;
    keto_stream_destroy(P.kstream);
    P.kstream = nullptr;
    if (keto_stream_create(P.device, &P.kstream) != KETO_OK) throw Error(KETO_E_DEVICE, "stream creation failed");
}

Snapshot *closure_snapshot(Partition &P, const keto_tuple *t, uint64_t n_tuples) {
    keto_snapshot_config cfg = P.cfg;
    cfg.n_uuids = (uint32_t)std::max<uint64_t>(1, P.n_local);
    return build_snapshot(&cfg, t, n_tuples, true, false);  // (one batch: no weights)
}

void throw_last(int rc) {
    char buf[512];
    keto_last_error(buf, sizeof buf);
    throw Error(rc, buf);
}
}  // namespace

namespace {
// stage 1: the batch's keys, subjects and closure into slot S (the closure functions work on
// P.closure / P.bq, so the slot's buffers are swapped in for the duration)
void stage_closure(Partition &P, Partition::Slot &S, const keto_query *q, uint64_t n) {
    KETO_HIP(hipSetDevice(P.device));
    ScratchStream on_hs(P.hs);  // (the closure's buffers are used on P.hs)
    S.st = keto_partition_stats{};
    S.st.batches = 1;
    std::swap(P.closure, S.closure);
    std::swap(P.bq, S.bq);
    try {
        auto t0 = std::chrono::steady_clock::now();
        DevBuf &keys = P.bkeys, &subj = P.bsubj;
        const uint64_t n_subj = batch_keys(P, q, n, keys, subj);
        if (P.verbose)
            fprintf(stderr, "[keto partition] batch keys + %llu subjects: %.3f ms\n", (unsigned long long)n_subj, secs(t0) * 1e3);
        S.nt = closure(P, dptr<uint64_t>(keys), n, dptr<uint32_t>(subj), n_subj, true, S.st);
        S.st.closure_s = secs(t0);
        S.levels = P.cur_levels;
    } catch (...) {
        std::swap(P.closure, S.closure);
        std::swap(P.bq, S.bq);
        throw;
    }
    std::swap(P.closure, S.closure);
    std::swap(P.bq, S.bq);
}

// stage 2: slot S's closure over the compact id space, its snapshot, the Check kernels, the
// decisions out
void stage_check(Partition &P, Partition::Slot &S, uint64_t n, uint8_t *allowed, int32_t *err, uint32_t flags) {
    KETO_HIP(hipSetDevice(P.device));
    keto_partition_stats &st = S.st;
    auto t0 = std::chrono::steady_clock::now();
    keto_query *dq = dptr<keto_query>(S.bq);  // the batch, uploaded by batch_keys
    {
        ScratchStream on_hs2(P.hs2);  // (the remap's buffers are used on P.hs2; the build below runs on the null stream)
        remap_ids(P, dptr<keto_tuple>(S.closure), S.nt, dq, nullptr, n, P.hs2);
    }
    std::unique_ptr<Snapshot> snap(closure_snapshot(P, dptr<keto_tuple>(S.closure), S.nt));
    st.build_s = secs(t0);
    t0 = std::chrono::steady_clock::now();
    ensure(P.bout, std::max<uint64_t>(1, n) * 8 + 256);
    uint8_t *d_allowed = dptr<uint8_t>(P.bout);
    int32_t *d_err = reinterpret_cast<int32_t *>(dptr<uint8_t>(P.bout) + (n + 255) / 256 * 256);
    const int rc = keto_check_batch(reinterpret_cast<keto_snapshot *>(snap.get()), P.kstream, dq, n, &P.limits, d_allowed,
                                    d_err, KETO_F_DEVICE_PTRS | (flags & (KETO_F_COUNT_WORK | KETO_F_ERR_DETAIL)));
    if (rc != KETO_OK) throw_last(rc);
    if (n) {
        // decisions through pinned staging; the error codes only when a query has one (a 4n-byte
        // pageable copy costs as much as the check kernels' tail)
        const size_t need = (n + 7) / 8 * 8 + 8;
        if (P.hpin_bytes < need) {
            if (P.hpin) KETO_HIP(hipHostFree(P.hpin));
            P.hpin = nullptr;
            P.hpin_bytes = 0;
            KETO_HIP(hipHostMalloc(&P.hpin, need * 2, 0));
            P.hpin_bytes = need * 2;
        }
        uint8_t *hp = static_cast<uint8_t *>(P.hpin);
        ensure(P.ctr2, 64);
        unsigned long long *any = dptr<unsigned long long>(P.ctr2);
        KETO_HIP(hipMemsetAsync(any, 0, 8, P.hs2));
        hipLaunchKernelGGL(k_any_nonzero, grid_for(n), dim3(BLK), 0, P.hs2, d_err, n, any);
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpyAsync(hp, d_allowed, n, hipMemcpyDeviceToHost, P.hs2));
        KETO_HIP(hipMemcpyAsync(hp + need - 8, any, 8, hipMemcpyDeviceToHost, P.hs2));
        KETO_HIP(hipStreamSynchronize(P.hs2));
        std::memcpy(allowed, hp, n);
        unsigned long long has_err = 0;
        std::memcpy(&has_err, hp + need - 8, 8);
        if (has_err) {
            KETO_HIP(hipMemcpyAsync(err, d_err, n * 4, hipMemcpyDeviceToHost, P.hs2));
            KETO_HIP(hipStreamSynchronize(P.hs2));
        } else {
            std::memset(err, 0, n * 4);
        }
    }
    st.run_s = secs(t0);
    if (flags & KETO_F_COUNT_WORK) {
        keto_work_counters wc{};
        if (keto_stream_counters(P.kstream, &wc, 1) == KETO_OK) {
            st.rows = wc.rows[0];
            st.edges = wc.edges[0];
            st.probes = wc.probes[0];
            st.queries = wc.queries[0];
        }
    }
    snap.reset();
    trim_stream(P);
}

// A job of one rank: the batches straight on the resident snapshot, enqueued one after another
// on the engine stream (KETO_F_ASYNC: each batch's H2D / D2H on the stream's copy streams beside
// its neighbours' kernels), one synchronisation at the end.  A counted batch runs synchronously.
void home_check_many(Partition &P, uint32_t nb, const keto_query *const *q, const uint64_t *n, uint8_t *const *allowed,
                     int32_t *const *err, uint32_t flags) {
    auto t0 = std::chrono::steady_clock::now();
    keto_snapshot *snap = reinterpret_cast<keto_snapshot *>(P.home.get());
    const bool count = (flags & KETO_F_COUNT_WORK) != 0;
    const uint32_t f = (flags & (KETO_F_COUNT_WORK | KETO_F_ERR_DETAIL)) | (count ? 0u : KETO_F_ASYNC);
    for (uint32_t k = 0; k < nb; k++) {
        const int rc = keto_check_batch(snap, P.kstream, q[k], n[k], &P.limits, allowed[k], err[k], f);
        if (rc != KETO_OK) {
            // batches 0..k-1 are still queued with the caller's buffers (their H2D reads and D2H
            // writes): they finish before the error goes back and the caller may free them
            char msg[512];
            keto_last_error(msg, sizeof msg);
            (void)keto_stream_sync(P.kstream);
            throw Error(rc, msg);
        }
    }
    const int rc = keto_stream_sync(P.kstream);
    if (rc != KETO_OK) throw_last(rc);
    keto_partition_stats st{};
    st.batches = nb;
    st.run_s = secs(t0) / std::max<uint32_t>(1, nb);
    if (count) {
        keto_work_counters wc{};
        if (keto_stream_counters(P.kstream, &wc, 1) == KETO_OK) {
            st.rows = wc.rows[0];
            st.edges = wc.edges[0];
            st.probes = wc.probes[0];
            st.queries = wc.queries[0];
        }
    }
    P.last = st;
    P.last_levels.clear();
}

// A job of several ranks: each batch through the distributed frontier over the resident
// partitions (frontier_dist.hip), then the queries it routed -- when any rank has some -- through
// the per-batch closure, every rank taking part with its own (possibly none).  A counted batch
// (KETO_F_COUNT_WORK: the DFS interpreter's work counters) runs on the closure path whole.
void dist_check_many(Partition &P, uint32_t nb, const keto_query *const *q, const uint64_t *n, uint8_t *const *allowed,
                     int32_t *const *err, uint32_t flags) {
    const bool count = (flags & KETO_F_COUNT_WORK) != 0;
    for (uint32_t k = 0; k < nb; k++) {
        auto t0 = std::chrono::steady_clock::now();
        keto_partition_stats st{};
        st.batches = 1;
        std::vector<uint32_t> routed;
        if (count) {
            routed.resize(n[k]);
            for (uint64_t i = 0; i < n[k]; i++) routed[i] = (uint32_t)i;
            P.last_levels.clear();
            P.last_gens.clear();
        } else {
            P.last_levels.clear();  // (the closure of the queries it routes, if any: below)
            DistStats ds{};
            dist_check(*P.dist, q[k], n[k], allowed[k], err[k], (flags & KETO_F_ERR_DETAIL) != 0, routed, ds);
            P.dstats = ds;
            st.generations = ds.generations;
            st.goals = ds.goals;
            st.routed = ds.routed;
            st.exchange_bytes = ds.bytes_exchanged;
            st.device_s = ds.device_s;
            st.exchange_s = ds.exchange_s;
            P.last_gens.clear();
            for (const keto_partition_level &l : dist_levels(*P.dist))  // (the engine's per-generation record)
                P.last_gens.push_back(keto_partition_generation{l.objects, l.request_bytes, l.tuples, l.tuple_bytes_sent, l.ms});
        }
        const uint64_t nr = routed.size();
        if (allreduce_max(P, nr) > 0) {
            std::vector<keto_query> sub(std::max<uint64_t>(1, nr));
            for (uint64_t i = 0; i < nr; i++) sub[i] = q[k][routed[i]];
            std::vector<uint8_t> a(std::max<uint64_t>(1, nr));
            std::vector<int32_t> e(std::max<uint64_t>(1, nr));
            Partition::Slot &S = P.slots[0];
            stage_closure(P, S, sub.data(), nr);
            stage_check(P, S, nr, a.data(), e.data(), flags);
            for (uint64_t i = 0; i < nr; i++) {
                allowed[k][routed[i]] = a[i];
                err[k][routed[i]] = e[i];
            }
            st.levels = S.st.levels;
            st.objects = S.st.objects;
            st.tuples = S.st.tuples;
            st.bytes_sent = S.st.bytes_sent;
            st.closure_s = S.st.closure_s;
            st.build_s = S.st.build_s;
            st.rows = S.st.rows;
            st.edges = S.st.edges;
            st.probes = S.st.probes;
            st.queries = S.st.queries;
            P.last_levels = S.levels;
        }
        st.run_s = secs(t0);
        P.last = st;
    }
}
}  // namespace

// Several batches in one call, in flight: while batch k is remapped, built and checked on this
// thread, the closure of batch k+1 -- its query upload included -- runs on a helper thread (its
// own stream; the collective, if any, is called from that thread, one batch after another as on
// every rank).  On one GPU the stages' kernels slow each other (both are random-access bound), so
// the gain is the hidden upload and host work: C3 x10, fresh batches, ~2 % (21.1-21.4 vs 21.5-21.7 ms).
// KETO_PART_SEQUENTIAL runs them one after another.
void partition_check_many(PartitionHandle *PH, uint32_t nb, const keto_query *const *q, const uint64_t *n,
                          uint8_t *const *allowed, int32_t *const *err, uint32_t flags) {
    Partition &P = *PH;
    KETO_HIP(hipSetDevice(P.device));
    if (!nb) return;
    if (P.dist) return dist_check_many(P, nb, q, n, allowed, err, flags);
    if (P.home) return home_check_many(P, nb, q, n, allowed, err, flags);
    if (getenv("KETO_PART_SEQUENTIAL")) {
        for (uint32_t k = 0; k < nb; k++) {
            stage_closure(P, P.slots[0], q[k], n[k]);
            stage_check(P, P.slots[0], n[k], allowed[k], err[k], flags);
            P.last = P.slots[0].st;
            P.last_levels = P.slots[0].levels;
        }
        return;
    }
    stage_closure(P, P.slots[0], q[0], n[0]);
    for (uint32_t k = 0; k < nb; k++) {
        std::exception_ptr ex;
        std::thread next;
        if (k + 1 < nb)
            next = std::thread([&, k] {
                try {
                    stage_closure(P, P.slots[(k + 1) & 1], q[k + 1], n[k + 1]);
                } catch (...) {
                    ex = std::current_exception();
                }
            });
        try {
            stage_check(P, P.slots[k & 1], n[k], allowed[k], err[k], flags);
        } catch (...) {
            if (next.joinable()) next.join();
            throw;
        }
        if (next.joinable()) next.join();
        P.last = P.slots[k & 1].st;
        P.last_levels = P.slots[k & 1].levels;
        if (ex) std::rethrow_exception(ex);
    }
}

void partition_check(PartitionHandle *PH, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, uint32_t flags) {
    partition_check_many(PH, 1, &q, &n, &allowed, &err, flags);
}

namespace {
// keto_expand_batch into P.xnodes / xoffs / xerr (grown until the trees fit)
void expand_into(Partition &P, keto_snapshot *snap, const keto_subject_set *roots, uint64_t n) {
    P.xoffs.assign(n + 1, 0);
    P.xerr.assign(std::max<uint64_t>(1, n), 0);
    if (P.xnodes.empty()) P.xnodes.resize(1u << 16);
    for (;;) {
        const int rc = keto_expand_batch(snap, P.kstream, roots, n, &P.limits, P.xnodes.data(), P.xnodes.size(),
                                         P.xoffs.data(), P.xerr.data());
        if (rc == KETO_E_CAPACITY) {
            P.xnodes.resize(P.xoffs[n]);
            continue;
        }
        if (rc != KETO_OK) throw_last(rc);
        break;
    }
}
}  // namespace

uint64_t partition_expand(PartitionHandle *PH, const keto_subject_set *roots, uint64_t n) {
    Partition &P = *PH;
    KETO_HIP(hipSetDevice(P.device));
    keto_partition_stats st{};
    st.batches = 1;
    auto t0 = std::chrono::steady_clock::now();
    if (P.home) {  // one rank: the resident snapshot
        expand_into(P, reinterpret_cast<keto_snapshot *>(P.home.get()), roots, n);
        st.run_s = secs(t0);
        P.last = st;
        P.last_levels.clear();
        return P.xoffs[n];
    }
    if (P.dist && !getenv("KETO_PART_XCLOSURE")) {  // several ranks: rows fetched from the resident partitions, walked here
        DistExpandStats xs;
        dist_expand(*P.dist, roots, n, P.xnodes, P.xoffs, P.xerr, xs);
        st.levels = xs.levels;
        st.objects = xs.rows;
        st.tuples = xs.entries;
        st.bytes_sent = xs.bytes_sent;
        st.closure_s = xs.fetch_s;
        st.run_s = secs(t0);
        st.exchange_s = xs.exchange_s;
        P.last = st;
        P.last_levels = xs.per_level;
        return P.xoffs[n];
    }
    DevBuf dr(std::max<uint64_t>(1, n) * sizeof(keto_subject_set)), keys(std::max<uint64_t>(1, n) * 8);
    uint64_t nt = 0;
    {
        ScratchStream on_hs(P.hs);  // (the closure's and the remap's buffers are used on P.hs)
        if (n) KETO_HIP(hipMemcpyAsync(dr.p, roots, n * sizeof(keto_subject_set), hipMemcpyHostToDevice, P.hs));
        if (n)
            hipLaunchKernelGGL(k_root_keys, grid_for(n), dim3(BLK), 0, P.hs, dptr<keto_subject_set>(dr), n,
                               dptr<uint64_t>(keys));
        nt = closure(P, dptr<uint64_t>(keys), n, nullptr, 0, false, st);
        st.closure_s = secs(t0);
        t0 = std::chrono::steady_clock::now();
        remap_ids(P, dptr<keto_tuple>(P.closure), nt, nullptr, dptr<keto_subject_set>(dr), n, P.hs);
    }
    std::vector<keto_subject_set> lroots(n);
    if (n) KETO_HIP(hipMemcpy(lroots.data(), dr.p, n * sizeof(keto_subject_set), hipMemcpyDeviceToHost));
    std::vector<uint32_t> uniq(P.n_local);
    if (P.n_local) KETO_HIP(hipMemcpy(uniq.data(), P.uniq.p, P.n_local * 4, hipMemcpyDeviceToHost));
    std::unique_ptr<Snapshot> snap(closure_snapshot(P, dptr<keto_tuple>(P.closure), nt));
    st.build_s = secs(t0);
    t0 = std::chrono::steady_clock::now();
    expand_into(P, reinterpret_cast<keto_snapshot *>(snap.get()), lroots.data(), n);
    for (uint64_t i = 0; i < P.xoffs[n]; i++)  // the trees' subject ids back to the global id space
        if (P.xnodes[i].s_obj < P.n_local) P.xnodes[i].s_obj = uniq[P.xnodes[i].s_obj];
    st.run_s = secs(t0);
    snap.reset();
    trim_stream(P);
    P.last = st;
    P.last_levels = P.cur_levels;
    return P.xoffs[n];
}

void partition_expand_result(PartitionHandle *PH, keto_tree_node *nodes, uint64_t cap, uint64_t *offsets, int32_t *err) {
    Partition &P = *PH;
    const uint64_t n = P.xoffs.empty() ? 0 : P.xoffs.size() - 1;
    const uint64_t total = n ? P.xoffs[n] : 0;
    if (!offsets || (n && !err)) throw Error(KETO_E_INVALID, "null buffer");
    if (total > cap || (total && !nodes)) throw Error(KETO_E_CAPACITY, "expand output needs " + std::to_string(total) + " nodes");
    std::memcpy(offsets, P.xoffs.data(), (n + 1) * 8);
    if (n) std::memcpy(err, P.xerr.data(), n * 4);
    if (total) std::memcpy(nodes, P.xnodes.data(), total * sizeof(keto_tree_node));
}

void partition_stats(PartitionHandle *PH, keto_partition_stats *out) { *out = PH->last; }
void partition_levels(PartitionHandle *PH, keto_partition_level *out, uint32_t cap, uint32_t *n) {
    const auto &L = PH->last_levels;
    *n = (uint32_t)L.size();
    for (uint32_t i = 0; i < cap && i < L.size(); i++) out[i] = L[i];
}
void partition_generations(PartitionHandle *PH, keto_partition_generation *out, uint32_t cap, uint32_t *n) {
    const auto &G = PH->last_gens;
    *n = (uint32_t)G.size();
    for (uint32_t i = 0; i < cap && i < G.size(); i++) out[i] = G[i];
}
void partition_free(PartitionHandle *PH) { delete PH; }

}  // namespace keto
