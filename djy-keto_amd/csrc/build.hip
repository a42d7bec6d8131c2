// gfx950 snapshot builder kernels: relation tuples (uploaded once) -> device CSR snapshot.
//
// A 1B-tuple snapshot (BASELINE config 4) is dominated by random scatters into multi-GB
// arrays: per-node tuple counts, row fills, reverse-row fills, hash inserts.  On the host
// cores those are TLB-miss bound; on the device they are plain HBM atomics.  So the whole
// build runs here as one-thread-per-item kernels (no block-level cooperation, so the CPU
// kernel-debug harness in tools/cpuemu runs the same sources):
//   counting sorts by node / subject with atomic cursors, exclusive scans in three
//   chunked passes, per-row shard-order sorts (one thread per row), a bucketized
//   compare-and-swap hash for heavy subjects' membership probes.
// Row order is ORDER BY shard_id (big-endian UUID bytes; traverser.go:88,
// relationtuples.go:216), ties broken by tuple index: fully deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "device_common.hpp"

namespace keto {
namespace build {
namespace {

constexpr uint32_t BLK = 256;
constexpr uint32_t SCAN_TILE = 4096;  // elements per block of the scan
constexpr uint32_t SCAN_RUN = 16;     // consecutive elements per thread
constexpr uint32_t FLAG_GRID = 1024;  // blocks of the flag-marking kernels (one flush per block)
constexpr uint32_t LDS_FLAGS = 2048;  // flags deduplicated in LDS before the global stores

inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, (n + BLK - 1) / BLK)); }
inline dim3 grid_cap(uint64_t n, uint32_t cap) { return dim3((uint32_t)std::min<uint64_t>(grid_for(n).x, cap)); }

__device__ __forceinline__ uint64_t gid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }

__device__ __forceinline__ uint64_t shard_hi(const keto_tuple &t) {
    uint64_t h = 0;
    for (int k = 0; k < 8; k++) h = (h << 8) | t.shard_id[k];
    return h;
}
__device__ __forceinline__ uint64_t shard_lo(const keto_tuple &t) {
    uint64_t h = 0;
    for (int k = 8; k < 16; k++) h = (h << 8) | t.shard_id[k];
    return h;
}

// ---------------------------------------------------------------- block helpers
// Written against blockDim.x (not BLK) so the CPU emulation (one thread per block) runs them.
// Block sum of one value per thread (power-of-two blockDim); every thread gets the total.
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t s = blockDim.x >> 1; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    const uint32_t t = red[0];
    __syncthreads();
    return t;
}
// Block exclusive scan of one value per thread (Hillis-Steele in LDS); *total = the block's sum.
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *buf, uint32_t *total) {
    buf[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
        const uint32_t y = threadIdx.x >= off ? buf[threadIdx.x - off] : 0u;
        __syncthreads();
        buf[threadIdx.x] += y;
        __syncthreads();
    }
    const uint32_t incl = buf[threadIdx.x];
    *total = buf[blockDim.x - 1];
    __syncthreads();
    return incl - v;
}
// Lanes of a wave adding to the same counter in adjacent lanes (tuples of one row arrive
// together) take one atomic per run instead of one each: returns the lane's old value.  Lanes
// with !active neither add nor break the result of others.  Active lanes must be a prefix of the
// wave (the grid's tail): the last run ends at the last active lane.
__device__ __forceinline__ uint32_t run_atomic_inc(uint32_t *arr, uint32_t key, bool active) {
    const uint32_t lane = __lane_id();
    const uint32_t k = active ? key : NONE32;
    const uint32_t prev = __shfl_up(k, 1);
    const bool head = active && (lane == 0 || prev != k);
    const unsigned long long heads = __ballot(head), live = __ballot(active);
    const unsigned long long below = heads & ((2ull << lane) - 1ull);  // heads at or before this lane
    const uint32_t h = below ? 63u - (uint32_t)__clzll((long long)below) : 0u;
    const unsigned long long after = heads & ~((2ull << lane) - 1ull);
    const uint32_t width = 64u - (uint32_t)__clzll((long long)live);
    const uint32_t next = after ? (uint32_t)__ffsll((long long)after) - 1u : width;
    uint32_t base = 0;
    if (head) base = atomicAdd(&arr[key], next - lane);
    base = __shfl(base, (int)h);
    return base + (lane - h);
}
// the same for OR-ing bit masks into words (entity bits)
__device__ __forceinline__ void run_atomic_or(unsigned long long *arr, uint64_t word, unsigned long long m, bool active) {
    const uint32_t lane = __lane_id();
    const uint64_t w = active ? word : ~0ull;
    unsigned long long x = active ? m : 0ull;
    for (uint32_t off = 1; off < 64; off <<= 1) {  // OR of the lanes at distance < 2*off with the same word
        const unsigned long long y = __shfl_down(x, off);
        const uint64_t wy = __shfl_down(w, off);
        if (lane + off < 64 && wy == w) x |= y;
    }
    const uint64_t pw = __shfl_up(w, 1);  // (every lane shuffles: a lane left out of a shuffle reads as 0)
    const bool head = active && (lane == 0 || pw != w);
    if (head && (arr[w] & x) != x) atomicOr(&arr[w], x);
}

// ---------------------------------------------------------------- exclusive scan (u32)
// Tile c = [c * SCAN_TILE, (c + 1) * SCAN_TILE): coalesced sums, then a carried block scan in
// runs of SCAN_RUN consecutive elements per thread.
__global__ __launch_bounds__(BLK) void k_tile_sum(const uint32_t *v, uint64_t n, uint32_t *sums, uint64_t nt) {
    __shared__ uint32_t red[BLK];
    const uint64_t c = blockIdx.x;
    if (c >= nt) return;
    const uint64_t b = c * SCAN_TILE, e = std::min<uint64_t>(n, b + SCAN_TILE);
    uint32_t acc = 0;
    for (uint64_t i = b + threadIdx.x; i < e; i += blockDim.x) acc += v[i];
    const uint32_t t = block_sum(acc, red);
    if (threadIdx.x == 0) sums[c] = t;
}
// v[i] -> carry(c) + exclusive prefix within the tile; the last tile also writes v[n] = total
__global__ __launch_bounds__(BLK) void k_tile_apply(uint32_t *v, uint64_t n, const uint32_t *sums, uint64_t nt) {
    __shared__ uint32_t buf[BLK];
    const uint64_t c = blockIdx.x;
    if (c >= nt) return;
    const uint64_t b = c * SCAN_TILE, e = std::min<uint64_t>(n, b + SCAN_TILE);
    uint32_t carry = sums ? sums[c] : 0u;
    for (uint64_t r = b; r < e; r += (uint64_t)blockDim.x * SCAN_RUN) {
        const uint64_t i0 = r + (uint64_t)threadIdx.x * SCAN_RUN;
        uint32_t x[SCAN_RUN], acc = 0;
        for (uint32_t k = 0; k < SCAN_RUN; k++) {
            x[k] = i0 + k < e ? v[i0 + k] : 0u;
            acc += x[k];
        }
        uint32_t tot = 0;
        uint32_t o = carry + block_excl(acc, buf, &tot);
        for (uint32_t k = 0; k < SCAN_RUN; k++)
            if (i0 + k < e) {
                v[i0 + k] = o;
                o += x[k];
            }
        carry += tot;
    }
    if (c == nt - 1 && threadIdx.x == 0) v[n] = carry;
}

// ---------------------------------------------------------------- tuples
struct Limits {
    uint32_t n_ns, n_rel_caller, n_uuids, n_rel;
};

// flags marked by many threads (a handful of (namespace, relation) pairs / slots): deduplicated
// in the block's LDS when there are at most LDS_FLAGS of them, stored once per block at the end
struct BlockFlags {
    uint32_t *lds;
    uint32_t *g;
    uint32_t n;
    __device__ __forceinline__ void begin() {
        if (n <= LDS_FLAGS) {
            for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) lds[t] = 0;
            __syncthreads();
        }
    }
    __device__ __forceinline__ void set(uint32_t f) {
        if (n <= LDS_FLAGS) lds[f] = 1;
        else if (!g[f]) atomicOr(&g[f], 1u);
    }
    __device__ __forceinline__ void end() {
        if (n > LDS_FLAGS) return;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < n; t += blockDim.x)
            if (lds[t] && !g[t]) g[t] = 1;
    }
};
__global__ __launch_bounds__(BLK) void k_validate(const keto_tuple *t, uint64_t n, Limits L, uint32_t *used, uint32_t n_used,
                                                  unsigned long long *bad) {
    __shared__ uint32_t lf[LDS_FLAGS];
    BlockFlags F{lf, used, n_used};
    F.begin();
    for (uint64_t i = gid(); i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const keto_tuple x = t[i];
        if (x.ns >= L.n_ns || x.rel >= L.n_rel_caller || x.obj >= L.n_uuids || x.s_obj >= L.n_uuids || x.subj_kind > 1 ||
            (x.subj_kind == 1 && (x.s_ns >= L.n_ns || x.s_rel >= L.n_rel_caller))) {
            atomicMin(bad, (unsigned long long)i);
            continue;
        }
        F.set(x.ns * L.n_rel + x.rel);
        if (x.subj_kind == 1) F.set(x.s_ns * L.n_rel + x.s_rel);
    }
    F.end();
}

// a partitioned graph's snapshot (Ghosts::world > 1): a subject-set object another rank owns is
// an entity of the ghost namespace n_ns + s_ns (keto_object_owner)
struct Ghosts {
    uint32_t n_ns, rank, world;
    Placement pl;
    __device__ __forceinline__ uint32_t ns_of_set(uint32_t s_ns, uint32_t s_obj) const {
        if (world <= 1) return s_ns;
        const uint32_t o = place_owner(pl, s_ns, s_obj, world);
        return o == rank || o == PLACE_ALL ? s_ns : n_ns + s_ns;
    }
};
__global__ __launch_bounds__(BLK) void k_entity_bits(const keto_tuple *t, uint64_t n, uint64_t stride,
                                                     unsigned long long *bits, Ghosts G) {
    const uint64_t i = gid();
    const bool in = i < n;
    const keto_tuple x = in ? t[i] : keto_tuple{};
    const uint64_t ck = x.ns * stride + x.obj;
    run_atomic_or(bits, ck >> 6, 1ull << (ck & 63), in);
    const uint64_t cs = (uint64_t)(in && x.subj_kind == 1 ? G.ns_of_set(x.s_ns, x.s_obj) : 0u) * stride + x.s_obj;
    run_atomic_or(bits, cs >> 6, 1ull << (cs & 63), in && x.subj_kind == 1);
}
__global__ __launch_bounds__(BLK) void k_popc(const unsigned long long *bits, uint64_t nblk, uint32_t *cnt) {
    const uint64_t i = gid();
    if (i < nblk) cnt[i] = (uint32_t)__popcll(bits[i]);
}
// global set-bit rank -> entity id of each block's first set bit
__global__ __launch_bounds__(BLK) void k_rank_fix(uint32_t *rank, uint64_t nblk, uint64_t bpn, const uint32_t *ent_base,
                                                  const uint32_t *rank0) {
    const uint64_t i = gid();
    if (i >= nblk) return;
    const uint64_t ns = i / bpn;
    rank[i] = ent_base[ns] + (rank[i] - rank0[ns]);
}
__global__ __launch_bounds__(BLK) void k_ent_obj(const unsigned long long *bits, const uint32_t *rank, uint64_t nblk,
                                                 uint64_t bpn, uint64_t stride, uint32_t *ent_obj) {
    const uint64_t i = gid();
    if (i >= nblk) return;
    unsigned long long m = bits[i];
    uint32_t r = rank[i];
    const uint64_t base = i * 64 - (i / bpn) * stride;
    while (m) {
        const int j = __ffsll((long long)m) - 1;
        m &= m - 1;
        ent_obj[r++] = (uint32_t)(base + j);
    }
}
__global__ __launch_bounds__(BLK) void k_ent_table(const unsigned long long *bits, const uint32_t *rank, uint64_t nblk,
                                                   uint4 *out) {
    const uint64_t i = gid();
    if (i < nblk) out[i] = make_uint4((uint32_t)bits[i], (uint32_t)(bits[i] >> 32), rank[i], 0);
}

struct NodeMap {
    const unsigned long long *bits;
    const uint32_t *rank;
    const NsDev *ns;
    const uint32_t *slot_of;  // [ns table entries * n_rel]
    uint64_t stride;
    uint32_t n_rel, n_uuids;
    Ghosts G;
};
__device__ __forceinline__ uint32_t node_of(const NodeMap &M, uint32_t ns, uint32_t obj, uint32_t rel) {
    const uint64_t ck = ns * M.stride + obj;
    const unsigned long long m = M.bits[ck >> 6];
    const uint32_t e = M.rank[ck >> 6] + (uint32_t)__popcll(m & ((1ull << (ck & 63)) - 1ull));
    const NsDev nd = M.ns[ns];
    return nd.node_base + (e - nd.ent_base) * nd.n_slots + M.slot_of[(size_t)ns * M.n_rel + rel];
}
// row node, subject (node or uuid), shard key; tuple counts per row node and per subject
__global__ __launch_bounds__(BLK) void k_src_dst(const keto_tuple *t, uint64_t n, NodeMap M, uint32_t *src, uint32_t *dst,
                                                 unsigned long long *skey, uint32_t *all_cnt, uint32_t *rev_cnt) {
    const uint64_t i = gid();
    const bool in = i < n;
    uint32_t s = 0;
    if (in) {
        const keto_tuple x = t[i];
        s = node_of(M, x.ns, x.obj, x.rel);
        const uint32_t d = x.subj_kind == 1 ? node_of(M, M.G.ns_of_set(x.s_ns, x.s_obj), x.s_obj, x.s_rel) : x.s_obj;
        src[i] = s;
        dst[i] = x.subj_kind == 1 ? (d | SKEY_SET) : d;
        skey[i] = shard_hi(x);
        atomicAdd(&rev_cnt[x.subj_kind == 1 ? M.n_uuids + d : d], 1u);
    }
    (void)run_atomic_inc(all_cnt, s, in);  // a row's tuples mostly arrive together
}

__global__ __launch_bounds__(BLK) void k_scatter_rows(const uint32_t *src, uint64_t n, uint32_t *cur, uint32_t *row_idx) {
    const uint64_t i = gid();
    const bool in = i < n;
    const uint32_t p = run_atomic_inc(cur, in ? src[i] : 0u, in);
    if (in) row_idx[p] = (uint32_t)i;
}

// shard order within one row: (shard_hi, shard_lo, tuple index)
struct RowLess {
    const keto_tuple *t;
    const unsigned long long *skey;
    __device__ __forceinline__ bool operator()(uint32_t a, uint32_t b) const {
        const unsigned long long ka = skey[a], kb = skey[b];
        if (ka != kb) return ka < kb;
        const uint64_t la = shard_lo(t[a]), lb = shard_lo(t[b]);
        return la != lb ? la < lb : a < b;
    }
};
constexpr uint32_t ROW_SORT_MAX = 1u << 12;  // longer rows are sorted on the host
__device__ void sift(uint32_t *a, uint32_t root, uint32_t len, const RowLess &lt) {
    while (true) {
        uint32_t c = 2 * root + 1;
        if (c >= len) return;
        if (c + 1 < len && lt(a[c], a[c + 1])) c++;
        if (!lt(a[root], a[c])) return;
        const uint32_t tmp = a[root];
        a[root] = a[c];
        a[c] = tmp;
        root = c;
    }
}
__global__ __launch_bounds__(BLK) void k_sort_rows(const uint32_t *off, uint64_t n_rows, uint32_t *row_idx, RowLess lt,
                                                   uint32_t *long_rows, uint32_t *n_long) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    uint32_t *a = row_idx + off[v];
    const uint32_t len = off[v + 1] - off[v];
    if (len < 2) return;
    if (len > ROW_SORT_MAX) {
        long_rows[atomicAdd(n_long, 1u)] = (uint32_t)v;
        return;
    }
    if (len <= 16) {  // insertion sort
        for (uint32_t i = 1; i < len; i++) {
            const uint32_t x = a[i];
            uint32_t j = i;
            while (j > 0 && lt(x, a[j - 1])) {
                a[j] = a[j - 1];
                j--;
            }
            a[j] = x;
        }
        return;
    }
    for (uint32_t r = len / 2; r-- > 0;) sift(a, r, len, lt);  // heap sort
    for (uint32_t e = len - 1; e > 0; e--) {
        const uint32_t tmp = a[0];
        a[0] = a[e];
        a[e] = tmp;
        sift(a, 0, e, lt);
    }
}

__global__ __launch_bounds__(BLK) void k_gather(const keto_tuple *t, const uint32_t *idx, uint64_t n, keto_tuple *out) {
    const uint64_t i = gid();
    if (i < n) out[i] = t[idx[i]];
}

__global__ __launch_bounds__(BLK) void k_row_fill(const uint32_t *off, uint64_t n_rows, const uint32_t *row_idx,
                                                  const uint32_t *dst, uint32_t *all_subj, uint32_t *set_cnt,
                                                  const unsigned long long *skey, unsigned long long *all_shard) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    uint32_t c = 0;
    for (uint32_t p = off[v]; p < off[v + 1]; p++) {
        const uint32_t d = dst[row_idx[p]];
        all_subj[p] = d;
        if (all_shard) all_shard[p] = skey[row_idx[p]];
        c += (d & SKEY_SET) ? 1 : 0;
    }
    set_cnt[v] = c;
}
__global__ __launch_bounds__(BLK) void k_set_fill(const uint32_t *all_off, const uint32_t *set_off, uint64_t n_rows,
                                                  const uint32_t *all_subj, uint32_t *set_dst) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    uint32_t o = set_off[v];
    for (uint32_t p = all_off[v]; p < all_off[v + 1]; p++)
        if (all_subj[p] & SKEY_SET) set_dst[o++] = all_subj[p] & ~SKEY_SET;
}
// row descriptor {begin, end, first edge, second edge} (edges NONE32 past the end): rows of
// <= 2 subject sets -- TTU parents, most ACL and group rows -- need no edge load at all
__global__ __launch_bounds__(BLK) void k_set_row(const uint32_t *set_off, uint64_t n_rows, const uint32_t *set_dst,
                                                 uint4 *set_row) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    const uint32_t b = set_off[v], e = set_off[v + 1];
    set_row[v] = make_uint4(b, e, e > b ? set_dst[b] : NONE32, e > b + 1 ? set_dst[b + 1] : NONE32);
}
__global__ __launch_bounds__(BLK) void k_row_inline(uint4 *set_row, uint64_t n_rows, const uint32_t *set_dst) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    uint4 r = set_row[v];
    r.z = r.y > r.x ? set_dst[r.x] : NONE32;
    r.w = r.y > r.x + 1 ? set_dst[r.x + 1] : NONE32;
    set_row[v] = r;
}

// ---------------------------------------------------------------- reverse rows + probe hash
__global__ __launch_bounds__(BLK) void k_heavy_count(const uint32_t *rev_off, uint64_t n_subj, unsigned long long *heavy) {
    __shared__ uint32_t red[BLK];
    uint32_t acc = 0;  // (a block's heavy tuples fit: < 2^32 tuples in all)
    for (uint64_t v = gid(); v < n_subj; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t len = rev_off[v + 1] - rev_off[v];
        if (len > PROBE_K) acc += len;
    }
    const uint32_t t = block_sum(acc, red);
    if (threadIdx.x == 0 && t) atomicAdd(heavy, (unsigned long long)t);
}
__global__ __launch_bounds__(BLK) void k_scatter_rev(const uint32_t *src, const uint32_t *dst, uint64_t n, uint32_t n_uuids,
                                                     const uint32_t *rev_off, uint32_t *cur, uint32_t *rev_nodes,
                                                     unsigned long long *probe, uint64_t bmask) {
    const uint64_t i = gid();
    if (i >= n) return;
    const uint32_t d = dst[i];
    const uint64_t v = (d & SKEY_SET) ? (uint64_t)n_uuids + (d & ~SKEY_SET) : d;
    rev_nodes[atomicAdd(&cur[v], 1u)] = src[i];
    if (rev_off[v + 1] - rev_off[v] <= PROBE_K) return;
    // heavy subject: membership key into 16-byte buckets of two keys, linear probing
    const unsigned long long key = ((v << 32) | src[i]) + 1;
    uint64_t b = mix64(key) & bmask;
    while (true) {
        for (int k = 0; k < 2; k++) {
            const unsigned long long old = atomicCAS(&probe[2 * b + k], 0ull, key);
            if (old == 0 || old == key) return;  // inserted, or a duplicate tuple's key
        }
        b = (b + 1) & bmask;
    }
}

// ---------------------------------------------------------------- scheduling weights
__global__ __launch_bounds__(BLK) void k_weight(const uint32_t *set_off, const uint32_t *set_dst, uint64_t n_rows,
                                                const uint32_t *w, uint32_t *nw, uint32_t *changed) {
    const uint64_t v = gid();
    if (v >= n_rows) return;
    uint64_t acc = 1;
    for (uint32_t i = set_off[v]; i < set_off[v + 1] && acc < WEIGHT_CAP; i++) acc += w[set_dst[i] & ~EDGE_ALIAS];
    const uint32_t r = (uint32_t)std::min<uint64_t>(acc, WEIGHT_CAP);
    nw[v] = r;
    if (r != w[v]) *changed = 1;
}
// global slots whose rows hold a subject set somewhere (relinfo RI_SETROWS)
__global__ __launch_bounds__(BLK) void k_slot_setrows(const uint4 *set_row, uint64_t n_rows, const NsDev *ns, uint32_t n_ns,
                                                      uint32_t *flag, uint32_t n_flags) {
    __shared__ uint32_t lf[LDS_FLAGS];
    BlockFlags F{lf, flag, n_flags};
    F.begin();
    for (uint64_t i = gid(); i < n_rows; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 r = set_row[i];
        if (r.x == r.y) continue;
        uint32_t lo = 0, hi = n_ns;  // last namespace whose node_base <= i
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (ns[m].node_base <= i) lo = m;
            else hi = m;
        }
        F.set(ns[lo].slot_base + (uint32_t)((i - ns[lo].node_base) % ns[lo].n_slots));
    }
    F.end();
}

// slots holding a subject-id tuple: a direct check of any other slot against a subject id fails
__global__ __launch_bounds__(BLK) void k_slot_idrows(const keto_tuple *t, uint64_t n, const uint32_t *slot_of,
                                                     uint32_t n_rel, const NsDev *ns, uint32_t *flag, uint32_t n_flags) {
    __shared__ uint32_t lf[LDS_FLAGS];
    BlockFlags F{lf, flag, n_flags};
    F.begin();
    for (uint64_t i = gid(); i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (t[i].subj_kind != 0) continue;
        const uint32_t k = slot_of[(size_t)t[i].ns * n_rel + t[i].rel];
        if (k != NO_SLOT) F.set(ns[t[i].ns].slot_base + k);
    }
    F.end();
}

__global__ __launch_bounds__(BLK) void k_fill32(uint32_t *a, uint64_t n, uint32_t x) {
    const uint64_t i = gid();
    if (i < n) a[i] = x;
}
__global__ __launch_bounds__(BLK) void k_alias_mark(uint32_t *set_dst, uint64_t n, const uint32_t *vkey) {
    const uint64_t i = gid();
    if (i < n && vkey[set_dst[i]] != set_dst[i]) set_dst[i] |= EDGE_ALIAS;
}

// a ghost child (another rank's object) is a remote edge
__global__ __launch_bounds__(BLK) void k_remote_mark(uint32_t *set_dst, uint64_t n, uint32_t n_owned) {
    const uint64_t i = gid();
    if (i >= n) return;
    if ((set_dst[i] & ~(EDGE_ALIAS | EDGE_REMOTE)) >= n_owned) set_dst[i] |= EDGE_REMOTE;
}
__global__ __launch_bounds__(BLK) void k_leaf_mark(uint32_t *set_dst, uint64_t n, const uint4 *set_row) {
    const uint64_t i = gid();
    if (i >= n) return;
    const uint32_t c = set_dst[i] & ~(EDGE_ALIAS | EDGE_LEAF);
    const uint4 r = set_row[c];
    if (r.x == r.y) set_dst[i] |= EDGE_LEAF;
}
}  // namespace

// ---------------------------------------------------------------- host side
DevBuf::DevBuf(size_t b) : bytes(b) { p = scratch_get(std::max<size_t>(bytes, 16) + 16, &cap); }
DevBuf::~DevBuf() { scratch_put(p, cap); }
DevBuf::DevBuf(DevBuf &&o) noexcept : p(o.p), bytes(o.bytes), cap(o.cap) { o.p = nullptr; }
DevBuf &DevBuf::operator=(DevBuf &&o) noexcept {
    if (this != &o) {
        reset();
        p = o.p;
        bytes = o.bytes;
        cap = o.cap;
        o.p = nullptr;
    }
    return *this;
}
void DevBuf::reset() {
    scratch_put(p, cap);
    p = nullptr;
    bytes = cap = 0;
}
void *DevBuf::release() {
    void *q = p;
    p = nullptr;
    return q;
}

void scan_excl(uint32_t *v, uint64_t n, hipStream_t s) {
    const uint64_t nt = std::max<uint64_t>(1, (n + SCAN_TILE - 1) / SCAN_TILE);
    if (nt == 1) {
        hipLaunchKernelGGL(k_tile_apply, dim3(1), dim3(BLK), 0, s, v, n, nullptr, 1);
        KETO_HIP(hipGetLastError());
        return;
    }
    DevBuf sums(4 * (nt + 1));
    hipLaunchKernelGGL(k_tile_sum, dim3((uint32_t)nt), dim3(BLK), 0, s, v, n, sums.u32(), nt);
    KETO_HIP(hipGetLastError());
    scan_excl(sums.u32(), nt, s);
    hipLaunchKernelGGL(k_tile_apply, dim3((uint32_t)nt), dim3(BLK), 0, s, v, n, sums.u32(), nt);
    KETO_HIP(hipGetLastError());
}

uint32_t read_u32(const uint32_t *d, uint64_t i) {
    uint32_t x = 0;
    KETO_HIP(hipMemcpy(&x, d + i, 4, hipMemcpyDeviceToHost));
    return x;
}

void validate(const keto_tuple *t, uint64_t n, uint32_t n_ns, uint32_t n_rel_caller, uint32_t n_uuids, uint32_t n_rel,
              uint32_t *used, unsigned long long *bad) {
    hipLaunchKernelGGL(k_validate, grid_cap(n, FLAG_GRID), dim3(BLK), 0, 0, t, n, Limits{n_ns, n_rel_caller, n_uuids, n_rel}, used,
                       n_ns * n_rel, bad);
    KETO_HIP(hipGetLastError());
}

void entity_bits(const keto_tuple *t, uint64_t n, uint64_t stride, unsigned long long *bits, uint64_t nblk,
                 uint32_t *rank, uint32_t n_ns, uint32_t part_rank, uint32_t part_world, const Placement &place) {
    hipLaunchKernelGGL(k_entity_bits, grid_for(n), dim3(BLK), 0, 0, t, n, stride, bits, Ghosts{n_ns, part_rank, part_world, place});
    hipLaunchKernelGGL(k_popc, grid_for(nblk), dim3(BLK), 0, 0, bits, nblk, rank);
    KETO_HIP(hipGetLastError());
    scan_excl(rank, nblk);
}

void entity_ids(const unsigned long long *bits, uint32_t *rank, uint64_t nblk, uint64_t bpn, uint64_t stride,
                const uint32_t *ent_base, const uint32_t *rank0, uint32_t *ent_obj, uint4 *table) {
    hipLaunchKernelGGL(k_rank_fix, grid_for(nblk), dim3(BLK), 0, 0, rank, nblk, bpn, ent_base, rank0);
    hipLaunchKernelGGL(k_ent_obj, grid_for(nblk), dim3(BLK), 0, 0, bits, rank, nblk, bpn, stride, ent_obj);
    hipLaunchKernelGGL(k_ent_table, grid_for(nblk), dim3(BLK), 0, 0, bits, rank, nblk, table);
    KETO_HIP(hipGetLastError());
}

void rows(const RowsIn &in, RowsOut &out) {
    const uint64_t n = in.n, N = in.n_nodes, M = in.n_subj;
    static const bool verbose = getenv("KETO_BUILD_VERBOSE") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto step = [&](const char *what) {
        if (!verbose) return;
        KETO_HIP(hipStreamSynchronize(nullptr));
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto build]   rows/%-12s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    NodeMap map{in.bits, in.rank, in.ns, in.slot_of, in.stride, in.n_rel, in.n_uuids, Ghosts{in.n_ns, in.part_rank, in.part_world, in.place}};
    DevBuf src(4 * n), dst(4 * n), skey(8 * n);
    KETO_HIP(hipMemset(out.all_off, 0, 4 * (N + 1)));
    KETO_HIP(hipMemset(out.rev_off, 0, 4 * (M + 1)));
    hipLaunchKernelGGL(k_src_dst, grid_for(n), dim3(BLK), 0, 0, in.tuples, n, map, src.u32(), dst.u32(),
                       reinterpret_cast<unsigned long long *>(skey.p), out.all_off, out.rev_off);
    KETO_HIP(hipGetLastError());
    scan_excl(out.all_off, N);
    scan_excl(out.rev_off, M);
    step("count+scan");
    // tuples of each row node, in shard order
    DevBuf row_idx(4 * n);
    {
        DevBuf cur(4 * (N + 1));
        KETO_HIP(hipMemcpy(cur.p, out.all_off, 4 * (N + 1), hipMemcpyDeviceToDevice));
        hipLaunchKernelGGL(k_scatter_rows, grid_for(n), dim3(BLK), 0, 0, src.u32(), n, cur.u32(), row_idx.u32());
        KETO_HIP(hipGetLastError());
    }
    step("scatter");
    {
        DevBuf longs(4 * (n / ROW_SORT_MAX + 2)), n_long(4);
        KETO_HIP(hipMemset(n_long.p, 0, 4));
        RowLess lt{in.tuples, reinterpret_cast<const unsigned long long *>(skey.p)};
        hipLaunchKernelGGL(k_sort_rows, grid_for(N), dim3(BLK), 0, 0, out.all_off, N, row_idx.u32(), lt, longs.u32(),
                           n_long.u32());
        KETO_HIP(hipGetLastError());
        const uint32_t nl = read_u32(n_long.u32(), 0);
        if (nl) {  // rare very long rows: sorted on the host from the caller's tuples
            std::vector<uint32_t> lv(nl), seg;
            KETO_HIP(hipMemcpy(lv.data(), longs.p, 4ull * nl, hipMemcpyDeviceToHost));
            for (uint32_t v : lv) {
                const uint32_t b = read_u32(out.all_off, v), e = read_u32(out.all_off, v + 1);
                seg.resize(e - b);
                KETO_HIP(hipMemcpy(seg.data(), row_idx.u32() + b, 4ull * (e - b), hipMemcpyDeviceToHost));
                std::vector<keto_tuple> rec;
                if (!in.host_tuples) {  // device-resident tuples: fetch this row's records
                    DevBuf g(sizeof(keto_tuple) * (e - b));
                    hipLaunchKernelGGL(k_gather, grid_for(e - b), dim3(BLK), 0, 0, in.tuples, row_idx.u32() + b, e - b,
                                       static_cast<keto_tuple *>(g.p));
                    KETO_HIP(hipGetLastError());
                    rec.resize(e - b);
                    KETO_HIP(hipMemcpy(rec.data(), g.p, sizeof(keto_tuple) * (e - b), hipMemcpyDeviceToHost));
                }
                std::vector<uint32_t> pos(e - b);
                for (uint32_t k = 0; k < e - b; k++) pos[k] = k;
                auto shard = [&](uint32_t k) { return in.host_tuples ? in.host_tuples[seg[k]].shard_id : rec[k].shard_id; };
                std::sort(pos.begin(), pos.end(), [&](uint32_t a, uint32_t c) {
                    int r = std::memcmp(shard(a), shard(c), 16);
                    return r != 0 ? r < 0 : seg[a] < seg[c];
                });
                for (uint32_t k = 0; k < e - b; k++) pos[k] = seg[pos[k]];
                seg.swap(pos);
                KETO_HIP(hipMemcpy(row_idx.u32() + b, seg.data(), 4ull * (e - b), hipMemcpyHostToDevice));
            }
        }
    }
    step("shard sort");
    {
        DevBuf set_cnt(4 * (N + 1));
        hipLaunchKernelGGL(k_row_fill, grid_for(N), dim3(BLK), 0, 0, out.all_off, N, row_idx.u32(), dst.u32(), out.all_subj,
                           set_cnt.u32(), reinterpret_cast<const unsigned long long *>(skey.p), out.all_shard);
        KETO_HIP(hipGetLastError());
        scan_excl(set_cnt.u32(), N);
        out.n_set = read_u32(set_cnt.u32(), N);
        out.set_dst = DevBuf(4ull * (out.n_set + out.set_slack) + 16);
        hipLaunchKernelGGL(k_set_fill, grid_for(N), dim3(BLK), 0, 0, out.all_off, set_cnt.u32(), N, out.all_subj,
                           out.set_dst.u32());
        hipLaunchKernelGGL(k_set_row, grid_for(N), dim3(BLK), 0, 0, set_cnt.u32(), N, out.set_dst.u32(), out.set_row);
        KETO_HIP(hipGetLastError());
        // scheduling weights: capped path counts relaxed to a fixed point (<= WEIGHT_ROUNDS)
        if (out.weight) {
            DevBuf w2(4 * (N + 1)), changed(4);
            hipLaunchKernelGGL(k_fill32, grid_for(N), dim3(BLK), 0, 0, out.weight, N, 1u);
            uint32_t *w = out.weight, *nw = w2.u32();
            for (uint32_t round = 0; in.weights && round < WEIGHT_ROUNDS; round++) {
                KETO_HIP(hipMemset(changed.p, 0, 4));
                hipLaunchKernelGGL(k_weight, grid_for(N), dim3(BLK), 0, 0, set_cnt.u32(), out.set_dst.u32(), N, w, nw,
                                   changed.u32());
                KETO_HIP(hipGetLastError());
                std::swap(w, nw);
                if (!read_u32(changed.u32(), 0)) break;
            }
            if (w != out.weight) KETO_HIP(hipMemcpy(out.weight, w, 4 * N, hipMemcpyDeviceToDevice));
        }
    }
    row_idx.reset();
    step("rows+weights");
    // reverse rows (subject -> nodes holding it directly, unordered) + the heavy-subject probe hash
    {
        DevBuf heavy(8);
        KETO_HIP(hipMemset(heavy.p, 0, 8));
        hipLaunchKernelGGL(k_heavy_count, grid_cap(M, FLAG_GRID), dim3(BLK), 0, 0, out.rev_off, M,
                           reinterpret_cast<unsigned long long *>(heavy.p));
        KETO_HIP(hipGetLastError());
        unsigned long long h = 0;
        KETO_HIP(hipMemcpy(&h, heavy.p, 8, hipMemcpyDeviceToHost));
        uint64_t buckets = 1;
        while (buckets * 2 < h * 2 + 2) buckets <<= 1;  // load factor <= 1/2
        out.probe_buckets = buckets;
        out.probe_keys = h;
        out.probe = DevBuf(16 * buckets);
        KETO_HIP(hipMemset(out.probe.p, 0, 16 * buckets));
        DevBuf cur(4 * (M + 1));
        KETO_HIP(hipMemcpy(cur.p, out.rev_off, 4 * (M + 1), hipMemcpyDeviceToDevice));
        hipLaunchKernelGGL(k_scatter_rev, grid_for(n), dim3(BLK), 0, 0, src.u32(), dst.u32(), n, in.n_uuids, out.rev_off,
                           cur.u32(), out.rev_nodes, reinterpret_cast<unsigned long long *>(out.probe.p), buckets - 1);
        KETO_HIP(hipGetLastError());
    }
    KETO_HIP(hipStreamSynchronize(nullptr));  // (the build's own stream: other work on the device runs on)
    step("reverse+probe");
}

void slot_setrows(const uint4 *set_row, uint64_t n_rows, const NsDev *ns, uint32_t n_ns, uint32_t *flag, uint32_t n_slots) {
    hipLaunchKernelGGL(k_slot_setrows, grid_cap(n_rows, FLAG_GRID), dim3(BLK), 0, 0, set_row, n_rows, ns, n_ns, flag, n_slots);
    KETO_HIP(hipGetLastError());
}

void slot_idrows(const keto_tuple *t, uint64_t n, const uint32_t *slot_of, uint32_t n_rel, const NsDev *ns, uint32_t *flag,
                 uint32_t n_slots) {
    if (n) hipLaunchKernelGGL(k_slot_idrows, grid_cap(n, FLAG_GRID), dim3(BLK), 0, 0, t, n, slot_of, n_rel, ns, flag, n_slots);
    KETO_HIP(hipGetLastError());
}

void leaf_mark(uint32_t *set_dst, uint64_t n, uint4 *set_row, uint64_t n_rows) {
    if (n) hipLaunchKernelGGL(k_leaf_mark, grid_for(n), dim3(BLK), 0, 0, set_dst, n, set_row);
    hipLaunchKernelGGL(k_row_inline, grid_for(n_rows), dim3(BLK), 0, 0, set_row, n_rows, set_dst);  // inline copies too
    KETO_HIP(hipGetLastError());
}

void remote_mark(uint32_t *set_dst, uint64_t n, uint4 *set_row, uint64_t n_rows, uint32_t n_owned) {
    if (n) hipLaunchKernelGGL(k_remote_mark, grid_for(n), dim3(BLK), 0, 0, set_dst, n, n_owned);
    hipLaunchKernelGGL(k_row_inline, grid_for(n_rows), dim3(BLK), 0, 0, set_row, n_rows, set_dst);  // inline copies too
    KETO_HIP(hipGetLastError());
    KETO_HIP(hipStreamSynchronize(nullptr));
}

void alias_mark(uint32_t *set_dst, uint64_t n, const uint32_t *vkey, uint4 *set_row, uint64_t n_rows) {
    hipLaunchKernelGGL(k_alias_mark, grid_for(n), dim3(BLK), 0, 0, set_dst, n, vkey);
    hipLaunchKernelGGL(k_row_inline, grid_for(n_rows), dim3(BLK), 0, 0, set_row, n_rows, set_dst);  // inline copies too
    KETO_HIP(hipGetLastError());
}

}  // namespace build
}  // namespace keto
