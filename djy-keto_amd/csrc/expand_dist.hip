// Expand over a graph partitioned by object across the ranks of a job (BASELINE config 5's
// "batched Expand trees"), over the resident partitions of frontier_dist.hip -- no closure
// snapshot, no per-batch build.
//
// expand.Engine.BuildTree (internal/expand/engine.go:54-124) is a sequential DFS whose visited set
// is global per call: which revisit becomes a leaf depends on pre-order.  It reads, per subject
// set it visits, that node's tuples in shard order (GetRelationTuples, persistence/sql/
// relationtuples.go:207-247).  Every node it can visit lies within max_depth - 1 hops of the root
// (a node at rest depth <= 1 is a leaf: its row only says whether it is nil), so:
//   1. rows: a level-synchronous fetch from the rows' owners -- per level one all-to-all of node
//      keys, the owners read their Expand rows (all_off / all_subj, shard order) and one all-to-all
//      sends the rows back; the next level is the subject sets of the rows received (a seen set
//      drops the nodes fetched before).  Rows land in a device hash table {node key -> row}.
//   2. the walk: one lane per root runs the reference's DFS over that table -- the visited set
//      (exact 64-bit keys: the object and the slot's visited class, H3) and the frame stack in
//      HBM scratch -- in two passes (count, then emit in root order).
// Ids are global throughout (the partitions' uuid space is the job's), so the trees are the
// API-form records of keto_expand_batch with no remapping.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "device_common.hpp"
#include "frontier_dist.hpp"

namespace keto {
namespace {

constexpr uint32_t XB = 256;
inline dim3 xgrid(uint64_t n, uint64_t cap = 1u << 16) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + XB - 1) / XB, cap)));
}
__device__ __forceinline__ uint64_t xgid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t xstride() { return (uint64_t)gridDim.x * blockDim.x; }

// a node key over global ids: (ns | rel << 15) << 32 | obj (ns < 2^15, rel < 2^16)
__host__ __device__ __forceinline__ uint64_t nkey(uint32_t ns, uint32_t obj, uint32_t rel) {
    return ((uint64_t)(std::min(ns, 0x7FFFu) | (std::min(rel, 0xFFFFu) << 15)) << 32) | obj;
}
__device__ __forceinline__ uint32_t key_owner(uint64_t k, const Dest &D) {  // keto_object_owner / keto_placement
    return D.owner((uint32_t)(k >> 32) & 0x7FFFu, (uint32_t)k);
}
// a row entry: {object or subject id, 1 << 31 | ns | rel << 15 for a subject set, else 0}
constexpr uint32_t XE_SET = 1u << 31;

// ---- 1. fetching rows

// keys per owner, then grouped by owner (order within an owner free)
__global__ __launch_bounds__(XB) void kx_hist(const uint64_t *k, uint32_t n, Dest D, uint32_t *hist) {
    for (uint64_t i = xgid(); i < n; i += xstride()) atomicAdd(&hist[key_owner(k[i], D)], 1u);
}
__global__ __launch_bounds__(XB) void kx_scatter(const uint64_t *k, uint32_t n, Dest D, uint32_t *cur, uint64_t *out) {
    for (uint64_t i = xgid(); i < n; i += xstride()) out[atomicAdd(&cur[key_owner(k[i], D)], 1u)] = k[i];
}
// owner side: the Expand row of a requested node (its object is this rank's): every tuple of it
__device__ __forceinline__ void row_of(const DevSnapshot &s, const Tables &T, uint64_t k, uint32_t &b, uint32_t &e) {
    b = e = 0;
    const uint32_t w = (uint32_t)(k >> 32), ns = w & 0x7FFFu, rel = w >> 15, obj = (uint32_t)k;
    if (ns >= s.n_ns) return;
    const uint32_t en = ent_lookup(s, ns, obj);
    if (en == NONE32) return;  // no tuple of the object
    const uint32_t node = t_node(T, ns, en, rel);
    if (node & VIRT_BIT) return;
    row_span(s.all_off, s.reloc, node, b, e);
}
__global__ __launch_bounds__(XB) void kx_row_len(DevSnapshot s, const uint64_t *req, uint32_t n, uint32_t *len) {
    const Tables T = global_tables(s);
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        uint32_t b, e;
        row_of(s, T, req[i], b, e);
        len[i] = e - b;
    }
}
__global__ __launch_bounds__(XB) void kx_row_fill(DevSnapshot s, const uint64_t *req, uint32_t n, const uint32_t *off, uint2 *out) {
    const Tables T = global_tables(s);
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        uint32_t b, e;
        row_of(s, T, req[i], b, e);
        uint2 *o = out + off[i];
        for (uint32_t j = b; j < e; j++) {
            const uint32_t sk = s.all_subj[j];
            if (!(sk & SKEY_SET)) {
                o[j - b] = make_uint2(sk, 0u);
                continue;
            }
            const uint32_t c = sk & ~SKEY_SET;
            const uint32_t cns = t_ns_of(T, c);
            const NsDev nd = T.ns[cns];
            const uint32_t co = c - nd.node_base;
            o[j - b] = make_uint2(s.ent_obj[nd.ent_base + co / nd.n_slots],
                                  XE_SET | t_real_ns(T, cns) | (s.slot_rel[nd.slot_base + co % nd.n_slots] << 15));
        }
    }
}
// requester side: row table {key + 1 lo, hi, offset into the pool, length}, open addressing
__global__ __launch_bounds__(XB) void kx_table_put(const uint64_t *keys, uint32_t n, const uint32_t *len, const uint32_t *off,
                                                   uint64_t pool_base, uint4 *tab, uint64_t mask) {
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        const uint64_t k = keys[i] + 1;
        uint64_t h = mix64(k) & mask;
        // (the keys of one launch are distinct -- the seen set asked for each once -- so a slot is
        // whoever's CAS claimed its first word; the walk reads the table in a later launch)
        while (atomicCAS(&tab[h].x, 0u, (uint32_t)k) != 0u) h = (h + 1) & mask;
        tab[h].y = (uint32_t)(k >> 32);
        tab[h].z = (uint32_t)(pool_base + off[i]);
        tab[h].w = len[i];
    }
}
// the next level: subject sets of the rows received that the seen set has not had
__global__ __launch_bounds__(XB) void kx_next(const uint2 *ent, uint32_t n, unsigned long long *seen, uint64_t mask, uint64_t *out,
                                              uint32_t *n_out) {
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        const uint2 e = ent[i];
        if (!(e.y & XE_SET)) continue;
        const unsigned long long k = nkey(e.y & 0x7FFFu, e.x, (e.y >> 15) & 0xFFFFu) + 1;
        uint64_t h = mix64(k) & mask;
        for (;;) {
            const unsigned long long p = atomicCAS(&seen[h], 0ull, k);
            if (p == 0ull) {
                out[atomicAdd(n_out, 1u)] = k - 1;
                break;
            }
            if (p == k) break;
            h = (h + 1) & mask;
        }
    }
}
__global__ __launch_bounds__(XB) void kx_seed(const keto_subject_set *r, uint32_t n, unsigned long long *seen, uint64_t mask,
                                              uint64_t *out, uint32_t *n_out) {
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        const unsigned long long k = nkey(r[i].ns, r[i].obj, r[i].rel) + 1;
        uint64_t h = mix64(k) & mask;
        for (;;) {
            const unsigned long long p = atomicCAS(&seen[h], 0ull, k);
            if (p == 0ull) {
                out[atomicAdd(n_out, 1u)] = k - 1;
                break;
            }
            if (p == k) break;
            h = (h + 1) & mask;
        }
    }
}

// ---- 2. the walk (expand/engine.go:54-124), one lane per root

struct Walk {
    DevSnapshot s;                  // (its namespace tables: the visited class of (ns, rel))
    const keto_subject_set *roots;
    uint32_t n;
    int32_t max_depth;
    const uint4 *tab;
    uint64_t tmask;
    const uint2 *pool;
    unsigned long long *vis;        // [lanes][vcap]: epoch << 48 | class << 32 | obj
    uint4 *stk;                     // [lanes][scap]
    uint32_t vcap, scap;
    const uint32_t *list;           // roots of this pass (null: all)
    uint32_t nl;
    unsigned long long *sizes;      // count pass out
    const unsigned long long *off;  // emit pass in
    keto_tree_node *out;
    int32_t *err;
    uint32_t emit;
};
__device__ __forceinline__ bool row_get(const Walk &W, uint64_t key, uint32_t &b, uint32_t &len) {
    const uint64_t k = key + 1;
    uint64_t h = mix64(k) & W.tmask;
    for (;;) {
        const uint4 t = W.tab[h];
        if (t.x == 0u && t.y == 0u) return false;
        if (t.x == (uint32_t)k && t.y == (uint32_t)(k >> 32)) {
            b = t.z;
            len = t.w;
            return true;
        }
        h = (h + 1) & W.tmask;
    }
}
// the visited key of a subject set: object + visited class of its slot (UUIDv5(obj, ns+"-"+rel),
// definitions.go:114-116: slots of equal ns+"-"+rel strings share a class)
__device__ __forceinline__ uint64_t vkey_of(const Walk &W, const Tables &T, uint32_t ns, uint32_t obj, uint32_t rel) {
    uint32_t cls = 0xFFFFu;  // (no slot: no tuple anywhere; never revisited under another name)
    if (ns < T.n_ns) {
        const uint32_t w = T.nsrel[(size_t)ns * T.n_rel + t_rel(T, rel)];
        if (nr_slot(w) != NO_SLOT) cls = W.s.vclass[T.ns[ns].slot_base + nr_slot(w)] & 0xFFFFu;
    }
    return ((uint64_t)cls << 32) | obj;
}
__device__ __forceinline__ int vis_add(unsigned long long *vis, uint32_t vcap, uint32_t epoch, uint64_t key, uint32_t &cnt) {
    const unsigned long long tag = ((unsigned long long)epoch << 48) | key;
    uint64_t h = mix64(key + 1) & (vcap - 1);
    for (;;) {
        const unsigned long long v = vis[h];
        if ((uint32_t)(v >> 48) != epoch) break;
        if (v == tag) return 1;  // seen
        h = (h + 1) & (vcap - 1);
    }
    if (2 * (cnt + 1) > vcap) return 2;  // full
    vis[h] = tag;
    cnt++;
    return 0;
}
__global__ __launch_bounds__(XB) void kx_walk(Walk W) {
    const Tables T = global_tables(W.s);
    const uint32_t lane = (uint32_t)xgid();
    unsigned long long *vis = W.vis + (size_t)lane * W.vcap;
    uint4 *stk = W.stk + (size_t)lane * W.scap;
    uint32_t epoch = 0;
    const uint32_t nq = W.list ? W.nl : W.n;
    for (uint64_t i = lane; i < nq; i += xstride()) {
        const uint32_t q = W.list ? W.list[i] : (uint32_t)i;
        if (W.emit && W.err[q]) continue;
        if (++epoch == 0xFFFFu) {  // (16-bit epochs: the table is cleared once they wrap)
            for (uint32_t j = 0; j < W.vcap; j++) vis[j] = 0;
            epoch = 1;
        }
        const keto_subject_set R = W.roots[q];
        int32_t d = R.max_depth;
        if (d <= 0 || W.max_depth < d) d = W.max_depth;  // :56-58
        keto_tree_node *out = W.emit ? W.out + W.off[q] : nullptr;
        uint64_t cnt = 0;
        bool full = false;
        uint32_t vc = 0, sp = 0;
        auto put = [&](uint32_t type, uint32_t kind, uint32_t obj, uint32_t ns, uint32_t rel, uint32_t nch) {
            if (out) {
                keto_tree_node o;
                o.type = type;
                o.subj_kind = kind;
                o.s_obj = obj;
                o.s_ns = kind ? ns : 0;
                o.s_rel = kind ? rel : 0;
                o.n_children = nch;
                out[cnt] = o;
            }
            cnt++;
        };
        uint32_t b = 0, len = 0;
        const bool virt = R.ns >= T.n_ns;
        if (!virt && vis_add(vis, W.vcap, epoch, vkey_of(W, T, R.ns, R.obj, R.rel), vc) == 2) full = true;  // root visited (:69-72)
        if (!virt && !full && row_get(W, nkey(R.ns, R.obj, R.rel), b, len) && len) {  // no tuples -> nil (:97-99)
            if (d <= 1) put(4, 1, R.obj, R.ns, R.rel, 0);  // :101-104
            else {
                put(1, 1, R.obj, R.ns, R.rel, len);
                uint4 top = make_uint4(b, b + len, (uint32_t)d, 0);
                for (;;) {
                    if (top.x == top.y) {
                        if (sp == 0) break;
                        top = stk[--sp];
                        continue;
                    }
                    const uint2 e = W.pool[top.x++];
                    if (!(e.y & XE_SET)) {  // subject id -> leaf (:60-67)
                        put(4, 0, e.x, 0, 0, 0);
                        continue;
                    }
                    const uint32_t cns = e.y & 0x7FFFu, crel = (e.y >> 15) & 0xFFFFu, cd = top.z - 1;
                    const int v = vis_add(vis, W.vcap, epoch, vkey_of(W, T, cns, e.x, crel), vc);
                    if (v == 2) {
                        full = true;
                        break;
                    }
                    uint32_t cb = 0, cl = 0;
                    if (v == 1 || !row_get(W, nkey(cns, e.x, crel), cb, cl) || cl == 0 || cd <= 1) {
                        put(4, 1, e.x, cns, crel, 0);  // revisit / nil / depth -> leaf (:101-117)
                        continue;
                    }
                    put(1, 1, e.x, cns, crel, cl);
                    if (sp + 1 >= W.scap) {
                        full = true;
                        break;
                    }
                    stk[sp++] = top;
                    top = make_uint4(cb, cb + cl, cd, 0);
                }
            }
        }
        if (!W.emit) {
            W.sizes[q] = full ? 0 : cnt;
            W.err[q] = full ? -1 : 0;  // (-1: the walk needs a larger visited table; the host reruns it)
        }
    }
}

__global__ __launch_bounds__(XB) void kx_add(uint32_t *v, uint32_t n, uint32_t x) {
    for (uint64_t i = xgid(); i < n; i += xstride()) v[i] += x;
}
// the seen set again, bigger: every key fetched so far (a list) re-entered
__global__ __launch_bounds__(XB) void kx_reseen(const uint64_t *keys, uint64_t n, unsigned long long *seen, uint64_t mask) {
    for (uint64_t i = xgid(); i < n; i += xstride()) {
        const unsigned long long k = keys[i] + 1;
        uint64_t h = mix64(k) & mask;
        while (atomicCAS(&seen[h], 0ull, k) != 0ull) h = (h + 1) & mask;
    }
}

struct XBuf {  // a growable device buffer keeping its first `keep` bytes
    void *p = nullptr;
    size_t cap = 0;
    XBuf() = default;
    XBuf(const XBuf &) = delete;
    XBuf &operator=(const XBuf &) = delete;
    ~XBuf() {
        if (p) (void)hipFree(p);
    }
    void swap(XBuf &o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
    void *need(size_t b, hipStream_t s, size_t keep = 0) {
        if (p && cap >= b) return p;
        void *q = nullptr;
        const size_t c = std::max<size_t>({b, cap * 2, 4096});
        KETO_HIP(hipMalloc(&q, c + 16));
        if (p && keep) KETO_HIP(hipMemcpyAsync(q, p, std::min(keep, cap), hipMemcpyDeviceToDevice, s));
        KETO_HIP(hipStreamSynchronize(s));
        if (p) {
            const hipError_t e = hipFree(p);
            if (e != hipSuccess)
                throw Error(KETO_E_DEVICE, std::string("XBuf: hipFree of a ") + std::to_string(cap) + "-byte block (growing to " +
                                               std::to_string(b) + ") failed: " + hipGetErrorString(e));
        }
        p = q;
        cap = c;
        return p;
    }
};

}  // namespace

void dist_expand(DistEngine &E, const keto_subject_set *roots, uint64_t n, std::vector<keto_tree_node> &nodes,
                 std::vector<uint64_t> &offsets, std::vector<int32_t> &err, DistExpandStats &st) {
    const DistView V = dist_view(E);
    KETO_HIP(hipSetDevice(V.device));
    ScratchStream on_hs(V.hs);  // (scan temporaries are used on the engine's stream)
    const uint32_t W = V.world;
    hipStream_t s = V.hs;
    const DevSnapshot &S = V.snap->dev;
    double wait_s = 0;
    const auto t0 = std::chrono::steady_clock::now();
    XBuf droots, seen, cur, next, sendk, recvk, lens, offs, ents, pool, tab, ctr, hist, allk, rowl, rowo;
    droots.need(std::max<uint64_t>(1, n) * sizeof(keto_subject_set), s);
    if (n) KETO_HIP(hipMemcpyAsync(droots.p, roots, n * sizeof(keto_subject_set), hipMemcpyHostToDevice, s));
    ctr.need(64, s);
    uint32_t *c = ctr.as<uint32_t>();
    // the seen set (keys asked for: the roots, then the subject sets of the rows received) and the
    // row table over the keys this rank fetched; both at most half full, grown as the fetch grows
    uint64_t seen_cap = 1u << 16, tab_cap = 1u << 16;
    while (seen_cap < 4 * std::max<uint64_t>(n, 1)) seen_cap <<= 1;
    seen.need(seen_cap * 8, s);
    KETO_HIP(hipMemsetAsync(seen.p, 0, seen_cap * 8, s));
    tab.need(tab_cap * 16, s);
    KETO_HIP(hipMemsetAsync(tab.p, 0, tab_cap * 16, s));
    KETO_HIP(hipMemsetAsync(c, 0, 4, s));
    cur.need(std::max<uint64_t>(1, n) * 8, s);
    if (n)
        hipLaunchKernelGGL(kx_seed, xgrid(n), dim3(XB), 0, s, droots.as<keto_subject_set>(), (uint32_t)n, seen.as<unsigned long long>(),
                           seen_cap - 1, cur.as<uint64_t>(), c);
    KETO_HIP(hipGetLastError());
    uint32_t ncur = 0;
    KETO_HIP(hipMemcpyAsync(&ncur, c, 4, hipMemcpyDeviceToHost, s));
    KETO_HIP(hipStreamSynchronize(s));
    uint64_t n_pool = 0, n_rows = 0;
    const int levels = std::max(1, V.limits.max_read_depth);
    for (int lvl = 0; lvl < levels; lvl++) {
        const auto tl = std::chrono::steady_clock::now();
        keto_partition_level L{};
        L.objects = ncur;
        // route this level's keys to their owners
        hist.need((size_t)W * 4 + 16, s);
        uint32_t *h = hist.as<uint32_t>();
        KETO_HIP(hipMemsetAsync(h, 0, (size_t)W * 4, s));
        if (ncur) hipLaunchKernelGGL(kx_hist, xgrid(ncur), dim3(XB), 0, s, cur.as<uint64_t>(), ncur, Dest{W, V.rank, V.place}, h);
        std::vector<uint32_t> cnt(W);
        KETO_HIP(hipMemcpyAsync(cnt.data(), h, (size_t)W * 4, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipStreamSynchronize(s));
        std::vector<uint64_t> sent(W), sendc(W);
        for (uint32_t r = 0; r < W; r++) {
            sent[r] = cnt[r];
            sendc[r] = cnt[r] | (ncur ? 1ull << 63 : 0ull);
        }
        const std::vector<uint64_t> rc = dist_alltoall(V, sendc, wait_s);
        bool any = false;
        std::vector<uint64_t> recv(W);
        uint64_t nrecv = 0;
        for (uint32_t r = 0; r < W; r++) {
            any |= (rc[r] >> 63) & 1u;
            recv[r] = rc[r] & ((1ull << 63) - 1);
            nrecv += recv[r];
        }
        if (!any) break;  // no rank has keys left: every row any walk can read is here
        st.levels++;
        sendk.need(std::max<uint32_t>(1, ncur) * 8, s);
        if (ncur) {
            std::vector<uint32_t> cu(W, 0);
            for (uint32_t r = 1; r < W; r++) cu[r] = cu[r - 1] + cnt[r - 1];
            KETO_HIP(hipMemcpyAsync(h, cu.data(), (size_t)W * 4, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(kx_scatter, xgrid(ncur), dim3(XB), 0, s, cur.as<uint64_t>(), ncur, Dest{W, V.rank, V.place}, h, sendk.as<uint64_t>());
        }
        std::vector<uint64_t> sb(W), rb(W);
        for (uint32_t r = 0; r < W; r++) {
            sb[r] = sent[r] * 8;
            rb[r] = recv[r] * 8;
            if (r != V.rank) L.request_bytes += sb[r];
        }
        recvk.need(std::max<uint64_t>(1, nrecv) * 8, s);
        dist_alltoallv(V, sendk.p, sb, recvk.p, rb, wait_s);
        // owner side: the rows of the keys received, in receive order
        lens.need((nrecv + 1) * 4, s);
        uint32_t *ln = lens.as<uint32_t>();
        KETO_HIP(hipMemsetAsync(ln, 0, (nrecv + 1) * 4, s));
        if (nrecv) hipLaunchKernelGGL(kx_row_len, xgrid(nrecv), dim3(XB), 0, s, S, recvk.as<uint64_t>(), (uint32_t)nrecv, ln);
        offs.need((nrecv + 1) * 4, s);
        uint32_t *of = offs.as<uint32_t>();
        KETO_HIP(hipMemcpyAsync(of, ln, (nrecv + 1) * 4, hipMemcpyDeviceToDevice, s));
        build::scan_excl(of, nrecv, s);
        std::vector<uint32_t> src_off(W + 1, 0);  // entries per source: the scan at the source boundaries
        {
            uint64_t at = 0;
            for (uint32_t r = 0; r <= W; r++) {
                KETO_HIP(hipMemcpyAsync(&src_off[r], of + at, 4, hipMemcpyDeviceToHost, s));
                if (r < W) at += recv[r];
            }
            KETO_HIP(hipStreamSynchronize(s));
        }
        const uint64_t n_out = src_off[W];
        ents.need(std::max<uint64_t>(1, n_out) * 8, s);
        if (nrecv)
            hipLaunchKernelGGL(kx_row_fill, xgrid(nrecv), dim3(XB), 0, s, S, recvk.as<uint64_t>(), (uint32_t)nrecv, of, ents.as<uint2>());
        KETO_HIP(hipGetLastError());
        // back: each key's row length (in the order the requester sent it), then the entries
        rowl.need((n_rows + ncur + 1) * 4, s, n_rows * 4);
        std::vector<uint64_t> lb(W), lr(W), eb(W);
        for (uint32_t r = 0; r < W; r++) {
            lb[r] = recv[r] * 4;
            lr[r] = sent[r] * 4;
            eb[r] = (uint64_t)(src_off[r + 1] - src_off[r]);
        }
        uint32_t *rl = rowl.as<uint32_t>() + n_rows;
        dist_alltoallv(V, ln, lb, rl, lr, wait_s);
        const std::vector<uint64_t> er = dist_alltoall(V, eb, wait_s);
        uint64_t n_in = 0;
        std::vector<uint64_t> eb8(W), er8(W);
        for (uint32_t r = 0; r < W; r++) {
            n_in += er[r];
            eb8[r] = eb[r] * 8;
            er8[r] = er[r] * 8;
            if (r != V.rank) L.tuple_bytes_sent += eb8[r];
        }
        pool.need((n_pool + n_in) * 8 + 16, s, n_pool * 8);
        dist_alltoallv(V, ents.p, eb8, pool.as<uint2>() + n_pool, er8, wait_s);
        // the rows into the table (their offsets: the scan of the lengths received, from the pool's
        // end); the keys and rows are kept as lists too, for growing the tables
        allk.need((n_rows + ncur) * 8 + 16, s, n_rows * 8);
        rowo.need((n_rows + ncur + 1) * 4, s, n_rows * 4);
        if (ncur) {
            KETO_HIP(hipMemcpyAsync(allk.as<uint64_t>() + n_rows, sendk.p, (uint64_t)ncur * 8, hipMemcpyDeviceToDevice, s));
            uint32_t *ro = rowo.as<uint32_t>() + n_rows;
            KETO_HIP(hipMemcpyAsync(ro, rl, (uint64_t)ncur * 4, hipMemcpyDeviceToDevice, s));
            KETO_HIP(hipMemsetAsync(ro + ncur, 0, 4, s));
            build::scan_excl(ro, ncur, s);
            if (n_pool) hipLaunchKernelGGL(kx_add, xgrid(ncur), dim3(XB), 0, s, ro, ncur, (uint32_t)n_pool);  // (pool positions)
        }
        const uint64_t rows_now = n_rows + ncur;
        if (2 * rows_now > tab_cap) {  // the row table, bigger: every row so far entered again
            while (2 * rows_now > tab_cap) tab_cap <<= 1;
            tab.need(tab_cap * 16, s);
            KETO_HIP(hipMemsetAsync(tab.p, 0, tab_cap * 16, s));
            if (n_rows)
                hipLaunchKernelGGL(kx_table_put, xgrid(n_rows), dim3(XB), 0, s, allk.as<uint64_t>(), (uint32_t)n_rows, rowl.as<uint32_t>(),
                                   rowo.as<uint32_t>(), 0ull, tab.as<uint4>(), tab_cap - 1);
        }
        if (ncur)
            hipLaunchKernelGGL(kx_table_put, xgrid(ncur), dim3(XB), 0, s, allk.as<uint64_t>() + n_rows, ncur, rl,
                               rowo.as<uint32_t>() + n_rows, 0ull, tab.as<uint4>(), tab_cap - 1);
        KETO_HIP(hipGetLastError());
        n_rows = rows_now;
        // the next level: subject sets of these rows not asked for before -- none once the
        // depth makes their nodes leaves (the last level's rows only say nil or not)
        const uint64_t seen_now = n_rows + n_in;
        if (2 * seen_now > seen_cap) {
            while (2 * seen_now > seen_cap) seen_cap <<= 1;
            seen.need(seen_cap * 8, s);
            KETO_HIP(hipMemsetAsync(seen.p, 0, seen_cap * 8, s));
            hipLaunchKernelGGL(kx_reseen, xgrid(n_rows), dim3(XB), 0, s, allk.as<uint64_t>(), n_rows, seen.as<unsigned long long>(),
                               seen_cap - 1);
        }
        next.need(std::max<uint64_t>(1, n_in) * 8, s);
        KETO_HIP(hipMemsetAsync(c, 0, 4, s));
        if (n_in && lvl + 1 < levels)
            hipLaunchKernelGGL(kx_next, xgrid(n_in), dim3(XB), 0, s, pool.as<uint2>() + n_pool, (uint32_t)n_in,
                               seen.as<unsigned long long>(), seen_cap - 1, next.as<uint64_t>(), c);
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpyAsync(&ncur, c, 4, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipStreamSynchronize(s));
        n_pool += n_in;
        cur.swap(next);
        L.tuples = n_in;
        L.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count();
        st.per_level.push_back(L);
        st.bytes_sent += L.request_bytes + L.tuple_bytes_sent;
    }
    st.rows = n_rows;
    st.entries = n_pool;
    const auto t1 = std::chrono::steady_clock::now();
    st.fetch_s = std::chrono::duration<double>(t1 - t0).count();
    // the walks: count pass, root-order offsets, emit pass; roots whose visited set outgrows the
    // lane's table go again with a larger one
    offsets.assign(n + 1, 0);
    err.assign(std::max<uint64_t>(1, n), 0);
    nodes.clear();
    if (n) {
        XBuf sizes, offd, errd, vis, stk, out, lst;
        sizes.need(n * 8, s);
        offd.need((n + 1) * 8, s);
        errd.need(n * 4, s);
        const uint32_t scap = (uint32_t)levels + 2;
        Walk Wk{};
        Wk.s = S;
        Wk.roots = droots.as<keto_subject_set>();
        Wk.n = (uint32_t)n;
        Wk.max_depth = V.limits.max_read_depth;
        Wk.tab = tab.as<uint4>();
        Wk.tmask = tab_cap - 1;
        Wk.pool = pool.as<uint2>();
        Wk.scap = scap;
        Wk.sizes = sizes.as<unsigned long long>();
        Wk.err = errd.as<int32_t>();
        auto run = [&](uint32_t lanes, uint32_t vcap, const uint32_t *list, uint32_t nl, bool emit) {
            vis.need((size_t)lanes * vcap * 8, s);
            KETO_HIP(hipMemsetAsync(vis.p, 0, (size_t)lanes * vcap * 8, s));
            stk.need((size_t)lanes * scap * 16, s);
            Wk.vis = vis.as<unsigned long long>();
            Wk.stk = stk.as<uint4>();
            Wk.vcap = vcap;
            Wk.list = list;
            Wk.nl = nl;
            Wk.emit = emit ? 1u : 0u;
            hipLaunchKernelGGL(kx_walk, dim3((lanes + XB - 1) / XB), dim3(XB), 0, s, Wk);
            KETO_HIP(hipGetLastError());
        };
        const uint32_t lanes = (uint32_t)std::min<uint64_t>(n, 4096);
        run(lanes, 4096, nullptr, 0, false);
        std::vector<unsigned long long> hs(n);
        std::vector<int32_t> he(n);
        KETO_HIP(hipMemcpyAsync(hs.data(), sizes.p, n * 8, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipMemcpyAsync(he.data(), errd.p, n * 4, hipMemcpyDeviceToHost, s));
        KETO_HIP(hipStreamSynchronize(s));
        std::vector<uint32_t> redo;
        for (uint64_t i = 0; i < n; i++)
            if (he[i]) redo.push_back((uint32_t)i);
        if (!redo.empty()) {  // one lane per such root, a visited table over every row fetched
            uint64_t vc = 4096;
            while (vc < 2 * (n_rows + 1)) vc <<= 1;
            lst.need(redo.size() * 4, s);
            KETO_HIP(hipMemcpyAsync(lst.p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
            run((uint32_t)std::min<size_t>(redo.size(), 64), (uint32_t)vc, lst.as<uint32_t>(), (uint32_t)redo.size(), false);
            KETO_HIP(hipMemcpyAsync(hs.data(), sizes.p, n * 8, hipMemcpyDeviceToHost, s));
            KETO_HIP(hipMemcpyAsync(he.data(), errd.p, n * 4, hipMemcpyDeviceToHost, s));
            KETO_HIP(hipStreamSynchronize(s));
        }
        for (uint64_t i = 0; i < n; i++) {
            if (he[i]) throw Error(KETO_E_LIMIT, "partitioned Expand: a tree outgrew its visited table");
            offsets[i + 1] = offsets[i] + hs[i];
        }
        KETO_HIP(hipMemcpyAsync(offd.p, offsets.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
        const uint64_t total = offsets[n];
        out.need(std::max<uint64_t>(1, total) * sizeof(keto_tree_node), s);
        Wk.out = out.as<keto_tree_node>();
        Wk.off = offd.as<unsigned long long>();
        run(lanes, 4096, nullptr, 0, true);
        if (!redo.empty()) {
            uint64_t vc = 4096;
            while (vc < 2 * (n_rows + 1)) vc <<= 1;
            run((uint32_t)std::min<size_t>(redo.size(), 64), (uint32_t)vc, lst.as<uint32_t>(), (uint32_t)redo.size(), true);
        }
        nodes.resize(total);
        if (total) KETO_HIP(hipMemcpyAsync(nodes.data(), out.p, total * sizeof(keto_tree_node), hipMemcpyDeviceToHost, s));
        KETO_HIP(hipStreamSynchronize(s));
    }
    st.walk_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    st.exchange_s = wait_s;
}

}  // namespace keto
