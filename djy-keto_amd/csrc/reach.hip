// Reachability tables: per node of a "tabled" relation slot, the nodes reachable from it over
// subject-set rows.  The frontier engines decide a sub-check checkIsAllowed(n, d > 1) on such a
// node NotMember where it is spawned when no node of Reach(n) holds the query subject in its own
// row (frontier_goal.inc reach_prunes; oracle/refsem.c u_reach_prunes states the rule and why it
// is exact): on Drive-style graphs that is most nested-group expand-subject goal chains
// (internal/check/engine.go:102-164 on rows of Group#members), decided with one table read
// instead of a goal per group along the chain.
//
// Tabled slot: pure (no rewrite, no ASTRelationFor error: definitions.go:37-62), some row holds a
// subject set (RI_SETROWS) and some tuple's subject set names it (an expand-subject child can be
// one of its nodes).  Tabled node: every node of its reach is pure and |Reach| <= REACH_CAP.
// Snapshots whose visited keys alias (D.vkey) carry none; in a partition's snapshot a reach that
// meets a ghost node (another rank's object: its rows live there) leaves its node untabled.  Layout: reach_base[global slot] = first entry of the slot in reach_idx (NONE32: not
// tabled), reach_idx[base + entity - ent_base] = {offset, count} (count NONE32: not tabled) into
// reach_pool, the reach without the node itself (its own row is what the caller tested).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_common.hpp"
#include "engine.hpp"

namespace keto {
namespace {

constexpr uint32_t RB = 256;

struct ReachIn {
    const uint4 *set_row;
    const uint32_t *set_dst;
    uint32_t edge_mask;
    const NsDev *ns;
    uint32_t n_ns;
    const uint32_t *relinfo;
    const uint4 *tslots;  // {first candidate, ns, slot in ns, 0} per tabled slot, ascending
    uint32_t n_tslots;
    uint64_t n_cand;
    uint32_t cap;      // REACH_CAP, or KETO_REACH_CAP (A/B)
    uint32_t n_owned;  // the first ghost node (a partition's snapshot; else every node)
};

__device__ __forceinline__ uint32_t ns_of_node(const NsDev *ns, uint32_t n_ns, uint32_t node) {
    uint32_t lo = 0, hi = n_ns;  // last namespace whose node_base <= node
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (ns[m].node_base <= node) lo = m;
        else hi = m;
    }
    return lo;
}
__device__ __forceinline__ bool node_pure(const ReachIn &R, uint32_t node) {
    const NsDev nd = R.ns[ns_of_node(R.ns, R.n_ns, node)];
    const uint32_t ri = R.relinfo[nd.slot_base + (node - nd.node_base) % nd.n_slots];
    return ri_status(ri) != REL_ERROR && !ri_rw(ri);
}

// slots some subject-set edge points into: the ns table and the flags in LDS when they fit (one
// global store per flag and block), else straight to memory
constexpr uint32_t T_NS = 256, T_FLAGS = 4096;
__global__ __launch_bounds__(RB) void k_slot_targets(const uint32_t *set_dst, uint64_t n, uint32_t edge_mask, const NsDev *ns,
                                                     uint32_t n_ns, uint32_t *flag, uint32_t n_flags) {
    __shared__ NsDev lns[T_NS + 1];
    __shared__ uint32_t lf[T_FLAGS];
    const bool lt = n_ns < T_NS, lfl = n_flags <= T_FLAGS;
    if (lt)
        for (uint32_t t = threadIdx.x; t <= n_ns; t += blockDim.x) lns[t] = ns[t];
    if (lfl)
        for (uint32_t t = threadIdx.x; t < n_flags; t += blockDim.x) lf[t] = 0;
    __syncthreads();
    const NsDev *nst = lt ? lns : ns;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = set_dst[i] & edge_mask;
        const NsDev nd = nst[ns_of_node(nst, n_ns, c)];
        const uint32_t g = nd.slot_base + (c - nd.node_base) % nd.n_slots;
        if (lfl) lf[g] = 1;
        else if (!flag[g]) atomicOr(&flag[g], 1u);  // (read first: most edges find the flag set)
    }
    if (!lfl) return;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n_flags; t += blockDim.x)
        if (lf[t] && !flag[t]) flag[t] = 1;
}

// One wave per candidate node: a breadth-first walk of its reach with the list in registers
// (entry k on lane k % 64, register k / 64).  Pass 1 (FILL = false) counts, pass 2 writes the
// record {count, entry 0, entry 1, pool offset} and the entries past the first two at the offset
// pass 1's scan gave (pool runs padded to 4 entries: the engine reads them in 16-byte windows).
// `list` (incremental builds): the candidates to walk, else all of them.
__device__ __forceinline__ uint32_t pool_need(uint32_t n) { return n > 2 ? (n - 2 + 3) & ~3u : 0u; }
template <bool FILL>
__global__ __launch_bounds__(RB) void k_reach(ReachIn R, const uint32_t *list, uint64_t n_items, uint4 *idx, uint32_t *lens,
                                              uint32_t *pool, uint32_t pool_base, unsigned long long *total) {
    static_assert(REACH_CAP_MAX <= 128, "two list registers per lane");
    const uint32_t wpb = blockDim.x >= 64 ? blockDim.x / 64 : 1;  // (the CPU emulation: one-lane blocks)
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    unsigned long long acc_pool = 0, acc_tabled = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * wpb + threadIdx.x / 64; i < n_items; i += nw) {
        const uint64_t t = list ? list[i] : i;
        uint32_t lo = 0, hi = R.n_tslots;  // the candidate's slot
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (R.tslots[m].x <= t) lo = m;
            else hi = m;
        }
        const uint4 ts = R.tslots[lo];
        const NsDev nd = R.ns[ts.y];
        const uint32_t g = nd.node_base + (uint32_t)(t - ts.x) * nd.n_slots + ts.z;
        uint32_t cnt = 1, head = 0;
        bool ok = true;
#ifdef KETO_CPUEMU  // one lane: the list in an array
        uint32_t L[REACH_CAP_MAX];
        L[0] = g;
        while (ok && head < cnt) {
            const uint32_t n = L[head++];
            if (n >= R.n_owned || !node_pure(R, n)) {  // (a ghost: its row is another rank's)
                ok = false;
                break;
            }
            const uint4 row = R.set_row[n];
            for (uint32_t j = row.x; j < row.y && ok; j++) {
                const uint32_t c = R.set_dst[j] & R.edge_mask;
                bool fresh = true;
                for (uint32_t k = 0; k < cnt; k++)
                    if (L[k] == c) fresh = false;
                if (!fresh) continue;
                if (cnt == R.cap) ok = false;
                else L[cnt++] = c;
            }
        }
        const uint32_t n = ok ? cnt - 1 : 0u;  // the reach without g
        if constexpr (!FILL) {
            lens[i] = pool_need(n);
            if (ok) {
                acc_pool += pool_need(n);
                acc_tabled++;
            }
        } else {
            if (!ok) {
                idx[t] = make_uint4(NONE32, NONE32, NONE32, 0u);
            } else {
                const uint32_t off = pool_base + lens[i];
                for (uint32_t k = 2; k < n; k++) pool[off + k - 2] = L[k + 1];
                for (uint32_t k = n; k < pool_need(n) + 2 && k >= 2; k++) pool[off + k - 2] = NONE32;
                idx[t] = make_uint4(n, n > 0 ? L[1] : NONE32, n > 1 ? L[2] : NONE32, off);
            }
        }
#else
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t e0 = lane == 0 ? g : NONE32, e1 = NONE32;
        while (ok && head < cnt) {
            const uint32_t n = __shfl(head < 64 ? e0 : e1, (int)(head & 63u));
            head++;
            if (n >= R.n_owned || !node_pure(R, n)) {  // (a ghost: its row is another rank's)
                ok = false;
                break;
            }
            const uint4 row = R.set_row[n];
            for (uint32_t b = row.x; b < row.y && ok; b += 64) {
                const uint32_t j = b + lane;
                const uint32_t c = j < row.y ? (R.set_dst[j] & R.edge_mask) : NONE32;
                bool fresh = c != NONE32;
                for (uint32_t k = 0; k < cnt; k++)
                    if (__shfl(k < 64 ? e0 : e1, (int)(k & 63u)) == c) fresh = false;
                unsigned long long m = __ballot(fresh);
                while (m) {  // the new children in edge order, each once
                    const int lead = __ffsll((long long)m) - 1;
                    const uint32_t v = __shfl(c, lead);
                    if (cnt == R.cap) {
                        ok = false;
                        break;
                    }
                    if (lane == (cnt & 63u)) {
                        if (cnt < 64) e0 = v;
                        else e1 = v;
                    }
                    cnt++;
                    m &= ~__ballot(fresh && c == v);
                }
            }
        }
        const uint32_t n = ok ? cnt - 1 : 0u;  // the reach without g: entry k is list entry k + 1
        if constexpr (!FILL) {
            if (lane == 0) lens[i] = pool_need(n);
            if (ok) {  // (summed per wave, added once at the end: same-address atomics serialise)
                acc_pool += pool_need(n);
                acc_tabled++;
            }
        } else {
            const uint32_t x1 = __shfl(e0, 1), x2 = __shfl(e0, 2);
            if (!ok) {
                if (lane == 0) idx[t] = make_uint4(NONE32, NONE32, NONE32, 0u);
            } else {
                const uint32_t off = pool_base + lens[i], need = pool_need(n);
                // list entry L = lane (e0) / 64 + lane (e1) is reach entry L - 1, pool slot L - 3
                if (lane >= 3 && lane - 3 < need) pool[off + lane - 3] = lane <= n ? e0 : NONE32;
                if (64 + lane - 3 < need) pool[off + 61 + lane] = 64 + lane <= n ? e1 : NONE32;
                if (lane == 0) idx[t] = make_uint4(n, n > 0 ? x1 : NONE32, n > 1 ? x2 : NONE32, off);
            }
        }
#endif
    }
    if constexpr (!FILL) {
        if ((threadIdx.x & 63u) == 0 && acc_tabled) {
            atomicAdd(total, acc_pool);
            atomicAdd(total + 1, acc_tabled);
        }
    }
}


// a patch's ancestor walk: the parents (over subject-set rows: the reverse rows of the nodes as
// subjects) of this level's nodes not seen yet, into the next level.  seen: open addressing over
// node + 1 (0 = empty), a power-of-two table the caller sizes past twice the walk's bound
// (only parents in tabled slots: every node of a tabled reach but its root is some row's subject
// set, pure, with subject-set rows -- a node of a tabled slot)
__device__ __forceinline__ bool seen_insert(uint32_t *seen, uint32_t mask, uint32_t node) {
    const uint32_t key = node + 1u;
    for (uint32_t h = (uint32_t)mix64(key) & mask;; h = (h + 1) & mask) {
        const uint32_t v = seen[h];
        if (v == key) return false;
        if (v == 0) {
            const uint32_t o = atomicCAS(&seen[h], 0u, key);
            if (o == 0) return true;
            if (o == key) return false;
        }
    }
}
__global__ __launch_bounds__(RB) void k_seen_init(const uint32_t *nodes, uint32_t n, uint32_t *seen, uint32_t mask) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        (void)seen_insert(seen, mask, nodes[i]);
}
__global__ __launch_bounds__(RB) void k_anc_level(const uint32_t *front, uint32_t n, const uint32_t *rev_off, const uint4 *reloc,
                                                  const uint32_t *rev_nodes, uint32_t n_uuids, const NsDev *ns, uint32_t n_ns, const uint32_t *relinfo,
                                                  uint32_t *seen, uint32_t mask, uint32_t *next, uint32_t *next_n, uint32_t cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t si = (uint64_t)n_uuids + front[i];
        uint32_t j, e;
        row_span(rev_off, reloc, si, j, e);
        for (; j < e; j++) {
            const uint32_t p = rev_nodes[j];
            const NsDev nd = ns[ns_of_node(ns, n_ns, p)];
            if (!(relinfo[nd.slot_base + (p - nd.node_base) % nd.n_slots] & RI_REACH)) continue;
            if (!seen_insert(seen, mask, p)) continue;
            const uint32_t at = atomicAdd(next_n, 1u);
            if (at < cap) next[at] = p;
        }
    }
}
__global__ __launch_bounds__(RB) void k_count_tabled(const uint4 *idx, uint64_t n, unsigned long long *out) {
    unsigned long long c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += idx[i].x != NONE32;
    if (c) atomicAdd(out, c);
}
// the candidates among nodes (tabled slots' nodes), compacted
__global__ __launch_bounds__(RB) void k_cand_of(const uint32_t *nodes, uint32_t n, const NsDev *ns, uint32_t n_ns, const uint32_t *base,
                                                uint32_t *out, uint32_t *out_n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = nodes[i];
        const NsDev nd = ns[ns_of_node(ns, n_ns, c)];
        const uint32_t b = base[nd.slot_base + (c - nd.node_base) % nd.n_slots];
        if (b != NONE32) out[atomicAdd(out_n, 1u)] = b + (c - nd.node_base) / nd.n_slots;
    }
}
}  // namespace

namespace {
// the tabled slots of s: base[global slot] = first candidate or NONE32, ts = {first candidate, ns,
// slot, 0} per tabled slot; the candidate count (0: none, or past the index's range)
uint64_t tabled_slots(Snapshot &s, std::vector<uint32_t> &base, std::vector<uint4> &ts) {
    using build::DevBuf;
    DevSnapshot &D = s.dev;
    const uint32_t n_slots = (uint32_t)s.relinfo.size();
    std::vector<uint32_t> target(n_slots, 0);
    if (s.slot_in.size() == n_slots) {  // a room snapshot keeps the counts (its set_dst holds moved rows' old copies)
        for (uint32_t g = 0; g < n_slots; g++) target[g] = s.slot_in[g] != 0;
    } else {
        DevBuf flag(4ull * n_slots);
        KETO_HIP(hipMemset(flag.p, 0, 4ull * n_slots));
        const uint64_t ne = s.info.n_set_edges;
        hipLaunchKernelGGL(k_slot_targets, dim3((uint32_t)std::min<uint64_t>(2048, (ne + RB - 1) / RB)), dim3(RB), 0, 0, D.set_dst,
                           ne, D.edge_mask, D.ns, D.n_ns, flag.u32(), n_slots);
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(target.data(), flag.p, 4ull * n_slots, hipMemcpyDeviceToHost));
    }
    base.assign(n_slots, NONE32);
    ts.clear();
    uint64_t n_cand = 0;
    for (uint32_t ns = 0; ns < s.n_ns; ns++)
        for (uint32_t k = 0; k < s.ns[ns].n_slots; k++) {
            const uint32_t g = s.ns[ns].slot_base + k, ri = s.relinfo[g];
            if (!target[g] || !ri_setrows(ri) || ri_rw(ri) || ri_status(ri) == REL_ERROR) continue;
            base[g] = (uint32_t)n_cand;
            ts.push_back(make_uint4((uint32_t)n_cand, ns, k, 0));
            n_cand += s.ns[ns + 1].ent_base - s.ns[ns].ent_base;
            if (n_cand >= (1ull << 31)) return 0;  // (past the index's range: no tables)
        }
    return n_cand;
}
// RI_REACH on the tabled slots (a fresh relinfo copy: a patched snapshot may share its base's)
void reach_bits(Snapshot &s, const std::vector<uint32_t> &base) {
    for (size_t g = 0; g < s.relinfo.size(); g++)
        s.relinfo[g] = (s.relinfo[g] & ~RI_REACH) | (g < base.size() && base[g] != NONE32 ? RI_REACH : 0u);
    // (an advance writes the snapshot's own array where it lies: engines read s.dev at launch)
    uint32_t *ri = s.dev.relinfo && s.sole(s.dev.relinfo) ? const_cast<uint32_t *>(s.dev.relinfo)
                                                          : static_cast<uint32_t *>(s.alloc(4 * std::max<size_t>(1, s.relinfo.size()) + 16));
    if (!s.relinfo.empty()) KETO_HIP(hipMemcpy(ri, s.relinfo.data(), 4 * s.relinfo.size(), hipMemcpyHostToDevice));
    s.dev.relinfo = ri;
}
}  // namespace

// The tables of snapshot s (its rows, relation info and ns table are on the device); nothing
// when none of its slots qualifies, its visited keys alias, or KETO_NO_REACH is set (A/B runs:
// the oracle's RS_NO_REACH).  s.dev.reach_* are set, allocated through s.
void build_reach(Snapshot &s) {
    using build::DevBuf;
    DevSnapshot &D = s.dev;
    for (const void *p : {(const void *)D.reach_base, (const void *)D.reach_idx, (const void *)D.reach_pool})
        if (p && s.sole(p)) s.drop(p);  // (an advance rebuilding its own tables)
    D.reach_base = nullptr;
    D.reach_idx = nullptr;
    D.reach_pool = nullptr;
    s.reach_pool_cap = 0;
    s.info.n_reach = 0;
    s.reach_slots.clear();
    s.reach_cand = s.reach_pool_n = s.reach_pool_built = 0;
    bool had = false;
    for (uint32_t ri : s.relinfo) had |= (ri & RI_REACH) != 0;
    if (had) reach_bits(s, {});
    static const bool off = [] {
        const char *e = getenv("KETO_NO_REACH");
        return e && *e == '1';
    }();
    const uint32_t n_slots = (uint32_t)s.relinfo.size();
    if (off || D.vkey || !n_slots || !s.info.n_set_edges) return;
    std::vector<uint32_t> base;
    std::vector<uint4> ts;
    const uint64_t n_cand = tabled_slots(s, base, ts);
    if (!n_cand) return;
    if (ts.empty()) return;
    uint4 *idx = static_cast<uint4 *>(s.alloc(16 * n_cand + 16));
    DevBuf lens(4 * n_cand + 16), tot(16), d_ts(16 * ts.size());
    KETO_HIP(hipMemset(tot.p, 0, 16));
    KETO_HIP(hipMemcpy(d_ts.p, ts.data(), 16 * ts.size(), hipMemcpyHostToDevice));
    static const uint32_t cap = [] {
        const char *e = getenv("KETO_REACH_CAP");
        const uint32_t c = e ? (uint32_t)atoi(e) : REACH_CAP;
        return c >= 1 && c <= REACH_CAP_MAX ? c : REACH_CAP;
    }();
    ReachIn R{D.set_row, D.set_dst, D.edge_mask, D.ns, D.n_ns, D.relinfo, static_cast<const uint4 *>(d_ts.p), (uint32_t)ts.size(),
              n_cand, cap, D.n_ns_x != D.n_ns ? D.n_owned : NONE32};
    const dim3 grid((uint32_t)std::min<uint64_t>(65536, (n_cand + RB / 64 - 1) / (RB / 64)));  // (4 waves a block)
    hipLaunchKernelGGL(k_reach<false>, grid, dim3(RB), 0, 0, R, nullptr, n_cand, idx, lens.u32(), nullptr, 0u,
                       static_cast<unsigned long long *>(tot.p));
    KETO_HIP(hipGetLastError());
    unsigned long long cn[2] = {0, 0};
    KETO_HIP(hipMemcpy(cn, tot.p, 16, hipMemcpyDeviceToHost));
    const unsigned long long total = cn[0];
    if (total >= (1ull << 31)) return;  // (the allocation of idx goes back with the snapshot)
    build::scan_excl(lens.u32(), n_cand);
    const uint64_t pool_cap = s.room.reloc_cap ? total + total / 16 + (1u << 16) : total;  // (advances append)
    uint32_t *pool = static_cast<uint32_t *>(s.alloc(4 * pool_cap + 16));
    hipLaunchKernelGGL(k_reach<true>, grid, dim3(RB), 0, 0, R, nullptr, n_cand, idx, lens.u32(), pool, 0u, nullptr);
    KETO_HIP(hipGetLastError());
    uint32_t *d_base = static_cast<uint32_t *>(s.alloc(4ull * n_slots + 16));
    KETO_HIP(hipMemcpy(d_base, base.data(), 4ull * n_slots, hipMemcpyHostToDevice));
    KETO_HIP(hipStreamSynchronize(nullptr));
    D.reach_base = d_base;
    D.reach_idx = idx;
    D.reach_pool = pool;
    s.info.n_reach = cn[1];
    reach_bits(s, base);
    s.reach_slots = std::move(base);
    s.reach_cand = n_cand;
    s.reach_pool_n = s.reach_pool_built = total;
    s.reach_pool_cap = pool_cap;
}

void patch_reach(Snapshot &s, const Snapshot &B, const std::vector<uint32_t> &touched_nodes) {
    using build::DevBuf;
    static const bool verbose = getenv("KETO_PATCH_VERBOSE") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char *what) {  // KETO_PATCH_VERBOSE: the walk's parts
        if (!verbose) return;
        KETO_HIP(hipDeviceSynchronize());
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[keto patch]     reach %-10s %.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    DevSnapshot &D = s.dev;
    const DevSnapshot &Bd = B.dev;
    if (!Bd.reach_idx || B.reach_slots.empty() || D.vkey || D.n_ns_x != D.n_ns) return build_reach(s);
    std::vector<uint32_t> base;
    std::vector<uint4> ts;
    const uint64_t n_cand = tabled_slots(s, base, ts);
    if (n_cand != B.reach_cand || base != B.reach_slots) return build_reach(s);  // (the tabled slots changed)
    phase("slots");
    // the touched nodes and their ancestors within cap - 1 hops: a node farther from every
    // touched node reaches one only over a path of more than cap nodes whose edges the patch left
    // alone -- untabled before and after
    static const uint32_t cap = [] {
        const char *e = getenv("KETO_REACH_CAP");
        const uint32_t c = e ? (uint32_t)atoi(e) : REACH_CAP;
        return c >= 1 && c <= REACH_CAP_MAX ? c : REACH_CAP;
    }();
    // (the walk's nodes at most VCAP -- more: rebuild whole; a hash set of 4 VCAP slots, 4 MB +
    // a 2 MB level list: no allocation that grows with the graph)
    constexpr uint32_t VCAP = 1u << 19;
    std::vector<uint32_t> t0(touched_nodes);
    std::sort(t0.begin(), t0.end());
    t0.erase(std::unique(t0.begin(), t0.end()), t0.end());
    if (t0.size() > VCAP / 2) return build_reach(s);
    DevBuf seen(16ull * VCAP + 16), lv(4ull * VCAP + 16), cnt(16);
    KETO_HIP(hipMemset(seen.p, 0, 16ull * VCAP));
    const uint32_t mask = 4 * VCAP - 1;
    uint32_t *all = lv.u32();
    if (!t0.empty()) {
        KETO_HIP(hipMemcpy(all, t0.data(), 4 * t0.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_seen_init, dim3((uint32_t)std::min<uint64_t>(1024, (t0.size() + RB - 1) / RB)), dim3(RB), 0, 0, all,
                           (uint32_t)t0.size(), seen.u32(), mask);
        KETO_HIP(hipGetLastError());
    }
    uint64_t total = t0.size(), lo = 0;
    std::vector<uint32_t> ri(s.relinfo);  // (the slot flags of the new tables, before reach_bits sets them)
    for (size_t g = 0; g < ri.size(); g++) ri[g] = (ri[g] & ~RI_REACH) | (base[g] != NONE32 ? RI_REACH : 0u);
    DevBuf d_ri(4 * std::max<size_t>(1, ri.size()) + 16);
    if (!ri.empty()) KETO_HIP(hipMemcpy(d_ri.p, ri.data(), 4 * ri.size(), hipMemcpyHostToDevice));
    for (uint32_t level = 1; level < cap && lo < total; level++) {
        const uint64_t n = total - lo;
        KETO_HIP(hipMemset(cnt.p, 0, 4));
        hipLaunchKernelGGL(k_anc_level, dim3((uint32_t)std::min<uint64_t>(4096, (n + RB - 1) / RB)), dim3(RB), 0, 0, all + lo, (uint32_t)n,
                           D.rev_off, D.reloc, D.rev_nodes, D.n_uuids, D.ns, D.n_ns, d_ri.u32(), seen.u32(), mask, all + total, cnt.u32(),
                           (uint32_t)(VCAP - total));
        KETO_HIP(hipGetLastError());
        uint32_t got = 0;
        KETO_HIP(hipMemcpy(&got, cnt.p, 4, hipMemcpyDeviceToHost));
        if (total + got > VCAP) return build_reach(s);
        lo = total;
        total += got;
    }
    phase("ancestors");
    // their candidates, walked again into a copy of the base's tables with the new lists appended
    DevBuf cl(4 * total + 16), d_base(4ull * base.size() + 16), d_ts(16 * ts.size()), lens(4 * total + 16), tot(16);
    KETO_HIP(hipMemcpy(d_base.p, base.data(), 4ull * base.size(), hipMemcpyHostToDevice));
    KETO_HIP(hipMemcpy(d_ts.p, ts.data(), 16 * ts.size(), hipMemcpyHostToDevice));
    KETO_HIP(hipMemset(cnt.p, 0, 4));
    KETO_HIP(hipMemset(tot.p, 0, 16));
    if (total)
        hipLaunchKernelGGL(k_cand_of, dim3((uint32_t)std::min<uint64_t>(4096, (total + RB - 1) / RB)), dim3(RB), 0, 0, all, (uint32_t)total,
                           D.ns, D.n_ns, d_base.u32(), cl.u32(), cnt.u32());
    KETO_HIP(hipGetLastError());
    uint32_t nc = 0;
    KETO_HIP(hipMemcpy(&nc, cnt.p, 4, hipMemcpyDeviceToHost));
    ReachIn R{D.set_row, D.set_dst, D.edge_mask, D.ns, D.n_ns, D.relinfo, static_cast<const uint4 *>(d_ts.p), (uint32_t)ts.size(),
              n_cand, cap, NONE32};
    const dim3 grid((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(65536, ((uint64_t)nc + RB / 64 - 1) / (RB / 64))));
    // a copy of the base's records, or (an advance) the snapshot's own, rewritten where they lie
    const bool in_place = &s == &B && s.sole(D.reach_idx) && s.sole(D.reach_pool);
    const uint64_t base_pool_n = B.reach_pool_n;
    uint4 *idx = in_place ? const_cast<uint4 *>(D.reach_idx) : static_cast<uint4 *>(s.alloc(16 * n_cand + 16));
    if (!in_place) KETO_HIP(hipMemcpy(idx, Bd.reach_idx, 16 * n_cand, hipMemcpyDeviceToDevice));
    if (nc) {
        hipLaunchKernelGGL(k_reach<false>, grid, dim3(RB), 0, 0, R, cl.u32(), (uint64_t)nc, idx, lens.u32(), nullptr, 0u,
                           static_cast<unsigned long long *>(tot.p));
        KETO_HIP(hipGetLastError());
    }
    unsigned long long cn[2] = {0, 0};
    KETO_HIP(hipMemcpy(cn, tot.p, 16, hipMemcpyDeviceToHost));
    const uint64_t pool_n = base_pool_n + cn[0];
    if (pool_n >= (1ull << 31)) return build_reach(s);
    if (nc) build::scan_excl(lens.u32(), nc);
    uint32_t *pool;
    uint64_t pool_cap = pool_n;
    if (in_place && pool_n <= s.reach_pool_cap) {
        pool = const_cast<uint32_t *>(D.reach_pool);  // appended past the entries in use
        pool_cap = s.reach_pool_cap;
    } else {
        if (in_place) pool_cap = pool_n + pool_n / 16 + (1u << 16);
        pool = static_cast<uint32_t *>(s.alloc(4 * pool_cap + 16));
        if (base_pool_n) KETO_HIP(hipMemcpy(pool, Bd.reach_pool, 4 * base_pool_n, hipMemcpyDeviceToDevice));
        if (in_place) s.drop(D.reach_pool);
    }
    if (nc) {
        hipLaunchKernelGGL(k_reach<true>, grid, dim3(RB), 0, 0, R, cl.u32(), (uint64_t)nc, idx, lens.u32(), pool,
                           (uint32_t)base_pool_n, nullptr);
        KETO_HIP(hipGetLastError());
    }
    if (verbose) fprintf(stderr, "[keto patch]     reach: %zu touched nodes, %llu with ancestors, %u tabled walked again\n", t0.size(),
                         (unsigned long long)total, nc);
    phase("walks");
    if (!in_place) {  // (in place: the same slots, the same array)
        uint32_t *db = static_cast<uint32_t *>(s.alloc(4ull * base.size() + 16));
        KETO_HIP(hipMemcpy(db, base.data(), 4ull * base.size(), hipMemcpyHostToDevice));
        D.reach_base = db;
    }
    KETO_HIP(hipStreamSynchronize(nullptr));
    D.reach_idx = idx;
    D.reach_pool = pool;
    reach_bits(s, base);
    s.reach_slots = std::move(base);
    s.reach_cand = n_cand;
    s.reach_pool_n = pool_n;
    s.reach_pool_cap = pool_cap;
    if (&s != &B) s.reach_pool_built = B.reach_pool_built;  // (a copy patch: the base's build)
    KETO_HIP(hipMemset(cnt.p, 0, 8));
    hipLaunchKernelGGL(k_count_tabled, dim3((uint32_t)std::min<uint64_t>(4096, (n_cand + RB - 1) / RB)), dim3(RB), 0, 0, idx, n_cand,
                       static_cast<unsigned long long *>(cnt.p));
    KETO_HIP(hipGetLastError());
    unsigned long long nt = 0;
    KETO_HIP(hipMemcpy(&nt, cnt.p, 8, hipMemcpyDeviceToHost));
    s.info.n_reach = nt;
}

}  // namespace keto
