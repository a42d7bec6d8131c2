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
// Snapshots whose visited keys alias (D.vkey) and partitions (ghost rows live elsewhere) carry
// none.  Layout: reach_base[global slot] = first entry of the slot in reach_idx (NONE32: not
// tabled), reach_idx[base + entity - ent_base] = {offset, count} (count NONE32: not tabled) into
// reach_pool, the reach without the node itself (its own row is what the caller tested).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

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

// slots some subject-set edge points into
__global__ __launch_bounds__(RB) void k_slot_targets(const uint32_t *set_dst, uint64_t n, uint32_t edge_mask, const NsDev *ns,
                                                     uint32_t n_ns, uint32_t *flag) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = set_dst[i] & edge_mask;
        const NsDev nd = ns[ns_of_node(ns, n_ns, c)];
        const uint32_t g = nd.slot_base + (c - nd.node_base) % nd.n_slots;
        if (!flag[g]) atomicOr(&flag[g], 1u);  // (read first: most edges find the flag set)
    }
}

// One wave per candidate node: a breadth-first walk of its reach with the list in registers
// (entry k on lane k % 64, register k / 64).  Pass 1 (FILL = false) counts, pass 2 writes the
// list at the offset pass 1's scan gave.
template <bool FILL>
__global__ __launch_bounds__(RB) void k_reach(ReachIn R, uint2 *idx, uint32_t *lens, uint32_t *pool, unsigned long long *total) {
    static_assert(REACH_CAP <= 128, "two list registers per lane");
    const uint32_t wpb = blockDim.x >= 64 ? blockDim.x / 64 : 1;  // (the CPU emulation: one-lane blocks)
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    for (uint64_t t = (uint64_t)blockIdx.x * wpb + threadIdx.x / 64; t < R.n_cand; t += nw) {
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
        uint32_t L[REACH_CAP];
        L[0] = g;
        while (ok && head < cnt) {
            const uint32_t n = L[head++];
            if (!node_pure(R, n)) {
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
                if (cnt == REACH_CAP) ok = false;
                else L[cnt++] = c;
            }
        }
        if constexpr (!FILL) {
            lens[t] = ok ? cnt - 1 : 0u;
            idx[t] = make_uint2(0u, ok ? cnt - 1 : NONE32);
            if (ok && cnt > 1) atomicAdd(total, (unsigned long long)(cnt - 1));
            if (ok) atomicAdd(total + 1, 1ull);
        } else if (ok) {
            const uint32_t off = lens[t];
            for (uint32_t k = 1; k < cnt; k++) pool[off + k - 1] = L[k];
            idx[t].x = off;
        }
#else
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t e0 = lane == 0 ? g : NONE32, e1 = NONE32;
        while (ok && head < cnt) {
            const uint32_t n = __shfl(head < 64 ? e0 : e1, (int)(head & 63u));
            head++;
            if (!node_pure(R, n)) {
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
                    if (cnt == REACH_CAP) {
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
        if constexpr (!FILL) {
            if (lane == 0) {
                lens[t] = ok ? cnt - 1 : 0u;
                idx[t] = make_uint2(0u, ok ? cnt - 1 : NONE32);
                if (ok && cnt > 1) atomicAdd(total, (unsigned long long)(cnt - 1));
                if (ok) atomicAdd(total + 1, 1ull);
            }
        } else if (ok) {
            const uint32_t off = lens[t];  // (pass 1's counts, scanned)
            if (lane >= 1 && lane < cnt) pool[off + lane - 1] = e0;
            if (64 + lane < cnt) pool[off + 63 + lane] = e1;
            if (lane == 0) idx[t].x = off;
        }
#endif
    }
}

}  // namespace

// The tables of snapshot s (its rows, relation info and ns table are on the device); nothing
// when none of its slots qualifies, its visited keys alias, or KETO_NO_REACH is set (A/B runs:
// the oracle's RS_NO_REACH).  s.dev.reach_* are set, allocated through s.
void build_reach(Snapshot &s) {
    using build::DevBuf;
    DevSnapshot &D = s.dev;
    D.reach_base = nullptr;
    D.reach_idx = nullptr;
    D.reach_pool = nullptr;
    s.info.n_reach = 0;
    static const bool off = [] {
        const char *e = getenv("KETO_NO_REACH");
        return e && *e == '1';
    }();
    const uint32_t n_slots = (uint32_t)s.relinfo.size();
    if (off || D.vkey || D.n_ns_x != D.n_ns || !n_slots || !s.info.n_set_edges) return;
    std::vector<uint32_t> target(n_slots, 0);
    {
        DevBuf flag(4ull * n_slots);
        KETO_HIP(hipMemset(flag.p, 0, 4ull * n_slots));
        const uint64_t ne = s.info.n_set_edges;
        hipLaunchKernelGGL(k_slot_targets, dim3((uint32_t)std::min<uint64_t>(8192, (ne + RB - 1) / RB)), dim3(RB), 0, 0, D.set_dst,
                           ne, D.edge_mask, D.ns, D.n_ns, flag.u32());
        KETO_HIP(hipGetLastError());
        KETO_HIP(hipMemcpy(target.data(), flag.p, 4ull * n_slots, hipMemcpyDeviceToHost));
    }
    std::vector<uint32_t> base(n_slots, NONE32);
    std::vector<uint4> ts;
    uint64_t n_cand = 0;
    for (uint32_t ns = 0; ns < s.n_ns; ns++)
        for (uint32_t k = 0; k < s.ns[ns].n_slots; k++) {
            const uint32_t g = s.ns[ns].slot_base + k, ri = s.relinfo[g];
            if (!target[g] || !ri_setrows(ri) || ri_rw(ri) || ri_status(ri) == REL_ERROR) continue;
            base[g] = (uint32_t)n_cand;
            ts.push_back(make_uint4((uint32_t)n_cand, ns, k, 0));
            n_cand += s.ns[ns + 1].ent_base - s.ns[ns].ent_base;
            if (n_cand >= (1ull << 31)) return;  // (past the index's range: no tables)
        }
    if (ts.empty()) return;
    uint2 *idx = static_cast<uint2 *>(s.alloc(8 * n_cand + 16));
    DevBuf lens(4 * n_cand + 16), tot(16), d_ts(16 * ts.size());
    KETO_HIP(hipMemset(tot.p, 0, 16));
    KETO_HIP(hipMemcpy(d_ts.p, ts.data(), 16 * ts.size(), hipMemcpyHostToDevice));
    ReachIn R{D.set_row, D.set_dst, D.edge_mask, D.ns, D.n_ns, D.relinfo, static_cast<const uint4 *>(d_ts.p), (uint32_t)ts.size(),
              n_cand};
    const dim3 grid((uint32_t)std::min<uint64_t>(65536, (n_cand + RB / 64 - 1) / (RB / 64)));  // (4 waves a block)
    hipLaunchKernelGGL(k_reach<false>, grid, dim3(RB), 0, 0, R, idx, lens.u32(), nullptr,
                       static_cast<unsigned long long *>(tot.p));
    KETO_HIP(hipGetLastError());
    unsigned long long cn[2] = {0, 0};
    KETO_HIP(hipMemcpy(cn, tot.p, 16, hipMemcpyDeviceToHost));
    const unsigned long long total = cn[0];
    if (total >= (1ull << 31)) return;  // (the allocation of idx goes back with the snapshot)
    build::scan_excl(lens.u32(), n_cand);
    uint32_t *pool = static_cast<uint32_t *>(s.alloc(4 * total + 16));
    hipLaunchKernelGGL(k_reach<true>, grid, dim3(RB), 0, 0, R, idx, lens.u32(), pool, nullptr);
    KETO_HIP(hipGetLastError());
    uint32_t *d_base = static_cast<uint32_t *>(s.alloc(4ull * n_slots + 16));
    KETO_HIP(hipMemcpy(d_base, base.data(), 4ull * n_slots, hipMemcpyHostToDevice));
    KETO_HIP(hipStreamSynchronize(nullptr));
    D.reach_base = d_base;
    D.reach_idx = idx;
    D.reach_pool = pool;
    s.info.n_reach = cn[1];
}

}  // namespace keto
