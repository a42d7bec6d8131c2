// gfx950 batched Check for rewrite-free namespace configs (legacy / union-only Zanzibar).
//
// Without userset rewrites the reference recursion (engine.go:102-249) collapses to:
//   checkIsAllowed(n, d)  = [direct(n, d-1)] || expandSubject(n, d-1)
//   expandSubject(n, d)   = found-lookahead over n's subject-set row, then for each child c
//                           (visited-pruned, width-truncated) checkIsAllowed(c, d, skipDirect)
// Every group is an OR whose first IsMember/Err ends the WHOLE query, there is exactly one
// visited scope per query (opened by the root's expandSubject), and the only frames are
// expand-subject frames.  That makes a compact lane-per-query state machine: few states,
// small live state (<= 64 VGPRs target: 8 waves/SIMD), two independent 16-byte loads per
// step issued by every lane in the same instructions, frames of 32 B that carry the rest of
// the parent's edge window so returning from a child needs no edge reload.
//
// Child order is the reference's (oracle/refsem.c SCHED_EAGER): checkgroup's Add returns as
// soon as child k is handed to the group's consumer (concurrent_checkgroup.go:150-159), so the
// loop of engine.go:151-162 marks the following siblings visited -- up to the next one that
// was not -- before child k runs.  The lane keeps that next sibling `pend`ing (already marked)
// while child k runs.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace {

#ifndef KETO_GUARD
#define KETO_GUARD 8
#endif
// Tier-0 resident blocks per CU (4 x 256 lanes = 4 waves per SIMD), below the 6 the register
// budget allows, as in check.hip.  C2 tier-0 kernel at 4 / 5 / 6 blocks per CU: 7.72 / 7.78 /
// 7.94 ms.
#ifndef KETO_T0_BLOCKS_PER_CU
#define KETO_T0_BLOCKS_PER_CU 4
#endif

enum UState : uint32_t {
    U_IDLE = 0,
    U_START,   // start record of the resolve pre-pass (2 x 16 B)
    U_DPROBE,  // checkDirect of the root via the probe hash
    U_ROWOFF,  // {begin, end} of the current node's subject-set row
    U_SCAN,    // edge window of the found-lookahead
    U_SPROBE,  // hash probes of the lookahead (2 per step)
    U_CEDGE,   // edge window of the child loop
    U_VKEY,    // visited alias key
    U_VIS,     // visited slot pair
    U_POP,     // parent frame (2 x 16 B)
    U_DISP = 200,  // pseudo: the advance found the next unvisited sibling `nx` (or none)
};

// bit of the depth word: the current window is a row descriptor's two inline edges
// (set by U_ROWOFF for U_SCAN; kept in pushed frames so U_POP restores the window origin)
constexpr uint32_t FR_INLINE = 1u << 16;

struct UParams {
    DevSnapshot s;
    const uint4 *start;  // resolve pre-pass records, in work order
    const uint32_t *qlist;
    const uint32_t *qlist_count;
    uint32_t n;
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *next;
    uint32_t *ovf_list;
    uint32_t *ovf_count;
    unsigned long long *vis;
    uint4 *stack;  // 2 x uint4 per frame
    uint32_t *epochs;
    uint32_t vcap, scap;
    int32_t max_depth, max_width;
    unsigned long long *counters;
    uint32_t last_tier;
    uint32_t live_lanes;  // lanes [live_lanes, 64) of every wave take no queries
    uint32_t err_detail;
};

// word j (0..7) of the two consecutive windows v0, v1 -- selects, no scratch
__device__ __forceinline__ uint32_t w8(const uint4 &v0, const uint4 &v1, uint32_t j) {
    return j < 4 ? wword(v0, j) : wword(v1, j - 4);
}

__device__ __forceinline__ uint32_t probe_check(const uint4 &b, uint64_t key) {
    const uint64_t k0 = (uint64_t)b.x | ((uint64_t)b.y << 32), k1 = (uint64_t)b.z | ((uint64_t)b.w << 32);
    if (k0 == key || k1 == key) return 1;
    if (k0 == 0 || k1 == 0) return 0;
    return 2;
}

template <bool COUNT, bool LDS_TABLES>
__global__ __launch_bounds__(256) void check_union_kernel(UParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * 2 * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t pmask = (P.vcap >> 1) - 1;
    const uint32_t W = (uint32_t)P.max_width;
    const uint32_t lane = __lane_id();

    uint32_t q = 0, pos = 0, st = U_IDLE;
    bool exhausted = lane >= P.live_lanes;
    uint32_t sidx = NONE32;  // subject
    bool heavy = false;
    uint32_t R0 = NONE32, R1 = NONE32, R2 = NONE32, R3 = NONE32;
    // current expand-subject frame: node, cursor, end, depth, row begin; edge window
    uint32_t node = 0, cur = 0, end = 0, d = 0, rbeg = 0;
    uint4 ew = make_uint4(0, 0, 0, 0);
    uint32_t ew_lo = 1, ew_hi = 0;
    uint32_t sp = 0, vcount = 0, aux = 0, aux2 = 0;  // aux: probe bucket / visited pair
    uint32_t vk = 0;                                  // visited key of the child being inserted
    uint32_t pend = NONE32, nx = NONE32;              // marked sibling waiting to run / just found
    bool root_ss = false;
    const uint4 *la0 = nullptr, *la1 = nullptr;
    uint32_t ln = 0;
    uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
    unsigned long long c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0, c_wsteps = 0, c_lsteps = 0;

    while (true) {
        const bool need = (st == U_IDLE) && !exhausted;
        const unsigned long long mask = __ballot(need);
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(P.next, (uint32_t)__popcll(mask));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t my = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                if (my >= nq) exhausted = true;
                else {
                    pos = P.qlist ? P.qlist[my] : my;
                    st = U_START;
                    la0 = P.start + 2 * (size_t)pos;
                    la1 = la0 + 1;
                    ln = 2;
                    q_rows = q_edges = q_probes = 0;
                }
            }
        }
        if (__ballot(st != U_IDLE) == 0) break;
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        if (ln > 0) v0 = *la0;
        if (ln > 1) v1 = *la1;
        ln = 0;
        if (COUNT) {
            c_wsteps += lane == 0 ? 1 : 0;
            c_lsteps += st != U_IDLE ? 1 : 0;
        }
        if (st == U_IDLE) continue;

        // result: 0 = keep going, 1 = allowed, 2 = denied, 3 = relation error, 4 = overflow
        uint32_t fin = 0;
        // At most KETO_GUARD transitions per step; the rest carry over to the next step.  U_SCAN
        // entered by a transition reads its window from v0, which does not survive the step
        // boundary: such a lane always runs it before leaving.
        for (int guard = 0; (guard < KETO_GUARD || st == U_SCAN) && ln == 0 && fin == 0; guard++) {
            switch (st) {
            case U_START: {
                node = v0.x;
                sidx = v0.y;
                d = v0.z & 0xFFFFu;
                heavy = (v0.z & START_HEAVY) != 0;
                q = v0.w;
                R0 = v1.x;
                R1 = v1.y;
                R2 = v1.z;
                R3 = v1.w;
                // root checkIsAllowed(node, d, false) (engine.go:214-249)
                const NodeInfo ni = t_node_info(T, node);
                if (ri_status(ni.ri) == REL_ERROR) {
                    aux = t_relname(s, T, node, ni);
                    fin = 3;
                    break;
                }
                root_ss = ri_ss(ni.ri);
                if (d > 1) {  // checkDirect(d-1) (engine.go:167-208)
                    if (COUNT) q_probes++;
                    if (!(node & VIRT_BIT)) {
                        if (!heavy) {
                            if (R0 == node || R1 == node || R2 == node || R3 == node) {
                                fin = 1;
                                break;
                            }
                        } else {
                            aux = (uint32_t)mix64((((uint64_t)sidx << 32) | node) + 1) & s.probe_mask;
                            la0 = s.probe + aux;
                            ln = 1;
                            st = U_DPROBE;
                            break;
                        }
                    }
                }
                if (!root_ss || d <= 1) {
                    fin = 2;
                    break;
                }
                d -= 1;  // checkExpandSubject(root, d-1)
                epoch++;  // the query's one visited scope (graph_utils.go:38-43)
                vcount = 0;
                sp = 0;
                st = U_ROWOFF + 100;
                break;
            }
            case U_DPROBE: {
                const uint32_t r = probe_check(v0, (((uint64_t)sidx << 32) | node) + 1);
                if (r == 2) {
                    aux = (aux + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    break;
                }
                if (r == 1) {
                    fin = 1;
                    break;
                }
                if (!root_ss || d <= 1) {
                    fin = 2;
                    break;
                }
                d -= 1;
                epoch++;
                vcount = 0;
                sp = 0;
                st = U_ROWOFF + 100;
                break;
            }
            case U_ROWOFF + 100:  // enter expand-subject(node, d): rows (traverser.go:53-121)
                if (COUNT) q_rows++;
                if (node & VIRT_BIT) {
                    st = U_POP + 100;  // empty row: not a member, return
                    break;
                }
                la0 = s.set_row + node;
                ln = 1;
                st = U_ROWOFF;
                break;
            case U_ROWOFF:  // {begin, end, edge 0, edge 1}: the first two edges come inline
                rbeg = v0.x;
                end = v0.y;
                cur = rbeg;
                if (rbeg == end) {
                    st = U_POP + 100;
                    break;
                }
                v0 = make_uint4(v0.z, v0.w, NONE32, NONE32);
                d |= FR_INLINE;
                st = U_SCAN;
                break;
            case U_SCAN: {  // found-lookahead over one window (traverser.go:73-80, 109-111)
                ew = v0;
                if (d & FR_INLINE) {
                    d &= ~FR_INLINE;
                    ew_lo = cur;
                    ew_hi = cur + 2;
                } else {
                    ew_lo = cur - (uint32_t)((reinterpret_cast<uintptr_t>(s.set_dst + cur) >> 2) & 3);
                    ew_hi = ew_lo + 4;
                }
                if (!heavy) {
                    bool found = false;
                    while (cur < end && cur < ew_hi) {
                        const uint32_t c = wword(ew, cur - ew_lo) & s.edge_mask;
                        cur++;
                        if (COUNT) {
                            q_edges++;
                            q_probes++;
                        }
                        if (R0 == c || R1 == c || R2 == c || R3 == c) {
                            found = true;
                            break;
                        }
                    }
                    if (found) {
                        fin = 1;
                        break;
                    }
                } else if (cur < end) {  // two probes per step, in edge order
                    const uint32_t c0 = wword(ew, cur - ew_lo) & s.edge_mask;
                    aux = (uint32_t)mix64((((uint64_t)sidx << 32) | c0) + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    if (cur + 1 < end && cur + 1 < ew_hi) {
                        const uint32_t c1 = wword(ew, cur + 1 - ew_lo) & s.edge_mask;
                        aux2 = (uint32_t)mix64((((uint64_t)sidx << 32) | c1) + 1) & s.probe_mask;
                        la1 = s.probe + aux2;
                        ln = 2;
                    }
                    st = U_SPROBE;
                    break;
                }
                if (cur < end) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    break;
                }
                // lookahead done: width truncation, then the child loop (engine.go:141-162)
                if (end - rbeg > W) end = rbeg + (W > 0 ? W - 1 : 0);
                cur = rbeg;
                pend = NONE32;
                st = U_CEDGE + 100;
                break;
            }
            case U_SPROBE: {
                const uint32_t c0 = wword(ew, cur - ew_lo) & s.edge_mask;
                uint32_t r0 = probe_check(v0, (((uint64_t)sidx << 32) | c0) + 1);
                uint32_t r1 = 0;
                const bool two = cur + 1 < end && cur + 1 < ew_hi;
                uint32_t c1 = 0;
                if (two) {
                    c1 = wword(ew, cur + 1 - ew_lo) & s.edge_mask;
                    r1 = probe_check(v1, (((uint64_t)sidx << 32) | c1) + 1);
                }
                if (r0 == 2 || r1 == 2) {  // full buckets: continue those probes (rare)
                    if (r0 == 2) aux = (aux + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    if (two) {
                        if (r1 == 2) aux2 = (aux2 + 1) & s.probe_mask;
                        la1 = s.probe + aux2;
                        ln = 2;
                    }
                    break;
                }
                if (COUNT) {
                    q_edges++;
                    q_probes++;
                }
                if (r0 == 1) {
                    fin = 1;
                    break;
                }
                cur++;
                if (two) {
                    if (COUNT) {
                        q_edges++;
                        q_probes++;
                    }
                    if (r1 == 1) {
                        fin = 1;
                        break;
                    }
                    cur++;
                }
                if (cur < end && cur < ew_hi) {  // rest of the cached window
                    v0 = ew;
                    st = U_SCAN;
                    break;
                }
                if (cur < end) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    st = U_SCAN;
                    break;
                }
                if (end - rbeg > W) end = rbeg + (W > 0 ? W - 1 : 0);
                cur = rbeg;
                pend = NONE32;
                st = U_CEDGE + 100;
                break;
            }
            case U_CEDGE + 100: {  // advance: mark the next children until one was not visited (engine.go:151-160)
                if (cur >= end) {
                    nx = NONE32;
                    st = U_DISP;
                    break;
                }
                if (cur < ew_lo || cur >= ew_hi) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    st = U_CEDGE;
                    break;
                }
                const uint32_t raw = wword(ew, cur - ew_lo);
                cur++;
                aux2 = raw & s.edge_mask;  // child node
                if (raw & EDGE_ALIAS) {
                    la0 = win(s.vkey, aux2);
                    ln = 1;
                    st = U_VKEY;
                    break;
                }
                vk = aux2;
                aux = (uint32_t)mix64(vk) & pmask;
                la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                ln = 1;
                st = U_VIS;
                break;
            }
            case U_CEDGE:
                ew = v0;
                ew_lo = cur - (uint32_t)((reinterpret_cast<uintptr_t>(s.set_dst + cur) >> 2) & 3);
                ew_hi = ew_lo + 4;
                st = U_CEDGE + 100;
                break;
            case U_VKEY:
                vk = pick(s.vkey, aux2, v0);
                aux = (uint32_t)mix64(vk) & pmask;
                la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                ln = 1;
                st = U_VIS;
                break;
            case U_VIS: {  // CheckAndAddVisited (graph_utils.go:45-53), epoch-tagged
                const unsigned long long tag = ((unsigned long long)epoch << 32) | vk;
                const unsigned long long s0 = (unsigned long long)v0.x | ((unsigned long long)v0.y << 32);
                const unsigned long long s1 = (unsigned long long)v0.z | ((unsigned long long)v0.w << 32);
                const bool e0 = (uint32_t)(s0 >> 32) != epoch, e1 = (uint32_t)(s1 >> 32) != epoch;
                if (s0 == tag || (!e0 && s1 == tag)) {
                    st = U_CEDGE + 100;  // already visited
                    break;
                }
                if (!e0 && !e1) {
                    aux = (aux + 1) & pmask;
                    la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                    ln = 1;
                    break;
                }
                if (2 * (vcount + 1) > P.vcap) {
                    fin = 4;
                    break;
                }
                vis[2 * aux + (e0 ? 0 : 1)] = tag;
                vcount++;
                nx = aux2;
                st = U_DISP;
                break;
            }
            case U_DISP: {  // run the pending child; the one just found becomes pending
                if (pend == NONE32) {
                    if (nx == NONE32) {
                        st = U_POP + 100;  // no child left: NotMember
                        break;
                    }
                    pend = nx;  // the loop's first child: find its successor before it runs
                    st = U_CEDGE + 100;
                    break;
                }
                const uint32_t c = pend;
                pend = nx;
                // child checkIsAllowed(c, d, skipDirect=true) -> expandSubject(c, d-1) (engine.go:161)
                const NodeInfo ni = t_node_info(T, c);
                if (ri_status(ni.ri) == REL_ERROR) {
                    aux = t_relname(s, T, c, ni);
                    fin = 3;
                    break;
                }
                if (!ri_ss(ni.ri) || d <= 1) {  // empty group / Unknown: not a member
                    st = pend == NONE32 ? U_POP + 100 : U_CEDGE + 100;
                    break;
                }
                if (sp + 1 >= P.scap) {
                    fin = 4;
                    break;
                }
                // push the parent: cursor, end, depth, window end | the pending sibling and the
                // window's edges from the cursor on (at most 3: the window held edge cur-1)
                const bool inwin = cur >= ew_lo && cur < ew_hi;
                const uint32_t k0 = inwin ? cur - ew_lo : 0;
                stk[2 * sp] = make_uint4(cur, end, d, inwin ? ew_hi : cur);
                stk[2 * sp + 1] = make_uint4(pend, inwin ? wword(ew, k0) : NONE32,
                                             inwin && k0 + 1 < 4 ? wword(ew, k0 + 1) : NONE32,
                                             inwin && k0 + 2 < 4 ? wword(ew, k0 + 2) : NONE32);
                sp++;
                node = c;
                d -= 1;
                st = U_ROWOFF + 100;
                break;
            }
            case U_POP + 100:  // expand-subject returned NotMember
                if (sp == 0) {
                    fin = 2;
                    break;
                }
                sp--;
                la0 = stk + 2 * sp;
                la1 = la0 + 1;
                ln = 2;
                st = U_POP;
                break;
            case U_POP:  // a child returned NotMember: run the pending sibling next
                cur = v0.x;
                end = v0.y;
                d = v0.z & 0xFFFFu;
                ew_lo = cur;
                ew_hi = v0.w;
                pend = v1.x;
                ew = make_uint4(v1.y, v1.z, v1.w, NONE32);
                st = pend == NONE32 ? U_POP + 100 : U_CEDGE + 100;
                break;
            default:
                fin = 4;
            }
        }
        if (fin) {
            if (fin == 4) {
                if (P.last_tier) {
                    P.out_allowed[q] = 0;
                    P.out_err[q] = KETO_QERR_INTERNAL;
                } else {
                    P.ovf_list[atomicAdd(P.ovf_count, 1u)] = pos;
                }
            } else {
                P.out_allowed[q] = fin == 1 ? 1 : 0;
                P.out_err[q] = fin == 3 ? (int32_t)(KETO_QERR_NO_RELATION | (P.err_detail ? aux << 8 : 0u)) : 0;
                if (COUNT) {
                    c_rows += q_rows;
                    c_edges += q_edges;
                    c_probes += q_probes;
                    c_q++;
                }
            }
            st = U_IDLE;
            ln = 0;
        }
    }
    P.epochs[gl] = epoch;
    if (COUNT) {
        for (int off = 32; off > 0; off >>= 1) {
            c_rows += __shfl_down(c_rows, off);
            c_edges += __shfl_down(c_edges, off);
            c_probes += __shfl_down(c_probes, off);
            c_q += __shfl_down(c_q, off);
            c_lsteps += __shfl_down(c_lsteps, off);
        }
        if (lane == 0) {
            atomicAdd(&P.counters[0], c_rows);
            atomicAdd(&P.counters[1], c_edges);
            atomicAdd(&P.counters[2], c_probes);
            atomicAdd(&P.counters[4], c_q);
            atomicAdd(&P.counters[5], c_wsteps);
            atomicAdd(&P.counters[6], c_lsteps);
        }
    }
}

}  // namespace

void run_check_union(const Snapshot &s, Stream &st, const CheckLaunch &L) {
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    constexpr uint32_t BLOCK = 256;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    // HBM is plentiful (288 GB): tier 0 holds ~500 visited nodes per lane so restarts are rare
    const Tier t[3] = {Tier{cus * KETO_T0_BLOCKS_PER_CU * 256, 1024, 32},  // the persistent grid's lanes
                       Tier{cus * 64, 1u << 13, 512},
                       Tier{64, 1u << 20, 1u << 14}};
    ensure_scratch(st.union_scratch, t);
    run_resolve(s, st, L.queries, L.n, L.max_depth);
    Scratch &sc = st.union_scratch;
    uint32_t *list[2] = {st.lists, st.lists + st.list_cap};
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? s.dev.lds_bytes : 0;
    KETO_HIP(hipMemsetAsync(sc.ctrl, 0, 64, st.stream));
    for (int tier = 0; tier < 3; tier++) {
        UParams P{};
        P.s = s.dev;
        P.start = st.resolved;
        P.qlist = tier == 0 ? nullptr : list[tier - 1];
        P.qlist_count = tier == 0 ? nullptr : &sc.ctrl[3 + tier - 1];
        P.n = (uint32_t)L.n;
        P.out_allowed = L.out_allowed;
        P.out_err = L.out_err;
        P.next = &sc.ctrl[tier];
        P.ovf_list = tier < 2 ? list[tier] : nullptr;
        P.ovf_count = tier < 2 ? &sc.ctrl[3 + tier] : nullptr;
        P.vis = sc.vis[tier];
        P.stack = sc.stack[tier];
        P.epochs = sc.epochs[tier];
        P.vcap = t[tier].vcap;
        P.scap = t[tier].scap / 2;  // frames are 2 x uint4
        P.max_depth = L.max_depth;
        P.max_width = L.max_width;
        P.counters = st.counters + 8 * tier;
        P.last_tier = tier == 2;
        P.err_detail = L.err_detail;
        uint32_t lanes = t[tier].lanes;
        if (tier == 0) {  // persistent grid: exactly the resident blocks (occupancy API), capped by the batch
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&check_union_kernel<false, true>),
                                                             BLOCK, lds) != hipSuccess || per_cu <= 0)
                per_cu = 4;
            per_cu = std::min(per_cu, KETO_T0_BLOCKS_PER_CU);
            lanes = std::min<uint32_t>(lanes, (uint32_t)per_cu * cus * BLOCK);
            // a batch smaller than the resident grid is spread over more waves with fewer live
            // lanes each (check.hip: fewer distinct interpreter states per wave-step)
            const uint64_t waves = lanes / 64;
            P.live_lanes = (uint32_t)std::min<uint64_t>(64, (L.n + waves - 1) / waves);
            const uint64_t need = (L.n + P.live_lanes - 1) / P.live_lanes * 64;
            lanes = (uint32_t)std::min<uint64_t>(lanes, (need + BLOCK - 1) / BLOCK * BLOCK);
        } else {
            P.live_lanes = 64;
        }
        const uint32_t bs = std::min<uint32_t>(BLOCK, lanes);
        dim3 grid(lanes / bs), block(bs);
        if (tier == 0) st.mark_begin();
        if (lds_tables) {
            if (L.count) hipLaunchKernelGGL((check_union_kernel<true, true>), grid, block, lds, st.stream, P);
            else hipLaunchKernelGGL((check_union_kernel<false, true>), grid, block, lds, st.stream, P);
        } else {
            if (L.count) hipLaunchKernelGGL((check_union_kernel<true, false>), grid, block, 0, st.stream, P);
            else hipLaunchKernelGGL((check_union_kernel<false, false>), grid, block, 0, st.stream, P);
        }
        KETO_HIP(hipGetLastError());
        if (tier == 0) st.mark_end();
    }
}

}  // namespace keto
