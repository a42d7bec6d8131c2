// gfx950 batched Check with OPL userset rewrites: exact one-worker sequential semantics.
//
// The reference evaluates one Check as a recursion of goroutines issuing one SQL
// statement per hop (internal/check/{engine,rewrites,binop}.go).  Here every lane of a
// persistent 64-wide wavefront owns one query and walks the same recursion as an explicit
// stack of 16-byte frames (checkIsAllowed, expandSubject, rewrite, shortcut candidates,
// tuple-to-userset, inverted).  The walk is cut into steps that need at most one dependent
// global round trip: every loop iteration each lane issues its (up to two, independent)
// 16-byte loads in the same instructions as every other lane, then consumes them with
// ALU/LDS work only.  Live state is kept in scalars (no runtime-indexed private arrays,
// no scratch spills) so the kernel keeps a high wave occupancy for latency hiding.
//
// Data placement: CSR rows, reverse rows and the probe hash in HBM (L2 / Infinity Cache
// resident when small); namespace table, relation info and rewrite program in LDS; the
// subject's reverse row in VGPRs when short (<= PROBE_K), else membership = one probe into
// the bucketized hash; per-lane visited sets (epoch-tagged, never cleared) and frame stacks
// in scratch.  Queries whose visited set or stack outgrow a tier are re-run by the next tier
// (bigger scratch, fewer lanes) through an on-device list: no host round trip in a batch.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace {

constexpr uint32_t M_UNK = 0, M_IS = 1, M_NOT = 2;
__device__ __forceinline__ uint32_t mk_err(uint32_t e) { return e << 8; }
__device__ __forceinline__ bool decisive(uint32_t r) { return (r >> 8) != 0 || (r & 3u) == M_IS; }

// frame word w: bits 0-15 depth, 16-19 type, 20-23 phase, 24 skip_direct, 25 visited-scope owner
enum FrameType : uint32_t { F_IA = 0, F_ES = 1, F_RW = 2, F_SC = 3, F_TTU = 4, F_INV = 5 };
// FL_INLINE: S_FSCAN's window is the row descriptor's two inline edges (set by S_ROWOFF)
constexpr uint32_t FL_SKIP = 1u << 24, FL_OWNER = 1u << 25, FL_INLINE = 1u << 26;
__device__ __forceinline__ uint32_t fw(uint32_t type, uint32_t d, uint32_t phase = 0, uint32_t flags = 0) {
    return (d & 0xFFFFu) | (type << 16) | (phase << 20) | flags;
}
__device__ __forceinline__ uint32_t f_d(uint32_t w) { return w & 0xFFFFu; }
__device__ __forceinline__ uint32_t f_type(uint32_t w) { return (w >> 16) & 0xFu; }
__device__ __forceinline__ uint32_t f_phase(uint32_t w) { return (w >> 20) & 0xFu; }
__device__ __forceinline__ uint32_t set_phase(uint32_t w, uint32_t p) { return (w & ~(0xFu << 20)) | (p << 20); }

// ES child loop (oracle/refsem.c SCHED_EAGER): checkgroup's Add returns as soon as child k is
// handed to the group's consumer (concurrent_checkgroup.go:150-159), so engine.go:151-162 marks
// the following siblings -- up to the next one that was not visited -- before child k runs, and
// after a decisive child marks all the rest before its result is sent.  Phase-3 ES frames keep
// {x cursor, y end, z pending sibling (marked, not run yet; NONE32 = none)}; phase 4 = draining.
// lane states; "pseudo" states need no load and are run by the same step loop
enum State : uint32_t {
    S_IDLE = 0,
    S_START,    // start record of the resolve pre-pass (2 x 16 B)
    S_RUN,      // pseudo: execute / resume the top frame
    S_RET,      // pseudo: return `res` to the parent frame
    S_POP,      // parent frame
    S_DPROBE,   // probe-hash answer for checkDirect
    S_ROWOFF,   // {begin, end} of a subject-set row (ES or TTU)
    S_FSCAN,    // edge window of the ES found-lookahead
    S_FPROBE,   // probe-hash answers of the lookahead (<= 2)
    S_ESDONE,   // pseudo: lookahead exhausted -> truncate, open scope, child loop
    S_CNEXT,    // pseudo: ES child loop, next child
    S_CEDGE,    // edge window of the ES child loop
    S_VKEY,     // visited alias key
    S_VIS,      // visited slot pair
    S_TNEXT,    // pseudo: TTU loop, next parent
    S_TEDGE,    // edge window of the TTU loop
    S_SPROBE,   // probe-hash answers of the OR shortcut IN query (<= 2)
    S_CDISP,    // pseudo: the advance found the next unvisited sibling `cc` (NONE32: none left)
};

struct CheckParams {
    DevSnapshot s;
    const uint4 *start;     // resolve pre-pass records, in work order
    const uint32_t *qlist;  // tiers >= 1: start-record positions to (re)run
    const uint32_t *qlist_count;
    uint32_t n;
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *next;  // work-queue head
    uint32_t *ovf_list;
    uint32_t *ovf_count;
    unsigned long long *vis;  // [lanes * vcap]
    uint4 *stack;             // [lanes * scap]
    uint32_t *epochs;         // [lanes]
    uint32_t vcap, scap;
    int32_t max_depth, max_width;
    unsigned long long *counters;
    uint32_t last_tier;
    uint32_t live_lanes;  // lanes [live_lanes, 64) of every wave take no queries
    uint32_t err_detail;
};

#ifndef KETO_GUARD
#define KETO_GUARD 24
#endif
// Tier-0 resident blocks per CU (5 x 256 lanes = 5 waves per SIMD), below the 6 the register
// budget allows: fewer lanes, each running more queries, waste fewer lane-steps in the batch's
// tail.  C4 tier-0 kernel at 3 / 4 / 5 / 6 blocks per CU: 25.1 / 22.6 / 21.6 / 22.0 ms.
#ifndef KETO_T0_BLOCKS_PER_CU
#define KETO_T0_BLOCKS_PER_CU 5
#endif

__device__ __forceinline__ uint32_t w8(const uint4 &v0, const uint4 &v1, uint32_t j) {
    return j < 4 ? wword(v0, j) : wword(v1, j - 4);
}
// one probe bucket: 1 found, 0 absent, 2 continue with the next bucket
__device__ __forceinline__ uint32_t probe_check(const uint4 &b, uint64_t key) {
    const uint64_t k0 = (uint64_t)b.x | ((uint64_t)b.y << 32), k1 = (uint64_t)b.z | ((uint64_t)b.w << 32);
    if (k0 == key || k1 == key) return 1;
    if (k0 == 0 || k1 == 0) return 0;
    return 2;
}

template <bool COUNT, bool LDS_TABLES>
__global__ __launch_bounds__(256) void check_kernel(CheckParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t pmask = (P.vcap >> 1) - 1;
    const uint32_t W = (uint32_t)P.max_width;
    const uint32_t lane = __lane_id();

    uint32_t q = 0, pos = 0, st = S_IDLE;
    bool exhausted = lane >= P.live_lanes;
    uint32_t sidx = NONE32;  // subject
    bool heavy = false;
    uint32_t R0 = NONE32, R1 = NONE32, R2 = NONE32, R3 = NONE32;
    // interpreter
    uint4 top = make_uint4(0, 0, 0, 0);
    uint32_t sp = 0, res = 0, vcount = 0;
    bool have_res = false, scope = false;
    uint4 ew = make_uint4(0, 0, 0, 0);
    uint32_t ew_lo = 1, ew_hi = 0;      // edge indices present in ew
    uint32_t aux = 0, aux2 = 0;         // probe buckets / visited pair
    uint32_t pc0 = 0, pc1 = 0, pn = 0;  // probed nodes, count
    uint32_t cc = 0, vk = 0;            // child node / its visited key
    const uint4 *la0 = nullptr, *la1 = nullptr;
    uint32_t ln = 0;
    uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
    unsigned long long c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0, c_wsteps = 0, c_lsteps = 0;

    while (true) {
        // ---- refill idle lanes: one atomic per wavefront (ballot + mbcnt) --------------------
        const bool need = (st == S_IDLE) && !exhausted;
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
                    st = S_START;
                    la0 = P.start + 2 * (size_t)pos;
                    la1 = la0 + 1;
                    ln = 2;
                    q_rows = q_edges = q_probes = 0;
                }
            }
        }
        if (__ballot(st != S_IDLE) == 0) break;
        // ---- the load slot: every lane's loads in the same instructions ------------------------
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
        if (ln > 0) v0 = *la0;
        if (ln > 1) v1 = *la1;
        ln = 0;
        if (COUNT) {
            c_wsteps += lane == 0 ? 1 : 0;
            c_lsteps += st != S_IDLE ? 1 : 0;
        }
        if (st == S_IDLE) continue;

        // fin: 0 running, 1 finished (res), 2 scratch outgrown
        uint32_t fin = 0;
        // At most KETO_GUARD transitions per step; the rest carry over to the next step.  S_FSCAN
        // entered by a transition reads its window from v0 (set to the cached `ew`), which does
        // not survive the step boundary: such a lane always runs it before leaving.
        for (int guard = 0; (guard < KETO_GUARD || st == S_FSCAN) && ln == 0 && fin == 0; guard++) {
            const uint32_t w = top.w;
            const uint32_t d = f_d(w);
#ifdef KETO_PROF_STATES  // profiling builds only (tools/ab_build.sh, tools/prof_states.py)
            if (COUNT) {     // tiers 1-2 counter slots <- per dispatch key: rounds a wave runs it (1) or lanes in it (2)
                const int lead = __ffsll((long long)__ballot(true)) - 1;
                const uint32_t key = st == S_RUN ? 17 + f_type(w) : st;  // slots 7 and 15 are not exported
                const uint32_t keys[16] = {S_RET, S_POP, S_ROWOFF, S_FSCAN, S_ESDONE, S_CNEXT, S_VIS, S_CEDGE,
                                           S_TNEXT, 17, 18, 19, 20, 21, 22, S_TEDGE};
                for (uint32_t k = 0; k < 16; k++) {
                    const unsigned long long b = __ballot(key == keys[k]);
                    const unsigned long long v = KETO_PROF_STATES == 1 ? (b != 0) : (unsigned long long)__popcll(b);
                    if ((int)lane == lead && v) atomicAdd(&P.counters[8 + k], v);
                }
            }
#endif
            switch (st) {
            // ---------------------------------------------------------------- query entry
            case S_START:
                q = v0.w;
                sidx = v0.y;
                heavy = (v0.z & START_HEAVY) != 0;
                R0 = v1.x;
                R1 = v1.y;
                R2 = v1.z;
                R3 = v1.w;
                top = make_uint4(v0.x, 0, 0, fw(F_IA, v0.z & 0xFFFFu));  // checkIsAllowed(root, d, false)
                sp = 0;
                have_res = false;
                scope = false;
                st = S_RUN;
                break;
            // ---------------------------------------------------------------- returns
            case S_RET:
                if (sp == 0) {
                    fin = 1;  // CheckIsMember (engine.go:65-71)
                    break;
                }
                la0 = stk + (sp - 1);
                ln = 1;
                st = S_POP;
                break;
            case S_POP:
                top = v0;
                sp--;
                have_res = true;
                st = S_RUN;
                break;
            // ---------------------------------------------------------------- loads of frames
            case S_DPROBE: {  // checkDirect via the probe hash (engine.go:167-208)
                const uint32_t r = probe_check(v0, (((uint64_t)sidx << 32) | top.x) + 1);
                if (r == 2) {
                    aux = (aux + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    break;
                }
                if (r == 1) {
                    res = M_IS;
                    st = S_RET;
                    break;
                }
                top.w = set_phase(w, 3);
                st = S_RUN;
                break;
            }
            case S_ROWOFF: {
                const bool is_es = f_type(w) == F_ES;
                const uint32_t b = v0.x, e = v0.y;
                if (b == e) {
                    res = M_NOT;
                    st = S_RET;
                    break;
                }
                ew = make_uint4(v0.z, v0.w, NONE32, NONE32);  // the row's first two edges, inline
                ew_lo = b;
                ew_hi = b + 2;
                if (is_es) {
                    top = make_uint4(b, b, e, set_phase(w, 2) | FL_INLINE);  // x = row begin, y = cursor, z = end
                    v0 = ew;
                    st = S_FSCAN;
                } else {
                    top = make_uint4(top.x, b, e, set_phase(w, 2));  // x = computed relation
                    st = S_TNEXT;
                }
                break;
            }
            case S_FSCAN: {  // found-lookahead over one edge window (traverser.go:73-80, 109-111)
                ew = v0;
                uint32_t cur = top.y;
                const uint32_t e = top.z;
                if (w & FL_INLINE) {  // the row descriptor's edges (entered from S_ROWOFF)
                    top.w &= ~FL_INLINE;
                    ew_lo = cur;
                    ew_hi = cur + 2;
                } else {
                    ew_lo = cur - (uint32_t)((reinterpret_cast<uintptr_t>(s.set_dst + cur) >> 2) & 3);
                    ew_hi = ew_lo + 4;
                }
                if (!heavy) {
                    bool found = false;
                    while (cur < e && cur < ew_hi) {
                        const uint32_t c = wword(ew, cur - ew_lo) & ~EDGE_ALIAS;
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
                    top.y = cur;
                    if (found) {
                        res = M_IS;
                        st = S_RET;
                        break;
                    }
                } else if (cur < e) {  // up to two probes per step, in edge order
                    pc0 = wword(ew, cur - ew_lo) & ~EDGE_ALIAS;
                    aux = (uint32_t)mix64((((uint64_t)sidx << 32) | pc0) + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    pn = 1;
                    if (cur + 1 < e && cur + 1 < ew_hi) {
                        pc1 = wword(ew, cur + 1 - ew_lo) & ~EDGE_ALIAS;
                        aux2 = (uint32_t)mix64((((uint64_t)sidx << 32) | pc1) + 1) & s.probe_mask;
                        la1 = s.probe + aux2;
                        ln = 2;
                        pn = 2;
                    }
                    st = S_FPROBE;
                    break;
                }
                if (cur < e) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    break;  // next window, stay S_FSCAN
                }
                st = S_ESDONE;
                break;
            }
            case S_FPROBE: {
                const uint32_t r0 = probe_check(v0, (((uint64_t)sidx << 32) | pc0) + 1);
                const uint32_t r1 = pn > 1 ? probe_check(v1, (((uint64_t)sidx << 32) | pc1) + 1) : 0;
                if (r0 == 2 || r1 == 2) {  // full buckets: follow them (rare)
                    if (r0 == 2) aux = (aux + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    if (pn > 1) {
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
                    res = M_IS;
                    st = S_RET;
                    break;
                }
                top.y++;
                if (pn > 1) {
                    if (COUNT) {
                        q_edges++;
                        q_probes++;
                    }
                    if (r1 == 1) {
                        res = M_IS;
                        st = S_RET;
                        break;
                    }
                    top.y++;
                }
                if (top.y < top.z) {
                    if (top.y < ew_hi) {
                        v0 = ew;  // rest of the cached window
                        st = S_FSCAN;
                        break;
                    }
                    la0 = win(s.set_dst, top.y);
                    ln = 1;
                    st = S_FSCAN;
                    break;
                }
                st = S_ESDONE;
                break;
            }
            case S_ESDONE: {  // width truncation, visited scope, child loop (engine.go:141-162)
                const uint32_t b = top.x;
                uint32_t e = top.z;
                if (e - b > W) e = b + (W > 0 ? W - 1 : 0);  // results[:maxWidth-1]
                uint32_t flags = 0;
                if (!scope) {  // graph.InitVisited (graph_utils.go:38-43)
                    scope = true;
                    epoch++;
                    vcount = 0;
                    flags = FL_OWNER;
                }
                top = make_uint4(b, e, NONE32, fw(F_ES, d, 3, flags));  // x = cursor, y = end, z = pending
                st = S_CNEXT;
                break;
            }
            case S_CNEXT: {  // advance: mark the next children until one was not visited (engine.go:151-160)
                const uint32_t cur = top.x;
                if (cur >= top.y) {
                    cc = NONE32;
                    st = S_CDISP;
                    break;
                }
                if (cur < ew_lo || cur >= ew_hi) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    st = S_CEDGE;
                    break;
                }
                const uint32_t raw = wword(ew, cur - ew_lo);
                top.x = cur + 1;
                cc = raw & ~EDGE_ALIAS;
                if (raw & EDGE_ALIAS) {
                    la0 = win(s.vkey, cc);
                    ln = 1;
                    st = S_VKEY;
                    break;
                }
                vk = cc;
                aux = (uint32_t)mix64(vk) & pmask;
                la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                ln = 1;
                st = S_VIS;
                break;
            }
            case S_CEDGE:
                ew = v0;
                ew_lo = top.x - (uint32_t)((reinterpret_cast<uintptr_t>(s.set_dst + top.x) >> 2) & 3);
                ew_hi = ew_lo + 4;
                st = S_CNEXT;
                break;
            case S_VKEY:
                vk = pick(s.vkey, cc, v0);
                aux = (uint32_t)mix64(vk) & pmask;
                la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                ln = 1;
                st = S_VIS;
                break;
            case S_VIS: {  // CheckAndAddVisited (graph_utils.go:45-53), epoch-tagged slots
                const unsigned long long tag = ((unsigned long long)epoch << 32) | vk;
                const unsigned long long s0 = (unsigned long long)v0.x | ((unsigned long long)v0.y << 32);
                const unsigned long long s1 = (unsigned long long)v0.z | ((unsigned long long)v0.w << 32);
                const bool e0 = (uint32_t)(s0 >> 32) != epoch, e1 = (uint32_t)(s1 >> 32) != epoch;
                if (s0 == tag || (!e0 && s1 == tag)) {
                    st = S_CNEXT;  // already visited (engine.go:157-160)
                    break;
                }
                if (!e0 && !e1) {
                    aux = (aux + 1) & pmask;
                    la0 = reinterpret_cast<const uint4 *>(vis + 2 * aux);
                    ln = 1;
                    break;
                }
                if (2 * (vcount + 1) > P.vcap) {
                    fin = 2;
                    break;
                }
                vis[2 * aux + (e0 ? 0 : 1)] = tag;
                vcount++;
                st = S_CDISP;
                break;
            }
            case S_CDISP: {
                if (f_phase(w) == 4) {  // draining after a decisive child: mark, never run
                    if (cc == NONE32) st = S_RET;  // `res` still holds the decisive result
                    else st = S_CNEXT;
                    break;
                }
                const uint32_t c = top.z;
                top.z = cc;
                if (c == NONE32) {  // nothing was pending: the loop's first child, or none left
                    if (cc == NONE32) {
                        if (w & FL_OWNER) scope = false;
                        res = M_NOT;
                        st = S_RET;
                    } else {
                        st = S_CNEXT;  // find its successor before it runs
                    }
                    break;
                }
                // run the pending child checkIsAllowed(c, d, skipDirect=true) (engine.go:161)
                const NodeInfo ni = t_node_info(T, c);
                if (ri_status(ni.ri) == REL_ERROR) {  // engine.go:228-232: decisive
                    res = mk_err(KETO_QERR_NO_RELATION) | (t_relname(s, T, c, ni) << 16);
                    if (w & FL_OWNER) {
                        scope = false;
                        st = S_RET;
                    } else {
                        top.w = set_phase(w, 4);
                        st = cc == NONE32 ? S_RET : S_CNEXT;
                    }
                    break;
                }
                const bool rw = ri_rw(ni.ri);
                if (!rw && (!ri_ss(ni.ri) || d <= 1)) {  // empty group / Unknown -> not a member
                    if (cc == NONE32) {
                        if (w & FL_OWNER) scope = false;
                        res = M_NOT;
                        st = S_RET;
                    } else {
                        st = S_CNEXT;
                    }
                    break;
                }
                if (sp + 1 >= P.scap) {
                    fin = 2;
                    break;
                }
                stk[sp++] = top;
                // without a rewrite the child's group is just expandSubject(c, d-1)
                top = rw ? make_uint4(c, 0, 0, fw(F_IA, d, 0, FL_SKIP)) : make_uint4(c, 0, 0, fw(F_ES, d - 1));
                have_res = false;
                st = S_RUN;
                break;
            }
            case S_TNEXT: {  // TTU: next parent (rewrites.go:279-288)
                const uint32_t cur = top.y;
                if (cur >= top.z) {
                    res = M_NOT;
                    st = S_RET;
                    break;
                }
                if (cur < ew_lo || cur >= ew_hi) {
                    la0 = win(s.set_dst, cur);
                    ln = 1;
                    st = S_TEDGE;
                    break;
                }
                const uint32_t c = wword(ew, cur - ew_lo) & ~EDGE_ALIAS;
                top.y = cur + 1;
                if (COUNT) q_edges++;
                if (d <= 1) break;  // checkIsAllowed(..., <= 0) -> Unknown: next parent
                const NodeInfo ci = t_node_info(T, c);
                if (sp + 1 >= P.scap) {
                    fin = 2;
                    break;
                }
                stk[sp++] = top;
                top = make_uint4(t_sibling(T, c, ci, top.x), 0, 0, fw(F_IA, d - 1));
                have_res = false;
                st = S_RUN;
                break;
            }
            case S_TEDGE:
                ew = v0;
                ew_lo = top.y - (uint32_t)((reinterpret_cast<uintptr_t>(s.set_dst + top.y) >> 2) & 3);
                ew_hi = ew_lo + 4;
                st = S_TNEXT;
                break;
            case S_SPROBE: {  // OR shortcut `relation IN (...) LIMIT 1` (traverser.go:143-172)
                const uint32_t r0 = probe_check(v0, (((uint64_t)sidx << 32) | pc0) + 1);
                const uint32_t r1 = pn > 1 ? probe_check(v1, (((uint64_t)sidx << 32) | pc1) + 1) : 0;
                if (r0 == 2 || r1 == 2) {
                    if (r0 == 2) aux = (aux + 1) & s.probe_mask;
                    la0 = s.probe + aux;
                    ln = 1;
                    if (pn > 1) {
                        if (r1 == 2) aux2 = (aux2 + 1) & s.probe_mask;
                        la1 = s.probe + aux2;
                        ln = 2;
                    }
                    break;
                }
                if (COUNT) q_probes++;
                if (r0 == 1) {
                    res = M_IS;
                    st = S_RET;
                    break;
                }
                if (pn > 1) {
                    if (COUNT) q_probes++;
                    if (r1 == 1) {
                        res = M_IS;
                        st = S_RET;
                        break;
                    }
                }
                st = S_RUN;  // the RW frame continues from its cursor (phase 1)
                break;
            }
            // ---------------------------------------------------------------- frame execution
            case S_RUN: {
                uint32_t action = 0;  // 1 call `callee`, 2 return `res`
                uint4 callee = make_uint4(0, 0, 0, 0);
                switch (f_type(w)) {
                case F_IA: {  // checkIsAllowed (engine.go:214-249)
                    const uint32_t node = top.x;
                    uint32_t phase = f_phase(w);
                    if (phase == 0) {
                        if (d == 0) {  // :215-220
                            res = M_UNK;
                            action = 2;
                            break;
                        }
                        const NodeInfo ni = t_node_info(T, node);
                        top.y = ni.ri;
                        if (ri_status(ni.ri) == REL_ERROR) {  // :228-232
                            res = mk_err(KETO_QERR_NO_RELATION) | (t_relname(s, T, node, ni) << 16);
                            action = 2;
                            break;
                        }
                        if (ri_rw(ni.ri)) {  // :236-238
                            top.w = set_phase(w, 1);
                            callee = make_uint4(node, ri_op(ni.ri), 0, fw(F_RW, d));
                            action = 1;
                            break;
                        }
                        phase = 2;  // no rewrite: straight to the direct check
                    } else if (phase == 1) {  // the rewrite returned
                        have_res = false;
                        if (decisive(res)) {
                            action = 2;
                            break;
                        }
                        phase = 2;
                    }
                    const uint32_t ri = top.y;
                    if (phase == 2 && (!s.strict || !ri_rw(ri)) && !(w & FL_SKIP) && d > 1) {  // :239-243
                        if (COUNT) q_probes++;  // checkDirect(d-1) (:167-208)
                        if (!(node & VIRT_BIT)) {
                            if (!heavy) {
                                if (R0 == node || R1 == node || R2 == node || R3 == node) {
                                    res = M_IS;
                                    action = 2;
                                    break;
                                }
                            } else {
                                top.w = set_phase(w, 2);
                                aux = (uint32_t)mix64((((uint64_t)sidx << 32) | node) + 1) & s.probe_mask;
                                la0 = s.probe + aux;
                                ln = 1;
                                st = S_DPROBE;
                                break;
                            }
                        }
                    }
                    // expand-subject(d-1) as a tail call (:244-246); Unknown or no group -> NotMember
                    if (ri_ss(ri) && d > 1) {
                        top = make_uint4(node, 0, 0, fw(F_ES, d - 1));
                        break;
                    }
                    res = M_NOT;
                    action = 2;
                    break;
                }
                case F_ES:  // checkExpandSubject (engine.go:102-164)
                    if (f_phase(w) == 0) {
                        if (COUNT) q_rows++;
                        if (top.x & VIRT_BIT) {
                            res = M_NOT;
                            action = 2;
                            break;
                        }
                        la0 = s.set_row + top.x;
                        ln = 1;
                        top.w = set_phase(w, 1);
                        st = S_ROWOFF;
                        break;
                    }
                    have_res = false;  // phase 3: a child returned
                    ew_lo = 1;         // the edge window did not survive the child
                    ew_hi = 0;
                    if (decisive(res)) {
                        if (w & FL_OWNER) {  // the scope dies with this frame: no marks needed
                            scope = false;
                            action = 2;
                            break;
                        }
                        top.w = set_phase(w, 4);  // mark the remaining siblings, then return res
                        if (top.z == NONE32) {
                            action = 2;
                            break;
                        }
                        st = S_CNEXT;
                        break;
                    }
                    if (top.z == NONE32) {  // no sibling pending: the loop is done
                        if (w & FL_OWNER) scope = false;
                        res = M_NOT;
                        action = 2;
                        break;
                    }
                    st = S_CNEXT;  // find the pending sibling's successor, then run it
                    break;
                case F_RW: {  // checkSubjectSetRewrite (rewrites.go:33-134) + or/and (binop.go:18-73)
                    const uint32_t node = top.x;
                    const Op op = T.ops[top.y];
                    const uint32_t kind = (op.type_kind >> 8) & 0xFFu;
                    const bool is_or = kind == OPK_OR;
                    uint32_t phase = f_phase(w);
                    if (phase == 0) {
                        if (d == 0) {  // :39-42
                            res = M_UNK;
                            action = 2;
                            break;
                        }
                        if (kind == OPK_BAD) {  // :58-59
                            res = mk_err(KETO_QERR_NOT_IMPLEMENTED);
                            action = 2;
                            break;
                        }
                        phase = (is_or && ((op.type_kind >> 16) & 1u)) ? 1 : 3;
                        top.z = 0;
                    } else if (phase == 2) {  // shortcut candidates returned
                        have_res = false;
                        if (decisive(res)) {
                            action = 2;
                            break;
                        }
                        phase = 3;
                        top.z = 0;
                    } else if (phase == 4) {  // a child check returned
                        have_res = false;
                        if (is_or) {
                            if (decisive(res)) {  // binop.go:23-26
                                action = 2;
                                break;
                            }
                        } else if ((res >> 8) != 0 || (res & 3u) != M_IS) {  // binop.go:52-54
                            res = (res & ~3u) | M_NOT;
                            action = 2;
                            break;
                        }
                        phase = 3;
                    }
                    top.w = set_phase(w, phase);
                    const NodeInfo ni = t_node_info(T, node);
                    if (phase == 1) {  // shortcut IN probes in AST order (rewrites.go:62-92)
                        uint32_t k = top.z;
                        bool found = false;
                        pn = 0;
                        while (k < op.child_count && pn < 2 && !found) {
                            const Op ch = T.ops[T.op_children[op.child_begin + k]];
                            if ((ch.type_kind & 0xFFu) != OP_CSS) {
                                k++;
                                continue;
                            }
                            const uint32_t t = t_sibling(T, node, ni, ch.rel_computed & 0xFFFFu);
                            if (s.strict && !(t & VIRT_BIT)) {  // traverser.go:137-139
                                const NodeInfo ti = t_node_info(T, t);
                                if (ri_status(ti.ri) == REL_DECLARED && ri_rw(ti.ri)) {
                                    k++;
                                    continue;
                                }
                            }
                            if (heavy && !(t & VIRT_BIT)) {
                                if (pn == 0) pc0 = t;
                                else pc1 = t;
                                pn++;
                                k++;
                                continue;
                            }
                            if (pn) break;  // keep probe order: resolve the pending hash probes first
                            if (COUNT) q_probes++;
                            if (!(t & VIRT_BIT) && (R0 == t || R1 == t || R2 == t || R3 == t)) found = true;
                            k++;
                        }
                        top.z = k;
                        if (found) {
                            res = M_IS;
                            action = 2;
                            break;
                        }
                        if (pn) {
                            aux = (uint32_t)mix64((((uint64_t)sidx << 32) | pc0) + 1) & s.probe_mask;
                            la0 = s.probe + aux;
                            ln = 1;
                            if (pn > 1) {
                                aux2 = (uint32_t)mix64((((uint64_t)sidx << 32) | pc1) + 1) & s.probe_mask;
                                la1 = s.probe + aux2;
                                ln = 2;
                            }
                            st = S_SPROBE;
                            break;
                        }
                        if (k < op.child_count) break;  // more CSS children: next step
                        // no direct member: candidates checkIsAllowed(c, d-1, true) (rewrites.go:88-90)
                        top.w = set_phase(w, 2);
                        callee = make_uint4(node, top.y, 0, fw(F_SC, d));
                        action = 1;
                        break;
                    }
                    // phase 3: next non-CSS (OR) / any (AND) child
                    uint32_t k = top.z;
                    while (k < op.child_count) {
                        const uint32_t ci = T.op_children[op.child_begin + k];
                        k++;
                        const Op ch = T.ops[ci];
                        const uint32_t ct = ch.type_kind & 0xFFu;
                        if (is_or && ct == OP_CSS) continue;  // handled by the shortcut (:95-98)
                        top.z = k;
                        top.w = set_phase(w, 4);
                        if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
                        else if (ct == OP_CSS)
                            callee = make_uint4(t_sibling(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
                        else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d - 1));  // :118
                        else callee = make_uint4(node, ci, 0, fw(F_INV, d));
                        action = 1;
                        break;
                    }
                    if (action == 1) break;
                    res = (!is_or && op.child_count > 0) ? M_IS : M_NOT;  // binop.go:19-21,38,42-44,62-65
                    action = 2;
                    break;
                }
                case F_SC: {  // shortcut candidates (rewrites.go:88-90)
                    if (have_res) {
                        have_res = false;
                        if (decisive(res)) {
                            action = 2;
                            break;
                        }
                    }
                    const uint32_t node = top.x;
                    const Op op = T.ops[top.y];
                    const NodeInfo ni = t_node_info(T, node);
                    uint32_t k = top.z;
                    while (k < op.child_count) {
                        const Op ch = T.ops[T.op_children[op.child_begin + k]];
                        k++;
                        if ((ch.type_kind & 0xFFu) != OP_CSS || d <= 1) continue;  // d-1 <= 0 -> Unknown
                        top.z = k;
                        callee = make_uint4(t_sibling(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0,
                                            fw(F_IA, d - 1, 0, FL_SKIP));
                        action = 1;
                        break;
                    }
                    if (action == 1) break;
                    res = M_NOT;
                    action = 2;
                    break;
                }
                case F_TTU:  // checkTupleToSubjectSet (rewrites.go:242-293)
                    if (f_phase(w) == 0) {
                        const Op op = T.ops[top.y];
                        const NodeInfo ni = t_node_info(T, top.x);
                        const uint32_t ts = t_sibling(T, top.x, ni, op.rel_computed & 0xFFFFu);
                        if (COUNT) q_rows++;
                        if (ts & VIRT_BIT) {
                            res = M_NOT;
                            action = 2;
                            break;
                        }
                        top = make_uint4(op.rel_computed >> 16, ts, 0, set_phase(w, 1));
                        la0 = s.set_row + ts;
                        ln = 1;
                        st = S_ROWOFF;
                        break;
                    }
                    have_res = false;  // a parent's check returned
                    if (decisive(res)) {
                        action = 2;
                        break;
                    }
                    ew_lo = 1;  // window unknown after the child: reload
                    ew_hi = 0;
                    st = S_TNEXT;
                    break;
                case F_INV: {  // checkInverted (rewrites.go:136-200)
                    if (have_res) {
                        have_res = false;
                        const uint32_t m = res & 3u;
                        if (m == M_IS) res = (res & ~3u) | M_NOT;
                        else if (m == M_NOT) res = (res & ~3u) | M_IS;
                        action = 2;
                        break;
                    }
                    const Op op = T.ops[top.y];
                    if (op.child_count != 1) {
                        res = mk_err(KETO_QERR_NOT_IMPLEMENTED);
                        action = 2;
                        break;
                    }
                    const uint32_t ci = T.op_children[op.child_begin];
                    const Op ch = T.ops[ci];
                    const uint32_t ct = ch.type_kind & 0xFFu;
                    const uint32_t node = top.x;
                    top.w = set_phase(w, 1);
                    if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
                    else if (ct == OP_CSS) {
                        const NodeInfo ni = t_node_info(T, node);
                        callee = make_uint4(t_sibling(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
                    } else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d));  // keeps depth (:171)
                    else callee = make_uint4(node, ci, 0, fw(F_INV, d));
                    action = 1;
                    break;
                }
                default:
                    res = mk_err(KETO_QERR_INTERNAL);
                    action = 2;
                }
                if (action == 1) {  // call: push the caller, run the callee
                    if (sp + 1 >= P.scap) {
                        fin = 2;
                        break;
                    }
                    stk[sp++] = top;
                    top = callee;
                    have_res = false;
                } else if (action == 2) {
                    st = S_RET;
                }
                break;
            }
            default:
                fin = 2;
            }
        }
        if (fin) {
            if (fin == 2) {  // scratch outgrown: hand the query to the next tier
                if (P.last_tier) {
                    P.out_allowed[q] = 0;
                    P.out_err[q] = KETO_QERR_INTERNAL;
                } else {
                    P.ovf_list[atomicAdd(P.ovf_count, 1u)] = pos;
                }
            } else {
                const uint32_t err = res >> 8;  // code | relation name id << 8 (KETO_F_ERR_DETAIL)
                P.out_allowed[q] = (err == 0 && (res & 3u) == M_IS) ? 1 : 0;
                P.out_err[q] = (int32_t)(P.err_detail ? err : err & 0xFFu);
                if (COUNT) {
                    c_rows += q_rows;
                    c_edges += q_edges;
                    c_probes += q_probes;
                    c_q++;
                }
            }
            st = S_IDLE;
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

// --------------------------------------------------------------------------------------
// host launcher

void run_check(const Snapshot &s, Stream &st, const CheckLaunch &L) {
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    constexpr uint32_t BLOCK = 256;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    // Queries that outgrow a tier's scratch go to the next (lanes, visited slots per lane,
    // frames per lane); HBM is plentiful (288 GB): tier 0 holds ~500 visited nodes per lane,
    // tier 1 ~4k, tier 2 ~500k.
    // Tier 0 is sized to the persistent grid it can ever launch (KETO_T0_BLOCKS_PER_CU resident
    // blocks per CU): 1.3k lanes x 9 KiB per CU, ~3 GiB per stream on 256 CUs.
    const Tier t[3] = {Tier{cus * KETO_T0_BLOCKS_PER_CU * 256, 1024, 64},  // the common case
                       Tier{cus * 64, 1u << 13, 1024},                      // wide visited scopes
                       Tier{64, 1u << 20, 1u << 14}};   // huge scopes / deep recursion
    ensure_scratch(st.check_scratch, t);
    run_resolve(s, st, L.queries, L.n, L.max_depth);
    Scratch &sc = st.check_scratch;
    uint32_t *list[2] = {st.lists, st.lists + st.list_cap};
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = lds_tables ? s.dev.lds_bytes : 0;
    KETO_HIP(hipMemsetAsync(sc.ctrl, 0, 64, st.stream));
    for (int tier = 0; tier < 3; tier++) {
        CheckParams P{};
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
        P.scap = t[tier].scap;
        P.max_depth = L.max_depth;
        P.max_width = L.max_width;
        P.counters = st.counters + 8 * tier;
        P.last_tier = tier == 2;
        P.err_detail = L.err_detail;
        uint32_t lanes = t[tier].lanes;
        if (tier == 0) {  // persistent grid: the resident blocks (occupancy API), capped by the batch
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&check_kernel<false, true>),
                                                             BLOCK, lds) != hipSuccess || per_cu <= 0)
                per_cu = 4;
            per_cu = std::min(per_cu, KETO_T0_BLOCKS_PER_CU);
            lanes = std::min<uint32_t>(lanes, (uint32_t)per_cu * cus * BLOCK);
            // A batch smaller than the resident grid is spread over more waves with fewer live
            // lanes each: a wave-step then runs fewer distinct interpreter states, which is what
            // sets the step time (and so a small batch's latency).
            const uint64_t waves = lanes / 64;
            P.live_lanes = (uint32_t)std::min<uint64_t>(64, (L.n + waves - 1) / waves);
            const uint64_t need = (L.n + P.live_lanes - 1) / P.live_lanes * 64;
            lanes = (uint32_t)std::min<uint64_t>(lanes, (need + BLOCK - 1) / BLOCK * BLOCK);
        } else {
            P.live_lanes = 64;
        }
        const uint32_t bs = std::min<uint32_t>(BLOCK, lanes);  // every launched lane owns scratch
        dim3 grid(lanes / bs), block(bs);
        if (tier == 0) st.mark_begin();
        if (lds_tables) {
            if (L.count) hipLaunchKernelGGL((check_kernel<true, true>), grid, block, lds, st.stream, P);
            else hipLaunchKernelGGL((check_kernel<false, true>), grid, block, lds, st.stream, P);
        } else {
            if (L.count) hipLaunchKernelGGL((check_kernel<true, false>), grid, block, 0, st.stream, P);
            else hipLaunchKernelGGL((check_kernel<false, false>), grid, block, 0, st.stream, P);
        }
        KETO_HIP(hipGetLastError());
        if (tier == 0) st.mark_end();
    }
}

}  // namespace keto
