// EXPERIMENT -- not built, not part of the product (kept for the record; see DESIGN.md
// "Wave-per-query interpreter: tried, not adopted").  Measured on MI355X as the heavy-prefix
// tier in front of the lane kernel: C2 batch 10.0 ms vs 7.8 ms lane-only, C3 unchanged
// (21.25 ms); as the sole tier C3 46.7 ms.  Needs the asm("" ::: "memory") barriers at the
// top of both loops -- without them the gfx950 build hangs/faults while the CPU emulation
// passes.  Declaration it needs in engine.hpp:
//   void run_check_wave(const Snapshot &, Stream &, const CheckLaunch &, const uint32_t *n_dev,
//                       uint32_t *next, uint32_t *ovf_list, uint32_t *ovf_count,
//                       unsigned long long *counters);
// gfx950 batched Check with OPL userset rewrites: one 64-wide wavefront per query.
//
// Same exact one-worker sequential semantics as the lane-per-query interpreter (check.hip,
// which stays as the deep-scratch overflow tier), but the control flow is WAVE-UNIFORM: the
// frame machine of internal/check/{engine,rewrites,binop}.go runs once per wavefront, in
// scalar registers, so there is no divergence tax (a lane-per-query wave executes the union
// of all its lanes' interpreter states every step; measured: ~2400 VALU + 2400 SALU per load
// step, the C3 kernel issue-bound).  The 64 lanes work on the data-parallel parts:
//   * the EXISTS found-lookahead of a subject-set row (traverser.go:73-80, 109-111): one lane
//     per edge, 64 membership tests per round trip, the first hit found with a ballot;
//   * the query subject's reverse row (<= 64 nodes) hashed into LDS at query start, so every
//     checkDirect / lookahead / OR-shortcut membership is an LDS probe, not an HBM round trip;
//   * clearing the visited scope.
// Per-wave LDS holds the frame stack, the visited set (graph_utils.go:38-53), the reverse-row
// hash and an edge stack (each expanding row's children, kept for the child loop so the
// children cost no reload after each recursive call).  A query that outgrows any of them is
// handed to the lane-per-query interpreter's big-scratch tiers through the overflow list.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace {

constexpr uint32_t M_UNK = 0, M_IS = 1, M_NOT = 2;
__device__ __forceinline__ uint32_t mk_err(uint32_t e) { return e << 8; }
__device__ __forceinline__ bool decisive(uint32_t r) { return (r >> 8) != 0 || (r & 3u) == M_IS; }

// frame word w: bits 0-15 depth, 16-19 type, 20-23 phase, 24 skip_direct, 25 visited-scope
// owner, 26 ES children on the LDS edge stack
enum FrameType : uint32_t { F_IA = 0, F_ES = 1, F_RW = 2, F_SC = 3, F_TTU = 4, F_INV = 5 };
constexpr uint32_t FL_SKIP = 1u << 24, FL_OWNER = 1u << 25, FL_ESTK = 1u << 26;
__device__ __forceinline__ uint32_t fw(uint32_t type, uint32_t d, uint32_t phase = 0, uint32_t flags = 0) {
    return (d & 0xFFFFu) | (type << 16) | (phase << 20) | flags;
}
__device__ __forceinline__ uint32_t f_d(uint32_t w) { return w & 0xFFFFu; }
__device__ __forceinline__ uint32_t f_type(uint32_t w) { return (w >> 16) & 0xFu; }
__device__ __forceinline__ uint32_t f_phase(uint32_t w) { return (w >> 20) & 0xFu; }
__device__ __forceinline__ uint32_t set_phase(uint32_t w, uint32_t p) { return (w & ~(0xFu << 20)) | (p << 20); }

// per-wave LDS
constexpr uint32_t WF_CAP = 64;   // frames
constexpr uint32_t WV_CAP = 2048;  // visited slots (keys node+1); at most WV_CAP/2 entries
constexpr uint32_t WR_CAP = 128;  // reverse-row hash slots: subjects with <= LIGHT_MAX entries
constexpr uint32_t LIGHT_MAX = 64;
constexpr uint32_t WE_CAP = 256;  // edge stack entries
constexpr uint32_t WAVE_LDS = WF_CAP * 16 + (WV_CAP + WR_CAP + WE_CAP) * 4;
constexpr uint32_t WAVES_PER_BLOCK = 4;

struct WaveParams {
    DevSnapshot s;
    const uint4 *start;  // resolve pre-pass records, in work order
    uint32_t n;
    const uint32_t *n_dev;  // if set: the query count, read on the device (the heavy prefix of the work order)
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *next;
    uint32_t *ovf_list, *ovf_count;
    int32_t max_width;
    unsigned long long *counters;
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }



// Table reads whose values steer the interpreter, made provably wave-uniform (scalar
// registers, scalar branches: no exec-mask bookkeeping around the frame machine)
__device__ __forceinline__ NodeInfo node_info_u(const Tables &T, uint32_t node) {
    const NodeInfo r = t_node_info(T, node);
    return NodeInfo{uni(r.ns), uni(r.slot), uni(r.ri)};
}
__device__ __forceinline__ Op op_u(const Tables &T, uint32_t i) {
    const Op o = T.ops[i];
    return Op{uni(o.type_kind), uni(o.child_begin), uni(o.child_count), uni(o.rel_computed)};
}
__device__ __forceinline__ uint32_t child_u(const Tables &T, uint32_t i) { return uni(T.op_children[i]); }
__device__ __forceinline__ uint32_t sibling_u(const Tables &T, uint32_t node, const NodeInfo &ni, uint32_t rel) {
    return uni(t_sibling(T, node, ni, rel));
}

// wave-level ordering of this wave's LDS accesses across lanes
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) { return (uint32_t)mix64(x); }

// membership of (subject, node) in the heavy-subject probe hash (16-byte buckets of two keys)
__device__ __forceinline__ bool probe_member(const DevSnapshot &s, uint32_t sidx, uint32_t node) {
    const uint64_t key = (((uint64_t)sidx << 32) | node) + 1;
    uint32_t b = (uint32_t)mix64(key) & s.probe_mask;
    bool r = false;
    for (uint32_t i = 0; i <= s.probe_mask; i++) {  // load <= 1/2: an empty slot ends the probe
        const uint4 v = s.probe[b];
        const uint64_t k0 = (uint64_t)v.x | ((uint64_t)v.y << 32), k1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
        if (k0 == key || k1 == key) {
            r = true;
            break;
        }
        if (k0 == 0 || k1 == 0) break;
        b = (b + 1) & s.probe_mask;
    }
    return r;
}
// ExistsRelationTuples(node, subject): the LDS hash of a short reverse row, else the probe hash
__device__ __forceinline__ bool member_of(bool light, const uint32_t *rtab, const DevSnapshot &s, uint32_t sidx,
                                          uint32_t node);
__device__ __forceinline__ bool rtab_member(const uint32_t *rtab, uint32_t node) {
    uint32_t h = hash32(node) & (WR_CAP - 1);
    bool r = false;
    for (uint32_t i = 0; i < WR_CAP; i++) {  // <= 64 keys in 128 slots: an empty slot always ends the probe
        const uint32_t v = rtab[h];
#ifdef KETO_WAVE_DEBUG
        {
            const unsigned long long bh = __ballot(v == node + 1), bz = __ballot(v == 0), ba = __ballot(1);
            if (__lane_id() == 0 && i < 4) printf("  rtab_member node %u h %u v %u hit %llx zero %llx active %llx\n", node, h, v, bh, bz, ba);
        }
#endif
        if (v == node + 1) {
            r = true;
            break;
        }
        if (v == 0) break;
        h = (h + 1) & (WR_CAP - 1);
    }
    return r;
}

__device__ __forceinline__ bool member_of(bool light, const uint32_t *rtab, const DevSnapshot &s, uint32_t sidx,
                                          uint32_t node) {
    if (light) return rtab_member(rtab, node);
    return probe_member(s, sidx, node);
}

template <bool COUNT, bool LDS_TABLES>
__global__ __launch_bounds__(256) void check_wave_kernel(WaveParams P) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const DevSnapshot &s = P.s;
    const Tables T = LDS_TABLES ? stage_tables(s, lds) : global_tables(s);
    const uint32_t lane = __lane_id();
    const uint32_t WS = warpSize;
    const uint32_t wid = threadIdx.x / WS;
    char *wb = lds + (LDS_TABLES ? (s.lds_bytes + 15) / 16 * 16 : 0) + (size_t)wid * WAVE_LDS;
    uint4 *fstk = reinterpret_cast<uint4 *>(wb);
    uint32_t *vtab = reinterpret_cast<uint32_t *>(wb + WF_CAP * 16);
    uint32_t *rtab = vtab + WV_CAP;
    uint32_t *estk = rtab + WR_CAP;
    const uint32_t W = (uint32_t)P.max_width;
    unsigned long long c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0;
    const uint32_t nq = P.n_dev ? uni(*P.n_dev) : P.n;

    while (true) {
        asm volatile("" ::: "memory");
        uint32_t my = 0;
        if (lane == 0) my = atomicAdd(P.next, 1u);
        my = uni(__shfl(my, 0));
#ifdef KETO_WAVE_DEBUG
        if (lane == 0) printf("wave %u got %u of %u\n", wid, my, P.n);
#endif
        if (my >= nq) break;
        const uint4 r0 = P.start[2 * (size_t)my];
        const uint32_t root = uni(r0.x), sidx = uni(r0.y), q = uni(r0.w);
        const uint32_t d0 = uni(r0.z) & 0xFFFFu;
        // the subject's reverse row (relationtuples.go:249-261 read side): hashed into LDS when
        // short, else membership goes to the global probe hash
        uint32_t rb = 0, rlen = 0;
        if (sidx != NONE32) {
            rb = uni(s.rev_off[sidx]);
            rlen = uni(s.rev_off[sidx + 1]) - rb;
        }
        const bool light = rlen <= LIGHT_MAX;
        if (light) {
            for (uint32_t k = lane; k < WR_CAP; k += WS) rtab[k] = 0;
            wave_sync();
            for (uint32_t k = lane; k < rlen; k += WS) {
                const uint32_t node = s.rev_nodes[rb + k];
                uint32_t h = hash32(node) & (WR_CAP - 1);
                while (true) {
                    const uint32_t old = atomicCAS(&rtab[h], 0u, node + 1);
                    if (old == 0 || old == node + 1) break;
                    h = (h + 1) & (WR_CAP - 1);
                }
            }
            wave_sync();
        }
#ifdef KETO_WAVE_DEBUG
        if (lane == 0) printf("q%u root %u sidx %u d %u rb %u rlen %u light %d rtab %p wb %p lds %p WS %u\n", q, root, sidx, d0, rb, rlen,
                              (int)light, (void *)rtab, (void *)wb, (void *)lds, WS);
#endif
#define member(node) member_of(light, rtab, s, sidx, (node))                        // per lane
#define member_uni(node) (uni(member_of(light, rtab, s, sidx, (node)) ? 1u : 0u) != 0)  // wave-uniform node

#ifdef KETO_WAVE_MINIMAL
        const bool mm = member_uni(root);
        uint32_t res = mm ? M_IS : M_NOT, sp = 0;
        bool ovf = false;
        uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
#else
        uint4 top = make_uint4(root, 0, 0, fw(F_IA, d0));  // checkIsAllowed(root, d, false)
        uint32_t sp = 0, res = 0, etop = 0, vcount = 0;
        bool have_res = false, scope = false, ovf = false;
        uint32_t q_rows = 0, q_edges = 0, q_probes = 0;
        // every loop turn runs the top frame; `act` 1 = call `callee`, 2 = return `res`, 0 = top replaced
        uint32_t turns = 0;
        bool running = true;
        while (running) {
            // Optimization barrier: without a side effect in this loop the compiler's transforms
            // of the wave-uniform loop (forward-progress assumptions around the convergent
            // readfirstlane/ballot operations) produced a kernel that never left it on gfx950.
            asm volatile("" ::: "memory");
            uint32_t act = 0;
            uint4 callee = make_uint4(0, 0, 0, 0);
            const uint32_t w = top.w;
            const uint32_t d = f_d(w);
#ifdef KETO_WAVE_DEBUG
            if (lane == 0 && turns < 64)
                printf("q%u turn %u sp %u frame %u/%u d %u x %u y %u z %u res %x\n", q, turns, sp, f_type(w), f_phase(w), d,
                       top.x, top.y, top.z, res);
#endif
            if (++turns > (1u << 26)) ovf = true;  // every wave reaches an exit: a runaway walk is handed over
            switch (ovf ? 15u : f_type(w)) {
            case F_IA: {  // checkIsAllowed (engine.go:214-249)
                const uint32_t node = top.x;
                uint32_t phase = f_phase(w);
                if (phase == 0) {
                    if (d == 0) {  // :215-220
                        res = M_UNK;
                        act = 2;
                        break;
                    }
                    const NodeInfo ni = node_info_u(T, node);
                    top.y = ni.ri;
                    if (ri_status(ni.ri) == REL_ERROR) {  // :228-232
                        res = mk_err(KETO_QERR_NO_RELATION);
                        act = 2;
                        break;
                    }
                    if (ri_rw(ni.ri)) {  // :236-238
                        top.w = set_phase(w, 1);
                        callee = make_uint4(node, ri_op(ni.ri), 0, fw(F_RW, d));
                        act = 1;
                        break;
                    }
                } else {  // the rewrite returned
                    have_res = false;
                    if (decisive(res)) {
                        act = 2;
                        break;
                    }
                }
                const uint32_t ri = top.y;
                if ((!s.strict || !ri_rw(ri)) && !(w & FL_SKIP) && d > 1) {  // :239-243
                    if (COUNT) q_probes++;  // checkDirect(d-1) (:167-208)
                    const bool mem = !(node & VIRT_BIT) && member_uni(node);
#ifdef KETO_WAVE_DEBUG
                    {
                        const unsigned long long bm = __ballot(mem), ba = __ballot(1), bn = __ballot(node == 6);
                        if (lane == 0) printf("  IA direct %u -> %d ballot mem %llx active %llx node6 %llx\n", node, (int)mem, bm, ba, bn);
                    }
#endif
                    if (mem) {
                        res = M_IS;
                        act = 2;
                        break;
                    }
                }
                if (ri_ss(ri) && d > 1) {  // expand-subject(d-1) as a tail call (:244-246)
                    top = make_uint4(node, 0, 0, fw(F_ES, d - 1));
                    break;
                }
                res = M_NOT;  // Unknown or no group -> not a member
                act = 2;
                break;
            }
            case F_ES: {  // checkExpandSubject (engine.go:102-164) + TraverseSubjectSetExpansion
                // phase 3 frame: x = cursor - begin, y = end - begin, z = edge-stack offset
                // (FL_ESTK) or row begin in set_dst
                if (f_phase(w) == 0) {
                    if (COUNT) q_rows++;
                    const uint32_t node = top.x;
                    if (node & VIRT_BIT) {
                        res = M_NOT;
                        act = 2;
                        break;
                    }
                    const uint4 rd = s.set_row[node];
                    const uint32_t b = uni(rd.x), e0 = uni(rd.y);
                    if (b == e0) {
                        res = M_NOT;
                        act = 2;
                        break;
                    }
                    const uint32_t ez = uni(rd.z), ew = uni(rd.w);
                    // the row's edges go on the LDS edge stack when they fit (kept for the child loop)
                    const bool stack_edges = etop + (e0 - b) <= WE_CAP;
                    // found-lookahead: one lane per edge, in shard order; the first hit ends the row
                    bool found = false;
                    for (uint32_t c0 = b; c0 < e0; c0 += WS) {
                        const uint32_t i = c0 + lane;
                        uint32_t raw = NONE32;
                        if (i < e0) raw = i == b ? ez : (i == b + 1 ? ew : s.set_dst[i]);
                        if (stack_edges && i < e0) estk[etop + (i - b)] = raw;
                        const bool hit = i < e0 && member(raw & ~EDGE_ALIAS);
                        const unsigned long long m = __ballot(hit);
                        const uint32_t span = std::min<uint32_t>(WS, e0 - c0);
                        if (m) {
                            if (COUNT) {
                                const uint32_t k = (uint32_t)__ffsll((long long)m);
                                q_edges += k;
                                q_probes += k;
                            }
                            found = true;
                            break;
                        }
                        if (COUNT) {
                            q_edges += span;
                            q_probes += span;
                        }
                    }
                    if (found) {
                        res = M_IS;
                        act = 2;
                        break;
                    }
                    wave_sync();
                    uint32_t e = e0;
                    if (e - b > W) e = b + (W > 0 ? W - 1 : 0);  // results[:maxWidth-1] (engine.go:141-150)
                    uint32_t flags = 0;
                    if (!scope) {  // graph.InitVisited (graph_utils.go:38-43): a fresh scope
                        scope = true;
                        vcount = 0;
                        for (uint32_t k = lane; k < WV_CAP; k += WS) vtab[k] = 0;
                        wave_sync();
                        flags = FL_OWNER;
                    }
                    if (stack_edges) {
                        top = make_uint4(0, e - b, etop, fw(F_ES, d, 3, flags | FL_ESTK));
                        etop += e0 - b;
                    } else {
                        top = make_uint4(0, e - b, b, fw(F_ES, d, 3, flags));
                    }
                } else {  // a child returned
                    have_res = false;
                    if (decisive(res)) {
                        if (w & FL_OWNER) scope = false;
                        if (w & FL_ESTK) etop = top.z;
                        act = 2;
                        break;
                    }
                }
                // child loop (engine.go:151-162)
                const uint32_t fwd = top.w;
                while (top.x < top.y) {
                    const uint32_t raw = (fwd & FL_ESTK) ? uni(estk[top.z + top.x]) : uni(s.set_dst[top.z + top.x]);
                    top.x++;
                    const uint32_t cc = raw & ~EDGE_ALIAS;
                    const uint32_t vk = (raw & EDGE_ALIAS) ? uni(s.vkey[cc]) : cc;
                    // CheckAndAddVisited (graph_utils.go:45-53)
                    uint32_t h = hash32(vk) & (WV_CAP - 1);
                    bool seen = false;
                    while (true) {
                        const uint32_t v = uni(vtab[h]);
                        if (v == vk + 1) {
                            seen = true;
                            break;
                        }
                        if (v == 0) break;
                        h = (h + 1) & (WV_CAP - 1);
                    }
                    if (seen) continue;
                    if (2 * (vcount + 1) > WV_CAP) {
                        ovf = true;
                        break;
                    }
                    if (lane == 0) vtab[h] = vk + 1;
                    wave_sync();
                    vcount++;
                    // child checkIsAllowed(c, d, skipDirect=true) (engine.go:161)
                    const NodeInfo ni = node_info_u(T, cc);
                    if (ri_status(ni.ri) == REL_ERROR) {  // engine.go:228-232
                        res = mk_err(KETO_QERR_NO_RELATION);
                        act = 3;
                        break;
                    }
                    const bool rw = ri_rw(ni.ri);
                    if (!rw && (!ri_ss(ni.ri) || d <= 1)) continue;  // empty group / Unknown -> not a member
                    // without a rewrite the child's group is just expandSubject(c, d-1)
                    callee = rw ? make_uint4(cc, 0, 0, fw(F_IA, d, 0, FL_SKIP)) : make_uint4(cc, 0, 0, fw(F_ES, d - 1));
                    act = 1;
                    break;
                }
                if (ovf || act == 1) break;
                if (act == 0) res = M_NOT;  // children exhausted
                if (fwd & FL_OWNER) scope = false;
                if (fwd & FL_ESTK) etop = top.z;
                act = 2;
                break;
            }
            case F_RW: {  // checkSubjectSetRewrite (rewrites.go:33-134) + or/and (binop.go:18-73)
                const uint32_t node = top.x;
                const Op op = op_u(T, top.y);
                const uint32_t kind = (op.type_kind >> 8) & 0xFFu;
                const bool is_or = kind == OPK_OR;
                uint32_t phase = f_phase(w);
                if (phase == 0) {
                    if (d == 0) {  // :39-42
                        res = M_UNK;
                        act = 2;
                        break;
                    }
                    if (kind == OPK_BAD) {  // :58-59
                        res = mk_err(KETO_QERR_NOT_IMPLEMENTED);
                        act = 2;
                        break;
                    }
                    phase = (is_or && ((op.type_kind >> 16) & 1u)) ? 1 : 3;
                    top.z = 0;
                } else if (phase == 2) {  // shortcut candidates returned
                    have_res = false;
                    if (decisive(res)) {
                        act = 2;
                        break;
                    }
                    phase = 3;
                    top.z = 0;
                } else if (phase == 4) {  // a child check returned
                    have_res = false;
                    if (is_or) {
                        if (decisive(res)) {  // binop.go:23-26
                            act = 2;
                            break;
                        }
                    } else if ((res >> 8) != 0 || (res & 3u) != M_IS) {  // binop.go:52-54
                        res = (res & ~3u) | M_NOT;
                        act = 2;
                        break;
                    }
                    phase = 3;
                }
                top.w = set_phase(w, phase);
                const NodeInfo ni = node_info_u(T, node);
                if (phase == 1) {  // shortcut `relation IN (...)` probes in AST order (rewrites.go:62-92, traverser.go:123-191)
                    bool found = false;
                    for (uint32_t k = 0; k < op.child_count && !found; k++) {
                        const Op ch = op_u(T, child_u(T, op.child_begin + k));
                        if ((ch.type_kind & 0xFFu) != OP_CSS) continue;
                        const uint32_t t = sibling_u(T, node, ni, ch.rel_computed & 0xFFFFu);
                        if (s.strict && !(t & VIRT_BIT)) {  // traverser.go:137-139
                            const NodeInfo ti = node_info_u(T, t);
                            if (ri_status(ti.ri) == REL_DECLARED && ri_rw(ti.ri)) continue;
                        }
                        if (COUNT) q_probes++;
                        if (!(t & VIRT_BIT) && member_uni(t)) found = true;
                    }
                    if (found) {
                        res = M_IS;
                        act = 2;
                        break;
                    }
                    // no direct member: candidates checkIsAllowed(c, d-1, true) (rewrites.go:88-90)
                    top.w = set_phase(w, 2);
                    callee = make_uint4(node, top.y, 0, fw(F_SC, d));
                    act = 1;
                    break;
                }
                // phase 3: next non-CSS (OR) / any (AND) child
                uint32_t k = top.z;
                while (k < op.child_count) {
                    const uint32_t ci = child_u(T, op.child_begin + k);
                    k++;
                    const Op ch = op_u(T, ci);
                    const uint32_t ct = ch.type_kind & 0xFFu;
                    if (is_or && ct == OP_CSS) continue;  // handled by the shortcut (:95-98)
                    top.z = k;
                    top.w = set_phase(w, 4);
                    if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
                    else if (ct == OP_CSS)
                        callee = make_uint4(sibling_u(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
                    else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d - 1));  // :118
                    else callee = make_uint4(node, ci, 0, fw(F_INV, d));
                    act = 1;
                    break;
                }
                if (act == 1) break;
                res = (!is_or && op.child_count > 0) ? M_IS : M_NOT;  // binop.go:19-21,38,42-44,62-65
                act = 2;
                break;
            }
            case F_SC: {  // shortcut candidates (rewrites.go:88-90)
                if (have_res) {
                    have_res = false;
                    if (decisive(res)) {
                        act = 2;
                        break;
                    }
                }
                const uint32_t node = top.x;
                const Op op = op_u(T, top.y);
                const NodeInfo ni = node_info_u(T, node);
                uint32_t k = top.z;
                while (k < op.child_count) {
                    const Op ch = op_u(T, child_u(T, op.child_begin + k));
                    k++;
                    if ((ch.type_kind & 0xFFu) != OP_CSS || d <= 1) continue;  // d-1 <= 0 -> Unknown
                    top.z = k;
                    callee = make_uint4(sibling_u(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d - 1, 0, FL_SKIP));
                    act = 1;
                    break;
                }
                if (act == 1) break;
                res = M_NOT;
                act = 2;
                break;
            }
            case F_TTU: {  // checkTupleToSubjectSet (rewrites.go:242-293)
                // phase 1 frame: x = computed relation, y = cursor, z = end
                uint32_t first = NONE32;  // the row's first edge, inline in its descriptor
                if (f_phase(w) == 0) {
                    const Op op = op_u(T, top.y);
                    const NodeInfo ni = node_info_u(T, top.x);
                    const uint32_t ts = sibling_u(T, top.x, ni, op.rel_computed & 0xFFFFu);
                    if (COUNT) q_rows++;
                    if (ts & VIRT_BIT) {
                        res = M_NOT;
                        act = 2;
                        break;
                    }
                    const uint4 rd = s.set_row[ts];
                    top = make_uint4(op.rel_computed >> 16, uni(rd.x), uni(rd.y), set_phase(w, 1));
                    first = uni(rd.z);
                } else {  // a parent's check returned
                    have_res = false;
                    if (decisive(res)) {
                        act = 2;
                        break;
                    }
                }
                if (top.y < top.z) {  // next parent (rewrites.go:279-288)
                    const uint32_t raw = first != NONE32 ? first : uni(s.set_dst[top.y]);
                    const uint32_t c = raw & ~EDGE_ALIAS;
                    top.y++;
                    if (COUNT) q_edges++;
                    if (d > 1) {
                        const NodeInfo ci = node_info_u(T, c);
                        callee = make_uint4(sibling_u(T, c, ci, top.x), 0, 0, fw(F_IA, d - 1));
                        act = 1;
                        break;
                    }
                    // checkIsAllowed(..., <= 0) -> Unknown: the remaining parents alike
                    if (COUNT) q_edges += top.z - top.y;
                    top.y = top.z;
                }
                res = M_NOT;
                act = 2;
                break;
            }
            case F_INV: {  // checkInverted (rewrites.go:136-200)
                if (have_res) {
                    have_res = false;
                    const uint32_t m = res & 3u;
                    if (m == M_IS) res = (res & ~3u) | M_NOT;
                    else if (m == M_NOT) res = (res & ~3u) | M_IS;
                    act = 2;
                    break;
                }
                const Op op = op_u(T, top.y);
                if (op.child_count != 1) {
                    res = mk_err(KETO_QERR_NOT_IMPLEMENTED);
                    act = 2;
                    break;
                }
                const uint32_t ci = child_u(T, op.child_begin);
                const Op ch = op_u(T, ci);
                const uint32_t ct = ch.type_kind & 0xFFu;
                const uint32_t node = top.x;
                top.w = set_phase(w, 1);
                if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
                else if (ct == OP_CSS) {
                    const NodeInfo ni = node_info_u(T, node);
                    callee = make_uint4(sibling_u(T, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
                } else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d));  // keeps depth (:171)
                else callee = make_uint4(node, ci, 0, fw(F_INV, d));
                act = 1;
                break;
            }
            case 15:  // runaway: nothing to run
                break;
            default:
                res = mk_err(KETO_QERR_INTERNAL);
                act = 2;
            }
#ifdef KETO_WAVE_DEBUG
            if (lane == 0 && turns < 64) printf("  act %u ovf %d sp %u\n", act, (int)ovf, sp);
#endif
            act = uni(act);  // every decision above is wave-uniform: let the compiler see it
            if (act == 1 && sp >= WF_CAP) ovf = true;
            if (ovf) {
                running = false;
            } else if (act == 1) {  // call: push the caller, run the callee
                fstk[sp] = top;  // every lane stores the same frame
                sp++;
                top = callee;
                have_res = false;
            } else if (act >= 2) {  // return `res`
                if (sp == 0) {
                    running = false;  // CheckIsMember (engine.go:65-71)
                } else {
                    wave_sync();
                    sp--;
                    const uint4 f = fstk[sp];
                    top = make_uint4(uni(f.x), uni(f.y), uni(f.z), uni(f.w));
                    have_res = true;
                }
            }
        }
#endif  // KETO_WAVE_MINIMAL
#ifdef KETO_WAVE_DEBUG
        if (lane == 0) printf("q%u done res %x ovf %d sp %u\n", q, res, (int)ovf, sp);
#endif
        if (lane == 0) {
            if (ovf) {
                P.ovf_list[atomicAdd(P.ovf_count, 1u)] = my;
            } else {
                const uint32_t err = res >> 8;
                P.out_allowed[q] = (err == 0 && (res & 3u) == M_IS) ? 1 : 0;
                P.out_err[q] = (int32_t)err;
            }
        }
        if (COUNT && !ovf) {
            c_rows += q_rows;
            c_edges += q_edges;
            c_probes += q_probes;
            c_q++;
        }
    }
    if (COUNT && lane == 0) {
        atomicAdd(&P.counters[0], c_rows);
        atomicAdd(&P.counters[1], c_edges);
        atomicAdd(&P.counters[2], c_probes);
        atomicAdd(&P.counters[4], c_q);
    }
}

#undef member
#undef member_uni

}  // namespace

size_t wave_lds_bytes(const Snapshot &s) {
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    return (lds_tables ? (s.dev.lds_bytes + 15) / 16 * 16 : 0) + WAVES_PER_BLOCK * WAVE_LDS;
}

// the heavy queries of a batch (the longest-first prefix of the resolve pre-pass, count on the
// device), one wavefront each; overflow -> `ovf_list`
void run_check_wave(const Snapshot &s, Stream &st, const CheckLaunch &L, const uint32_t *n_dev, uint32_t *next,
                    uint32_t *ovf_list, uint32_t *ovf_count, unsigned long long *counters) {
    constexpr uint32_t BLOCK = 64 * WAVES_PER_BLOCK;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    const bool lds_tables = s.dev.lds_bytes <= LDS_TABLE_LIMIT;
    const size_t lds = wave_lds_bytes(s);
    WaveParams P{};
    P.s = s.dev;
    P.start = st.resolved;
    P.n = (uint32_t)L.n;
    P.n_dev = n_dev;
    P.out_allowed = L.out_allowed;
    P.out_err = L.out_err;
    P.next = next;
    P.ovf_list = ovf_list;
    P.ovf_count = ovf_count;
    P.max_width = L.max_width;
    P.counters = counters;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(&check_wave_kernel<false, true>),
                                                     BLOCK, lds) != hipSuccess || per_cu <= 0)
        per_cu = 4;
    // persistent grid: the resident blocks, capped by the batch (one wave per query in flight)
    const uint64_t want = (L.n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)per_cu * cus, want));
    if (lds_tables) {
        if (L.count) hipLaunchKernelGGL((check_wave_kernel<true, true>), dim3(blocks), dim3(BLOCK), lds, st.stream, P);
        else hipLaunchKernelGGL((check_wave_kernel<false, true>), dim3(blocks), dim3(BLOCK), lds, st.stream, P);
    } else {
        if (L.count) hipLaunchKernelGGL((check_wave_kernel<true, false>), dim3(blocks), dim3(BLOCK), lds, st.stream, P);
        else hipLaunchKernelGGL((check_wave_kernel<false, false>), dim3(blocks), dim3(BLOCK), lds, st.stream, P);
    }
    KETO_HIP(hipGetLastError());
}

}  // namespace keto
