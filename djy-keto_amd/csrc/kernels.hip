// gfx950 kernels: batched Check (exact sequential semantics) and Expand.
//
// Execution model (MI355X-first): the reference evaluates one Check as a
// recursion of goroutines that issue one SQL statement per hop.  Here every
// lane of a persistent 64-wide wavefront owns one query and walks the same
// recursion as an explicit frame stack (one-worker sequential order,
// SURVEY.md section 8.0 H3), so thousands of independent pointer chases are in
// flight per CU.  Rows are read straight from the HBM-resident CSR, membership
// probes go to the subject's reverse row (kept in VGPRs when short), visited
// sets are per-lane open-addressing tables in scratch tagged by an epoch so a
// new scope never has to be cleared.  Lanes refill from a global work queue
// with one atomic per wavefront (ballot + mbcnt).  A query whose visited set or
// stack outgrows its tier is handed to the next tier (bigger scratch, fewer
// lanes) by an on-device list, so the whole batch is three back-to-back
// launches with no host round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "engine.hpp"

namespace keto {

namespace {

// result word: bits 0-1 membership (0 unknown, 1 is, 2 not), bits 8-15 error
constexpr uint32_t M_UNK = 0, M_IS = 1, M_NOT = 2;
__device__ __forceinline__ uint32_t mk_err(uint32_t e) { return e << 8; }
__device__ __forceinline__ bool decisive(uint32_t r) { return (r >> 8) != 0 || (r & 3u) == M_IS; }

// frame word w: bits 0-15 depth, 16-19 type, 20-23 phase, 24 skip_direct, 25 scope owner,
//               26 shortcut done
enum FrameType : uint32_t { F_IA = 0, F_ES = 1, F_RW = 2, F_SC = 3, F_TTU = 4, F_INV = 5 };
__device__ __forceinline__ uint32_t fw(uint32_t type, uint32_t d, uint32_t phase = 0, uint32_t flags = 0) {
    return (d & 0xFFFFu) | (type << 16) | (phase << 20) | flags;
}
constexpr uint32_t FL_SKIP = 1u << 24, FL_OWNER = 1u << 25, FL_SCDONE = 1u << 26;
__device__ __forceinline__ uint32_t f_d(uint32_t w) { return w & 0xFFFFu; }
__device__ __forceinline__ uint32_t f_type(uint32_t w) { return (w >> 16) & 0xFu; }
__device__ __forceinline__ uint32_t f_phase(uint32_t w) { return (w >> 20) & 0xFu; }

struct CheckParams {
    DevSnapshot s;
    const keto_query *queries;
    const uint32_t *qlist;      // tier >= 2: indices of queries to (re)run
    const uint32_t *qlist_count;
    uint32_t n;                 // tier 1: number of queries
    uint8_t *out_allowed;
    int32_t *out_err;
    uint32_t *next;             // work-queue head
    uint32_t *ovf_list;         // overflow hand-off to the next tier
    uint32_t *ovf_count;
    unsigned long long *vis;    // [lanes * vcap]
    uint4 *stack;               // [lanes * scap]
    uint32_t *epochs;           // [lanes]
    uint32_t vcap, scap;
    int32_t max_depth, max_width;
    unsigned long long *counters;
    uint32_t last_tier;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

__device__ __forceinline__ uint32_t ns_of(const DevSnapshot &s, uint32_t node) {
    // last namespace whose node_base <= node
    uint32_t lo = 0, hi = s.n_ns;  // answer in [lo, hi)
    while (hi - lo > 1) {
        uint32_t m = (lo + hi) >> 1;
        if (s.ns[m].node_base <= node) lo = m;
        else hi = m;
    }
    return lo;
}

struct NodeInfo {
    uint32_t ns, slot, ri;  // ri: relinfo (virtual nodes: synthesized)
};

__device__ __forceinline__ NodeInfo node_info(const DevSnapshot &s, uint32_t node) {
    NodeInfo r;
    if (node & VIRT_BIT) {
        r.ns = (node >> 16) & 0x7FFFu;
        r.slot = NO_SLOT;
        uint32_t st = r.ns < s.n_ns ? nr_status(s.nsrel[(size_t)r.ns * s.n_rel + (node & 0xFFFFu)]) : REL_NIL;
        r.ri = make_ri(NO_OP, false, true, st, false);  // no rewrite: direct + expand of an empty row
        return r;
    }
    r.ns = ns_of(s, node);
    const NsDev nd = s.ns[r.ns];
    r.slot = (node - nd.node_base) % nd.n_slots;
    r.ri = s.relinfo[nd.slot_base + r.slot];
    return r;
}

// node for (same entity as `node`, relation `rel`) -- computed usersets / tuple-to-userset
__device__ __forceinline__ uint32_t sibling(const DevSnapshot &s, uint32_t node, const NodeInfo &ni, uint32_t rel) {
    uint32_t w = rel < s.n_rel ? s.nsrel[(size_t)ni.ns * s.n_rel + rel] : (REL_NIL << 16) | NO_SLOT;
    uint32_t slot = nr_slot(w);
    if (slot == NO_SLOT || (node & VIRT_BIT)) return VIRT_BIT | (ni.ns << 16) | (rel & 0xFFFFu);
    return node - ni.slot + slot;
}

__device__ __forceinline__ void row_of(const uint32_t *off, uint32_t node, uint32_t &b, uint32_t &e) {
    if (node & VIRT_BIT) {
        b = e = 0;
        return;
    }
    b = off[node];
    e = off[node + 1];
}

template <int K>
struct Subject {
    uint32_t rb, re;
    uint32_t R[K];
    bool in_regs;

    __device__ __forceinline__ void load(const DevSnapshot &s, uint32_t idx) {
        if (idx == NONE32) {
            rb = re = 0;
        } else {
            rb = s.rev_off[idx];
            re = s.rev_off[idx + 1];
        }
        in_regs = (re - rb) <= (uint32_t)K;
#pragma unroll
        for (int k = 0; k < K; k++) R[k] = (in_regs && rb + k < re) ? s.rev_nodes[rb + k] : NONE32;
    }
    // (node, subject) is a tuple?  == ExistsRelationTuples (relationtuples.go:249-261)
    __device__ __forceinline__ bool member(const DevSnapshot &s, uint32_t node) const {
        if (node & VIRT_BIT) return false;
        if (in_regs) {
            bool hit = false;
#pragma unroll
            for (int k = 0; k < K; k++) hit |= (R[k] == node);
            return hit;
        }
        uint32_t lo = rb, hi = re;
        while (lo < hi) {
            uint32_t m = (lo + hi) >> 1;
            uint32_t v = s.rev_nodes[m];
            if (v < node) lo = m + 1;
            else hi = m;
        }
        return lo < re && s.rev_nodes[lo] == node;
    }
};

__device__ __forceinline__ uint32_t entity_lookup(const DevSnapshot &s, uint32_t ns, uint32_t obj) {
    unsigned long long key = ((unsigned long long)ns << 32 | obj) + 1ull;
    uint32_t h = (uint32_t)mix64(key) & s.ent_mask;
    for (uint32_t probe = 0; probe <= s.ent_mask; probe++) {
        unsigned long long k = s.ent_keys[h];
        if (k == key) return s.ent_vals[h];
        if (k == 0) break;
        h = (h + 1) & s.ent_mask;
    }
    return NONE32;
}

// resolve (ns, obj, rel) to a node id (phantom entity for unknown objects)
__device__ __forceinline__ uint32_t resolve_node(const DevSnapshot &s, uint32_t ns, uint32_t obj, uint32_t rel,
                                                 bool phantom_ok) {
    if (ns >= s.n_ns) return phantom_ok ? (VIRT_BIT | (0x7FFFu << 16) | 0xFFFFu) : NONE32;
    uint32_t w = rel < s.n_rel ? s.nsrel[(size_t)ns * s.n_rel + rel] : (REL_NIL << 16) | NO_SLOT;
    uint32_t e = entity_lookup(s, ns, obj);
    if (e == NONE32) {
        if (!phantom_ok) return NONE32;
        e = s.ns[ns + 1].ent_base - 1;  // phantom entity of ns
    }
    if (nr_slot(w) == NO_SLOT) return phantom_ok ? (VIRT_BIT | (ns << 16) | (rel & 0xFFFFu)) : NONE32;
    const NsDev nd = s.ns[ns];
    return nd.node_base + (e - nd.ent_base) * nd.n_slots + nr_slot(w);
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

template <int K, bool COUNT, int TIER>
__global__ __launch_bounds__(256) void check_kernel(CheckParams P) {
    const DevSnapshot &s = P.s;
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t vmask = P.vcap - 1;
    const uint32_t W = (uint32_t)P.max_width;

    int32_t q = -1;
    bool exhausted = false;
    // per-query state
    Subject<K> subj;
    uint4 top = make_uint4(0, 0, 0, 0);
    uint32_t sp = 0, res = 0, vcount = 0;
    bool have_res = false, scope = false;
    uint64_t c_rows = 0, c_edges = 0, c_probes = 0, c_q = 0;
    uint32_t q_rows = 0, q_edges = 0, q_probes = 0;

    while (true) {
        // ---- refill idle lanes: one atomic per wavefront ----------------------------------
        bool need = (q < 0) && !exhausted;
        unsigned long long mask = __ballot(need);
        if (mask) {
            uint32_t base = 0;
            if (lane_id() == (uint32_t)__ffsll((long long)mask) - 1) base = atomicAdd(P.next, (uint32_t)__popcll(mask));
            base = __shfl(base, __ffsll((long long)mask) - 1);
            if (need) {
                uint32_t my = base + (uint32_t)__popcll(mask & ((1ull << lane_id()) - 1ull));
                if (my >= nq) {
                    exhausted = true;
                } else {
                    q = (int32_t)(P.qlist ? P.qlist[my] : my);
                    const keto_query Q = P.queries[q];
                    uint32_t root = resolve_node(s, Q.ns, Q.obj, Q.rel, true);
                    uint32_t sidx = NONE32;
                    if (Q.subj_kind == 0) {
                        if (Q.s_obj < s.n_uuids) sidx = Q.s_obj;
                    } else {
                        uint32_t sn = resolve_node(s, Q.s_ns, Q.s_obj, Q.s_rel, false);
                        if (sn != NONE32) sidx = s.n_uuids + sn;
                    }
                    subj.load(s, sidx);
                    int32_t d = Q.max_depth;
                    if (d <= 0 || P.max_depth < d) d = P.max_depth;  // engine.go:82-84
                    top = make_uint4(root, 0, 0, fw(F_IA, (uint32_t)d));
                    sp = 0;
                    have_res = false;
                    scope = false;
                    q_rows = q_edges = q_probes = 0;
                }
            }
        }
        if (__ballot(q >= 0) == 0) break;
        if (q < 0) continue;

        // ---- one interpreter step --------------------------------------------------------
        // action: 0 = continue with top, 1 = call (push top, top = callee), 2 = return res
        int action = 0;
        uint4 callee = make_uint4(0, 0, 0, 0);
        bool ovf = false;
        const uint32_t w = top.w;
        const uint32_t d = f_d(w);
        switch (f_type(w)) {
        case F_IA: {  // checkIsAllowed (engine.go:214-249)
            const uint32_t node = top.x;
            uint32_t phase = f_phase(w);
            if (phase == 0) {
                if (d == 0) {  // :215-220 (depth is stored clamped at >= 0)
                    res = M_UNK;
                    action = 2;
                    break;
                }
                NodeInfo ni = node_info(s, node);
                top.y = ni.ri;
                if (ri_status(ni.ri) == REL_ERROR) {  // :228-232
                    res = mk_err(KETO_QERR_NO_RELATION);
                    action = 2;
                    break;
                }
                if (ri_rw(ni.ri)) {  // :236-238
                    top.w = (w & ~(0xFu << 20)) | (1u << 20);
                    callee = make_uint4(node, ri_op(ni.ri), 0, fw(F_RW, d));
                    action = 1;
                    break;
                }
                phase = 1;
            } else if (phase == 1 && have_res) {  // rewrite returned
                have_res = false;
                if (decisive(res)) {
                    action = 2;
                    break;
                }
            }
            // phase 1: direct, then expand-subject (tail call)
            const uint32_t ri = top.y;
            if ((!s.strict || !ri_rw(ri)) && !(w & FL_SKIP)) {  // :239-243
                if (d > 1) {                                     // checkDirect guard (:168-173)
                    if (COUNT) q_probes++;
                    if (subj.member(s, node)) {
                        res = M_IS;
                        action = 2;
                        break;
                    }
                }
            }
            if (ri_ss(ri) && d > 1) {  // :244-246 -> checkExpandSubject(d-1); tail call
                top = make_uint4(node, 0, 0, fw(F_ES, d - 1));
                action = 0;
                break;
            }
            res = M_NOT;
            action = 2;
            break;
        }
        case F_ES: {  // checkExpandSubject (engine.go:102-164)
            uint32_t cur, end;
            if (f_phase(w) == 0) {
                uint32_t b, e;
                row_of(s.set_off, top.x, b, e);
                if (COUNT) q_rows++;
                bool found = false;
                for (uint32_t i = b; i < e; i++) {  // EXISTS lookahead (traverser.go:73-80, 109-111)
                    if (COUNT) {
                        q_edges++;
                        q_probes++;
                    }
                    if (subj.member(s, s.set_dst[i] & ~EDGE_ALIAS)) {
                        found = true;
                        break;
                    }
                }
                if (found) {
                    res = M_IS;
                    action = 2;
                    break;
                }
                uint32_t cnt = e - b;
                if (cnt > W) e = b + (W > 0 ? W - 1 : 0);  // results[:maxWidth-1] (engine.go:141-150)
                uint32_t flags = 0;
                if (!scope) {  // graph.InitVisited (graph_utils.go:38-43)
                    scope = true;
                    epoch++;
                    vcount = 0;
                    flags = FL_OWNER;
                }
                cur = b;
                end = e;
                top.w = fw(F_ES, d, 1, (w & FL_OWNER) | flags);
            } else {
                cur = top.y;
                end = top.z;
                if (have_res) {
                    have_res = false;
                    if (decisive(res)) {
                        if (top.w & FL_OWNER) scope = false;
                        action = 2;
                        break;
                    }
                }
            }
            // next child with visited check (engine.go:151-162)
            bool called = false;
            while (cur < end) {
                uint32_t c = s.set_dst[cur++];
                uint32_t key = (c & EDGE_ALIAS) ? s.vkey[c & ~EDGE_ALIAS] : c;
                c &= ~EDGE_ALIAS;
                // CheckAndAddVisited: per-lane open addressing, epoch-tagged
                uint32_t h = (uint32_t)mix64(key) & vmask;
                bool seen = false;
                unsigned long long tag = ((unsigned long long)epoch << 32) | key;
                while (true) {
                    unsigned long long v = vis[h];
                    if ((uint32_t)(v >> 32) != epoch) break;
                    if (v == tag) {
                        seen = true;
                        break;
                    }
                    h = (h + 1) & vmask;
                }
                if (seen) continue;
                if (2 * (vcount + 1) > P.vcap) {
                    ovf = true;
                    break;
                }
                vis[h] = tag;
                vcount++;
                // child checkIsAllowed(c, d, skipDirect=true); inline the common no-rewrite case
                NodeInfo ni = node_info(s, c);
                if (ri_status(ni.ri) == REL_ERROR) {
                    res = mk_err(KETO_QERR_NO_RELATION);
                    called = true;  // decisive: return it
                    break;
                }
                if (!ri_rw(ni.ri)) {
                    if (!ri_ss(ni.ri) || d <= 1) continue;  // empty group / UNK -> not a member
                    callee = make_uint4(c, 0, 0, fw(F_ES, d - 1));
                } else {
                    callee = make_uint4(c, 0, 0, fw(F_IA, d, 0, FL_SKIP));
                }
                top.y = cur;
                top.z = end;
                action = 1;
                called = true;
                break;
            }
            if (ovf || action == 1) break;
            if (called) {  // relation error from an inlined child
                if (top.w & FL_OWNER) scope = false;
                action = 2;
                break;
            }
            if (top.w & FL_OWNER) scope = false;
            res = M_NOT;
            action = 2;
            break;
        }
        case F_RW: {  // checkSubjectSetRewrite (rewrites.go:33-134) + or/and (binop.go:18-73)
            const uint32_t node = top.x;
            const Op op = s.ops[top.y];
            const uint32_t kind = (op.type_kind >> 8) & 0xFFu;
            const bool is_or = kind == OPK_OR;
            uint32_t k = top.z;
            uint32_t flags = w & FL_SCDONE;
            if (f_phase(w) == 0) {
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
            } else if (have_res) {
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
            }
            NodeInfo ni = node_info(s, node);
            if (is_or && (op.type_kind >> 16 & 1u) && !flags) {
                // OR computed-userset shortcut (rewrites.go:62-92 + traverser.go:123-191)
                flags = FL_SCDONE;
                bool found = false;
                for (uint32_t j = 0; j < op.child_count && !found; j++) {
                    const Op ch = s.ops[s.op_children[op.child_begin + j]];
                    if ((ch.type_kind & 0xFFu) != OP_CSS) continue;
                    uint32_t rel = ch.rel_computed & 0xFFFFu;
                    uint32_t t = sibling(s, node, ni, rel);
                    if (s.strict && !(t & VIRT_BIT)) {  // traverser.go:137-139
                        NodeInfo ti = node_info(s, t);
                        if (ri_status(ti.ri) == REL_DECLARED && ri_rw(ti.ri)) continue;
                    }
                    if (COUNT) q_probes++;
                    if (subj.member(s, t)) found = true;
                }
                if (found) {
                    res = M_IS;
                    action = 2;
                    break;
                }
                top.w = fw(F_RW, d, 1, flags);
                callee = make_uint4(node, top.y, 0, fw(F_SC, d));
                action = 1;
                break;
            }
            // next non-CSS (OR) / any (AND) child
            while (k < op.child_count) {
                const uint32_t ci = s.op_children[op.child_begin + k++];
                const Op ch = s.ops[ci];
                const uint32_t ct = ch.type_kind & 0xFFu;
                if (is_or && ct == OP_CSS) continue;  // handled by the shortcut (:95-98)
                top.z = k;
                top.w = fw(F_RW, d, 1, flags);
                if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
                else if (ct == OP_CSS) callee = make_uint4(sibling(s, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
                else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d - 1));  // restDepth-1 (:118)
                else callee = make_uint4(node, ci, 0, fw(F_INV, d));
                action = 1;
                break;
            }
            if (action == 1) break;
            res = (!is_or && op.child_count > 0) ? M_IS : M_NOT;  // binop.go:19-21,38,42-44,62-65
            action = 2;
            break;
        }
        case F_SC: {  // shortcut candidates: checkIsAllowed(c, d-1, skipDirect=true) (rewrites.go:88-90)
            const uint32_t node = top.x;
            if (have_res) {
                have_res = false;
                if (decisive(res)) {
                    action = 2;
                    break;
                }
            }
            const Op op = s.ops[top.y];
            uint32_t k = top.z;
            NodeInfo ni = node_info(s, node);
            while (k < op.child_count) {
                const Op ch = s.ops[s.op_children[op.child_begin + k++]];
                if ((ch.type_kind & 0xFFu) != OP_CSS) continue;
                if (d <= 1) continue;  // checkIsAllowed guard -> Unknown -> not a member
                top.z = k;
                callee = make_uint4(sibling(s, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d - 1, 0, FL_SKIP));
                action = 1;
                break;
            }
            if (action == 1) break;
            res = M_NOT;
            action = 2;
            break;
        }
        case F_TTU: {  // checkTupleToSubjectSet (rewrites.go:242-293)
            uint32_t cur, end, computed;
            if (f_phase(w) == 0) {
                const Op op = s.ops[top.y];
                NodeInfo ni = node_info(s, top.x);
                uint32_t ts = sibling(s, top.x, ni, op.rel_computed & 0xFFFFu);
                uint32_t b, e;
                row_of(s.set_off, ts, b, e);
                if (COUNT) q_rows++;
                cur = b;
                end = e;
                computed = op.rel_computed >> 16;
            } else {
                cur = top.y;
                end = top.z;
                computed = top.x;
                if (have_res) {
                    have_res = false;
                    if (decisive(res)) {
                        action = 2;
                        break;
                    }
                }
            }
            if (cur < end) {
                uint32_t c = s.set_dst[cur++] & ~EDGE_ALIAS;
                if (COUNT) q_edges++;
                top = make_uint4(computed, cur, end, fw(F_TTU, d, 1));
                if (d <= 1) {  // checkIsAllowed(…, <=0) -> Unknown: next parent
                    action = 0;
                    break;
                }
                NodeInfo ci = node_info(s, c);
                callee = make_uint4(sibling(s, c, ci, computed), 0, 0, fw(F_IA, d - 1));
                action = 1;
                break;
            }
            res = M_NOT;
            action = 2;
            break;
        }
        case F_INV: {  // checkInverted (rewrites.go:136-200)
            if (have_res) {
                have_res = false;
                uint32_t m = res & 3u;
                if (m == M_IS) res = (res & ~3u) | M_NOT;
                else if (m == M_NOT) res = (res & ~3u) | M_IS;
                action = 2;
                break;
            }
            const Op op = s.ops[top.y];
            if (op.child_count != 1) {
                res = mk_err(KETO_QERR_NOT_IMPLEMENTED);
                action = 2;
                break;
            }
            const uint32_t ci = s.op_children[op.child_begin];
            const Op ch = s.ops[ci];
            const uint32_t ct = ch.type_kind & 0xFFu;
            const uint32_t node = top.x;
            top.w = fw(F_INV, d, 1);
            if (ct == OP_TTU) callee = make_uint4(node, ci, 0, fw(F_TTU, d));
            else if (ct == OP_CSS) {
                NodeInfo ni = node_info(s, node);
                callee = make_uint4(sibling(s, node, ni, ch.rel_computed & 0xFFFFu), 0, 0, fw(F_IA, d));
            } else if (ct == OP_REWRITE) callee = make_uint4(node, ci, 0, fw(F_RW, d));  // keeps restDepth (:171)
            else callee = make_uint4(node, ci, 0, fw(F_INV, d));
            action = 1;
            break;
        }
        default:
            res = mk_err(KETO_QERR_INTERNAL);
            action = 2;
        }

        if (action == 1) {
            if (sp + 1 >= P.scap) ovf = true;
            else {
                stk[sp++] = top;
                top = callee;
                have_res = false;
            }
        }
        if (ovf) {
            if (P.last_tier) {
                P.out_allowed[q] = 0;
                P.out_err[q] = KETO_QERR_INTERNAL;
            } else {
                uint32_t slot = atomicAdd(P.ovf_count, 1u);
                P.ovf_list[slot] = (uint32_t)q;
            }
            q = -1;
            continue;
        }
        if (action == 2) {
            if (sp == 0) {  // CheckIsMember (engine.go:65-71)
                uint32_t err = res >> 8;
                P.out_allowed[q] = (err == 0 && (res & 3u) == M_IS) ? 1 : 0;
                P.out_err[q] = (int32_t)err;
                if (COUNT) {
                    c_rows += q_rows;
                    c_edges += q_edges;
                    c_probes += q_probes;
                    c_q++;
                }
                q = -1;
            } else {
                top = stk[--sp];
                have_res = true;
            }
        }
    }
    P.epochs[gl] = epoch;
    if (COUNT) {
        // wave reduction, one atomic per wave per counter
        for (int off = 32; off > 0; off >>= 1) {
            c_rows += __shfl_down(c_rows, off);
            c_edges += __shfl_down(c_edges, off);
            c_probes += __shfl_down(c_probes, off);
            c_q += __shfl_down(c_q, off);
        }
        if (lane_id() == 0) {
            atomicAdd(&P.counters[0], (unsigned long long)c_rows);
            atomicAdd(&P.counters[1], (unsigned long long)c_edges);
            atomicAdd(&P.counters[2], (unsigned long long)c_probes);
            atomicAdd(&P.counters[4], (unsigned long long)c_q);
        }
    }
}

// ------------------------------------------------------------------------------------
// Expand (expand/engine.go:54-124): one lane per root, explicit DFS stack, two passes
// (count, then emit into exclusive-scan offsets).

struct ExpandParams {
    DevSnapshot s;
    const keto_subject_set *roots;
    const uint32_t *qlist;
    const uint32_t *qlist_count;
    uint32_t n;
    int32_t max_depth;
    unsigned long long *sizes;
    const unsigned long long *offsets;
    uint32_t *out;
    int32_t *err;
    uint32_t *next;
    uint32_t *ovf_list, *ovf_count;
    unsigned long long *vis;
    uint4 *stack;
    uint32_t *epochs;
    uint32_t vcap, scap, emit, last_tier;
    unsigned long long *counters;
};

__device__ __forceinline__ bool vis_insert(unsigned long long *vis, uint32_t vmask, uint32_t epoch, uint32_t key,
                                           uint32_t &vcount, uint32_t vcap, bool &ovf) {
    uint32_t h = (uint32_t)mix64(key) & vmask;
    unsigned long long tag = ((unsigned long long)epoch << 32) | key;
    while (true) {
        unsigned long long v = vis[h];
        if ((uint32_t)(v >> 32) != epoch) break;
        if (v == tag) return true;
        h = (h + 1) & vmask;
    }
    if (2 * (vcount + 1) > vcap) {
        ovf = true;
        return false;
    }
    vis[h] = tag;
    vcount++;
    return false;
}

__global__ __launch_bounds__(256) void expand_kernel(ExpandParams P) {
    const DevSnapshot &s = P.s;
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t vmask = P.vcap - 1;
    unsigned long long c_rows = 0, c_edges = 0, c_out = 0;
    while (true) {
        uint32_t my = atomicAdd(P.next, 1u);
        if (my >= nq) break;
        const uint32_t q = P.qlist ? P.qlist[my] : my;
        if (P.emit && P.err[q] != 0) continue;  // count pass gave up on this root
        const keto_subject_set R = P.roots[q];
        int32_t d = R.max_depth;
        if (d <= 0 || P.max_depth < d) d = P.max_depth;  // :56-58
        uint32_t root = resolve_node(s, R.ns, R.obj, R.rel, true);
        epoch++;
        uint32_t vcount = 0;
        bool ovf = false;
        uint64_t cnt = 0;
        uint32_t *out = P.emit ? P.out + 3ull * P.offsets[q] : nullptr;
        auto emit = [&](uint32_t type, uint32_t skey, uint32_t nch) {
            if (out) {
                out[3 * cnt + 0] = type;
                out[3 * cnt + 1] = skey;
                out[3 * cnt + 2] = nch;
            }
            cnt++;
        };
        uint64_t rows = 0, edges = 0;
        if (!(root & VIRT_BIT)) {
            uint32_t key = root;
            if (s.vkey && ri_shared(node_info(s, root).ri)) key = s.vkey[root];
            vis_insert(vis, vmask, epoch, key, vcount, P.vcap, ovf);  // visited includes the root (:69-72)
            uint32_t b = s.all_off[root], e = s.all_off[root + 1];
            rows++;
            if (b != e) {  // no tuples on the first page -> nil (:97-99)
                if (d <= 1) emit(4, SKEY_SET | root, 0);  // :101-104
                else {
                    emit(1, SKEY_SET | root, e - b);
                    uint32_t sp = 0;
                    uint4 top = make_uint4(b, e, (uint32_t)d, 0);
                    while (true) {
                        if (top.x == top.y) {
                            if (sp == 0) break;
                            top = stk[--sp];
                            continue;
                        }
                        uint32_t sk = s.all_subj[top.x++];
                        edges++;
                        if (!(sk & SKEY_SET)) {  // subject id -> leaf (:60-67)
                            emit(4, sk, 0);
                            continue;
                        }
                        uint32_t c = sk & ~SKEY_SET;
                        uint32_t cd = top.z - 1;
                        uint32_t ck = c;
                        if (s.vkey && ri_shared(node_info(s, c).ri)) ck = s.vkey[c];
                        if (vis_insert(vis, vmask, epoch, ck, vcount, P.vcap, ovf)) {
                            emit(4, sk, 0);  // revisit -> nil -> leaf (:112-117)
                            continue;
                        }
                        if (ovf) break;
                        uint32_t cb = s.all_off[c], ce = s.all_off[c + 1];
                        rows++;
                        if (cb == ce || cd <= 1) {
                            emit(4, sk, 0);
                            continue;
                        }
                        emit(1, sk, ce - cb);
                        if (sp + 1 >= P.scap) {
                            ovf = true;
                            break;
                        }
                        stk[sp++] = top;
                        top = make_uint4(cb, ce, cd, 0);
                    }
                }
            }
        }
        if (ovf) {
            if (P.last_tier) {
                P.err[q] = KETO_QERR_INTERNAL;
                if (!P.emit) P.sizes[q] = 0;
            } else {
                uint32_t slot = atomicAdd(P.ovf_count, 1u);
                P.ovf_list[slot] = q;
            }
            continue;
        }
        if (!P.emit) {
            P.sizes[q] = cnt;
            P.err[q] = 0;
            c_rows += rows;
            c_edges += edges;
            c_out += cnt;
        }
    }
    P.epochs[gl] = epoch;
    if (P.counters && !P.emit) {
        atomicAdd(&P.counters[0], c_rows);
        atomicAdd(&P.counters[1], c_edges);
        atomicAdd(&P.counters[3], c_out);
    }
}

// ------------------------------------------------------------------------------------
// host side: tiers and workspace

constexpr int BLOCK = 256;

int num_cus(int device) {
    static int cached[64] = {0};
    if (device >= 0 && device < 64 && cached[device]) return cached[device];
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    if (device >= 0 && device < 64) cached[device] = cus;
    return cus;
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Allocate (once) disjoint per-tier regions: [ctrl][epochs t0..t2][vis t0][stack t0]...
// Zero-filled at allocation: every epoch starts at 0, so every visited tag is stale.
void ensure_scratch(Scratch &sc, const Tier t[3]) {
    if (sc.mem) return;
    size_t bytes = 256;
    for (int i = 0; i < 3; i++) bytes += align256((size_t)t[i].lanes * 4);
    for (int i = 0; i < 3; i++) bytes += align256((size_t)t[i].lanes * t[i].vcap * 8ull) + align256((size_t)t[i].lanes * t[i].scap * 16ull);
    KETO_HIP(hipMalloc(&sc.mem, bytes));
    KETO_HIP(hipMemset(sc.mem, 0, bytes));
    sc.bytes = bytes;
    char *p = static_cast<char *>(sc.mem);
    sc.ctrl = reinterpret_cast<uint32_t *>(p);
    p += 256;
    for (int i = 0; i < 3; i++) {
        sc.t[i] = t[i];
        sc.epochs[i] = reinterpret_cast<uint32_t *>(p);
        p += align256((size_t)t[i].lanes * 4);
    }
    for (int i = 0; i < 3; i++) {
        sc.vis[i] = reinterpret_cast<unsigned long long *>(p);
        p += align256((size_t)t[i].lanes * t[i].vcap * 8ull);
        sc.stack[i] = reinterpret_cast<uint4 *>(p);
        p += align256((size_t)t[i].lanes * t[i].scap * 16ull);
    }
}

void ensure_lists(Stream &st, uint64_t n) {
    if (st.list_cap >= n) return;
    if (st.lists) KETO_HIP(hipFree(st.lists));
    st.lists = nullptr;
    st.list_cap = 0;
    KETO_HIP(hipMalloc(&st.lists, 2 * n * sizeof(uint32_t)));
    st.list_cap = n;
}

}  // namespace

void run_check(const Snapshot &s, Stream &st, const CheckLaunch &L) {
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    const uint32_t cus = (uint32_t)num_cus(s.device);
    // (lanes, visited slots per lane, frames per lane)
    const Tier t[3] = {Tier{cus * 16 * 64, 128, 48},      // 16 waves / CU, the common case
                       Tier{cus * 64, 1u << 12, 512},     // wide visited scopes
                       Tier{64, 1u << 20, 1u << 14}};     // huge scopes / deep recursion
    ensure_scratch(st.check_scratch, t);
    ensure_lists(st, L.n);
    Scratch &sc = st.check_scratch;
    uint32_t *list[2] = {st.lists, st.lists + st.list_cap};
    // ctrl: [0..2] work-queue heads per tier, [3..4] overflow counts
    KETO_HIP(hipMemsetAsync(sc.ctrl, 0, 64, st.stream));
    for (int tier = 0; tier < 3; tier++) {
        CheckParams P{};
        P.s = s.dev;
        P.queries = L.queries;
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
        uint32_t lanes = t[tier].lanes;
        if (tier == 0) lanes = (uint32_t)std::min<uint64_t>(lanes, ((L.n + BLOCK - 1) / BLOCK) * BLOCK);
        // every launched lane owns scratch: lanes is a multiple of the block size
        const uint32_t bs = std::min<uint32_t>(BLOCK, lanes);
        dim3 grid(lanes / bs), block(bs);
        if (tier == 0) KETO_HIP(hipEventRecord(st.ev0, st.stream));
        // one instantiation per tier so profiles attribute time per tier
#define KETO_LAUNCH_CHECK(T)                                                                              \
    do {                                                                                                 \
        if (L.count) hipLaunchKernelGGL((check_kernel<8, true, T>), grid, block, 0, st.stream, P);       \
        else hipLaunchKernelGGL((check_kernel<8, false, T>), grid, block, 0, st.stream, P);              \
    } while (0)
        if (tier == 0) KETO_LAUNCH_CHECK(0);
        else if (tier == 1) KETO_LAUNCH_CHECK(1);
        else KETO_LAUNCH_CHECK(2);
#undef KETO_LAUNCH_CHECK
        KETO_HIP(hipGetLastError());
        if (tier == 0) KETO_HIP(hipEventRecord(st.ev1, st.stream));
    }
}

void run_expand(const Snapshot &s, Stream &st, const ExpandLaunch &L) {
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    const uint32_t cus = (uint32_t)num_cus(s.device);
    const Tier t[3] = {Tier{cus * 64, 1u << 12, 256}, Tier{256, 1u << 18, 1u << 13}, Tier{8, 1u << 24, 1u << 18}};
    ensure_scratch(st.expand_scratch, t);
    ensure_lists(st, L.n);
    Scratch &sc = st.expand_scratch;
    uint32_t *list[2] = {st.lists, st.lists + st.list_cap};
    KETO_HIP(hipMemsetAsync(sc.ctrl, 0, 64, st.stream));
    for (int tier = 0; tier < 3; tier++) {
        ExpandParams P{};
        P.s = s.dev;
        P.roots = L.roots;
        P.qlist = tier == 0 ? nullptr : list[tier - 1];
        P.qlist_count = tier == 0 ? nullptr : &sc.ctrl[3 + tier - 1];
        P.n = (uint32_t)L.n;
        P.max_depth = L.max_depth;
        P.sizes = reinterpret_cast<unsigned long long *>(L.sizes);
        P.offsets = reinterpret_cast<const unsigned long long *>(L.offsets);
        P.out = L.out;
        P.err = L.err;
        P.next = &sc.ctrl[tier];
        P.ovf_list = tier < 2 ? list[tier] : nullptr;
        P.ovf_count = tier < 2 ? &sc.ctrl[3 + tier] : nullptr;
        P.vis = sc.vis[tier];
        P.stack = sc.stack[tier];
        P.epochs = sc.epochs[tier];
        P.vcap = t[tier].vcap;
        P.scap = t[tier].scap;
        P.emit = L.emit;
        P.last_tier = tier == 2;
        P.counters = L.emit ? nullptr : st.counters + 8 * tier;
        uint32_t lanes = t[tier].lanes;
        if (tier == 0) lanes = (uint32_t)std::min<uint64_t>(lanes, ((L.n + BLOCK - 1) / BLOCK) * BLOCK);
        const uint32_t bs = std::min<uint32_t>(BLOCK, lanes);  // every launched lane owns scratch
        hipLaunchKernelGGL(expand_kernel, dim3(lanes / bs), dim3(bs), 0, st.stream, P);
        KETO_HIP(hipGetLastError());
    }
}

}  // namespace keto
