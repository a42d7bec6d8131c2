// gfx950 batched Expand (expand/engine.go:54-124): one lane per root, explicit DFS stack,
// global per-call visited set (root included), two passes -- count, then emit into the
// exclusive-scan offsets -- so the pre-order output needs no device-side allocation.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace {

__device__ __forceinline__ uint32_t node_ri(const DevSnapshot &s, uint32_t node) {
    return t_node_info(global_tables(s), node).ri;
}

__device__ __forceinline__ uint32_t resolve_node(const DevSnapshot &s, uint32_t ns, uint32_t obj, uint32_t rel) {
    if (ns >= s.n_ns) return VIRT_BIT | (0x7FFFu << 16) | 0xFFFFu;
    uint32_t e = ent_lookup(s, ns, obj);
    if (e == NONE32) e = s.ns[ns + 1].ent_base - 1;  // phantom entity: no tuples
    return t_node(global_tables(s), ns, e, rel);
}

// one output node in API form (Mapper.ToTree, uuid_mapping.go:356-385): a subject id, or a
// subject set mapped back to (namespace, object uuid id, relation name id)
__device__ __forceinline__ keto_tree_node api_node(const DevSnapshot &s, uint32_t type, uint32_t skey, uint32_t nch) {
    keto_tree_node o;
    o.type = type;
    o.n_children = nch;
    if (skey & SKEY_SET) {
        const uint32_t node = skey & ~SKEY_SET;
        const NodeInfo ni = t_node_info(global_tables(s), node);
        const NsDev nd = s.ns[ni.ns];
        o.subj_kind = 1;
        o.s_obj = s.ent_obj[nd.ent_base + (node - nd.node_base) / nd.n_slots];
        o.s_ns = ni.ns;
        o.s_rel = s.slot_rel[nd.slot_base + ni.slot];
    } else {
        o.subj_kind = 0;
        o.s_obj = skey;
        o.s_ns = 0;
        o.s_rel = 0;
    }
    return o;
}

struct ExpandParams {
    DevSnapshot s;
    const keto_subject_set *roots;
    const uint32_t *qlist;
    const uint32_t *qlist_count;
    uint32_t n;
    int32_t max_depth;
    unsigned long long *sizes;
    const unsigned long long *offsets;
    keto_tree_node *out;  // emit pass: API records (keto_mi355x.h), pre-order per root
    int32_t *err;
    uint32_t *next;
    uint32_t *ovf_list, *ovf_count;
    unsigned long long *vis;
    uint4 *stack;
    uint32_t *epochs;
    uint32_t vcap, scap, emit, last_tier;
    uint32_t live_lanes;  // lanes [live_lanes, 64) of every wave exit at once
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

// tier-0 lanes with scratch per CU (36 KB each)
#ifndef KETO_XLANES_PER_CU
#define KETO_XLANES_PER_CU 128
#endif

__global__ __launch_bounds__(256) void expand_kernel(ExpandParams P) {
    const DevSnapshot &s = P.s;
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long *vis = P.vis + (size_t)gl * P.vcap;
    uint4 *stk = P.stack + (size_t)gl * P.scap;
    uint32_t epoch = P.epochs[gl];
    const uint32_t nq = P.qlist ? *P.qlist_count : P.n;
    const uint32_t vmask = P.vcap - 1;
    if (__lane_id() >= P.live_lanes) return;  // no wave-level operations below
    unsigned long long c_rows = 0, c_edges = 0, c_out = 0;
    while (true) {
        uint32_t my = atomicAdd(P.next, 1u);
        if (my >= nq) break;
        const uint32_t q = P.qlist ? P.qlist[my] : my;
        if (P.emit && P.err[q] != 0) continue;  // count pass gave up on this root
        const keto_subject_set R = P.roots[q];
        int32_t d = R.max_depth;
        if (d <= 0 || P.max_depth < d) d = P.max_depth;  // :56-58
        uint32_t root = resolve_node(s, R.ns, R.obj, R.rel);
        epoch++;
        uint32_t vcount = 0;
        bool ovf = false;
        uint64_t cnt = 0;
        keto_tree_node *out = P.emit ? P.out + P.offsets[q] : nullptr;
        auto emit = [&](uint32_t type, uint32_t skey, uint32_t nch) {
            if (out) out[cnt] = api_node(s, type, skey, nch);
            cnt++;
        };
        uint64_t rows = 0, edges = 0;
        if (!(root & VIRT_BIT)) {
            uint32_t key = root;
            if (s.vkey && ri_shared(node_ri(s, root))) key = s.vkey[root];
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
                        if (s.vkey && ri_shared(node_ri(s, c))) ck = s.vkey[c];
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

}  // namespace

void run_expand(const Snapshot &s, Stream &st, const ExpandLaunch &L) {
    constexpr uint32_t BLOCK = 256;
    if (L.n == 0) return;
    if (L.n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    const uint32_t cus = (uint32_t)num_cus(s.device);
    const Tier t[3] = {Tier{cus * KETO_XLANES_PER_CU, 1u << 12, 256}, Tier{256, 1u << 18, 1u << 13}, Tier{8, 1u << 24, 1u << 18}};
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
        // tier 0: one-wave blocks, so a batch of a few thousand roots spreads over many CUs
        // instead of filling a handful of them (each lane walks a whole tree)
        // and a batch smaller than the scratch's lanes runs with fewer live lanes per wave: each
        // lane's DFS then shares its wave's issue with fewer divergent walks
        P.live_lanes = 64;
        if (tier == 0) {
            const uint64_t waves = lanes / 64;
            P.live_lanes = (uint32_t)std::min<uint64_t>(64, (L.n + waves - 1) / waves);
            lanes = (uint32_t)std::min<uint64_t>(lanes, (L.n + P.live_lanes - 1) / P.live_lanes * 64);
        }
        const uint32_t bs = std::min<uint32_t>(tier == 0 ? 64 : BLOCK, lanes);  // every launched lane owns scratch
        hipLaunchKernelGGL(expand_kernel, dim3(lanes / bs), dim3(bs), 0, st.stream, P);
        KETO_HIP(hipGetLastError());
    }
}

}  // namespace keto
