// gfx950 batched Expand (expand/engine.go:54-124).
//
// expand_wave (the default): one wavefront per root.  The walk is the reference's DFS in
// pre-order -- a child's subtree is finished before its next sibling is looked at, because the
// visited set (global per call, root included, :69-72, :112-117) decides what a later sibling
// becomes -- but every row is read by the whole wave at once: 64 entries per coalesced load,
// with the entries' own loads (row bounds, visited alias, the API form's entity and relation
// name) issued together.  Only the decision per subject-set entry (visited? expand?) is
// sequential, in LDS: the visited set (open addressing) and the DFS stack live there.  Nodes are
// written once, in pre-order, to the wave's staging region; a finished tree moves to the batch's
// stage in one coalesced copy, and the host's offsets place the trees in root order.
//
// expand_kernel: one lane per root, two passes (count, emit), per-lane visited tables in HBM --
// the fallback for the rare root whose visited set, stack or tree outgrows expand_wave's LDS /
// staging space (tiered scratch up to 2^23 visited nodes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

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
            uint32_t b, e;
            row_span(s.all_off, s.reloc, root, b, e);
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
                        uint32_t cb, ce;
                        row_span(s.all_off, s.reloc, c, cb, ce);
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

constexpr uint32_t XW_VIS = 2048;   // visited keys per wave (LDS, half full at most)
constexpr uint32_t XW_STACK = 64;   // DFS frames per wave (LDS): the walk is at most max_read_depth deep
constexpr uint32_t XW_PRIV = 8192;  // staged nodes per wave; a larger tree goes to the fallback
constexpr uint32_t XW_EMPTY = NONE32;
#ifdef KETO_CPUEMU
constexpr uint32_t XWW = 1;  // the CPU emulation runs one-lane waves (tools/cpuemu)
#else
constexpr uint32_t XWW = 64;  // wavefront width: the lanes that read one row chunk
#endif

struct ExpandWaveParams {
    DevSnapshot s;
    const keto_subject_set *roots;
    uint32_t n;
    int32_t max_depth;
    uint32_t priv_cap;              // <= XW_PRIV (tests lower it: KETO_XW_PRIV, mixed wave / fallback batches)
    uint2 *priv;                    // [grid][XW_PRIV]: the tree being walked, as walk records (below)
    uint2 *stage;                   // finished trees, in completion order
    unsigned long long stage_cap;
    unsigned long long *stage_top;
    unsigned long long *sizes, *soff;  // [n]: nodes of each tree, its offset in `stage` (NONE: fallback)
    int32_t *err;
    uint32_t *next;                 // root queue
    const uint32_t *order;          // queue position -> root (expand_order: heavy roots first); null: batch order
    uint32_t *fb_list, *fb_count;   // roots for expand_kernel
    unsigned long long *counters;   // rows, edges, -, out nodes
    // span output (keto_expand_batch_spans): a finished tree goes straight to dout (the caller's
    // pinned buffer, mapped, or a device buffer) at the run dtop hands it, in API form -- root i at
    // first[i] -- while the other roots still walk; null: the stage, placed in root order later
    keto_tree_node *dout;
    unsigned long long dcap, *dtop;
    uint64_t *first;
};

// A walk record is what the DFS decides about a node: {subject key, n_children | XR_UNION}.  The
// API form (namespace, object uuid, relation name: two more dependent loads per node) is made by
// expand_place, in parallel over the batch, off the walk's serial chain of row loads.
constexpr uint32_t XR_UNION = 1u << 31;

__device__ __forceinline__ uint2 walk_rec(uint32_t skey, bool un, uint32_t nch) {
    return make_uint2(skey, un ? (nch | XR_UNION) : 0u);
}

// lane j's x for the whole wave, j uniform: a scalar read instead of an LDS-crossbar shuffle
__device__ __forceinline__ uint32_t wave_at(uint32_t x, uint32_t j) {
#ifdef KETO_CPUEMU
    return __shfl(x, j);
#else
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)j);
#endif
}

// The wave kernel's queue order: roots whose path-count weight (the snapshot's scheduling weights,
// a capped count of the paths below a node) reaches `heavy` first, the rest after -- a batch's walk
// lasts at least as long as its longest tree, which should not start last in some wave's queue.
// One atomic per class per wave (as resolve.hip's heavy-first work order).
__global__ __launch_bounds__(256) void expand_order(DevSnapshot s, const keto_subject_set *roots, uint32_t n, uint32_t heavy,
                                                    uint32_t *order, uint32_t *ctr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, lane = __lane_id();
    const bool valid = i < n;
    bool hv = false;
    if (valid) {
        const uint32_t node = resolve_node(s, roots[i].ns, roots[i].obj, roots[i].rel);
        hv = !(node & VIRT_BIT) && s.weight[node] >= heavy;
    }
    const unsigned long long mh = __ballot(valid && hv), ml = __ballot(valid && !hv), below = (1ull << lane) - 1ull;
    uint32_t bh = 0, bl = 0;
    const int leader = __ffsll((long long)(mh | ml)) - 1;
    if ((int)lane == leader) {
        if (mh) bh = atomicAdd(&ctr[0], (uint32_t)__popcll(mh));
        if (ml) bl = atomicAdd(&ctr[1], (uint32_t)__popcll(ml));
    }
    if (leader >= 0) {
        bh = __shfl(bh, leader);
        bl = __shfl(bl, leader);
    }
    if (valid) order[hv ? bh + (uint32_t)__popcll(mh & below) : n - 1 - (bl + (uint32_t)__popcll(ml & below))] = i;
}

// one root per wavefront: see the file comment
__global__ __launch_bounds__(64) void expand_wave(ExpandWaveParams P) {
    __shared__ uint32_t vis[XW_VIS];
    __shared__ uint4 stk[XW_STACK];
    const DevSnapshot &s = P.s;
    const uint32_t lane = threadIdx.x;
    uint2 *priv = P.priv + (size_t)blockIdx.x * XW_PRIV;
    unsigned long long c_rows = 0, c_edges = 0, c_out = 0;
    for (;;) {
        uint32_t q = 0;
        if (lane == 0) q = atomicAdd(P.next, 1u);
        q = __shfl(q, 0);
        if (q >= P.n) break;
        if (P.order) q = P.order[q];
        for (uint32_t i = lane; i < XW_VIS; i += XWW) vis[i] = XW_EMPTY;
        __syncthreads();
        const keto_subject_set R = P.roots[q];
        int32_t d = R.max_depth;
        if (d <= 0 || P.max_depth < d) d = P.max_depth;  // :56-58
        const uint32_t root = resolve_node(s, R.ns, R.obj, R.rel);
        uint32_t cnt = 0, vcount = 0, sp = 0;
        uint64_t rows = 0, edges = 0;
        bool fail = false;
        // visited check-and-insert (CheckAndAddVisited), in walk order: the whole wave probes XWW
        // consecutive slots at once -- the key is present when it comes before the first empty slot
        // of the probe sequence, else it goes into that slot (one LDS read per probe window instead
        // of one per slot on lane 0; C4's 4,096 roots: walk 0.650 -> 0.628 ms with wave_at below)
        auto visit = [&](uint32_t key) -> bool {
            for (uint32_t h = (uint32_t)mix64(key) & (XW_VIS - 1);; h = (h + XWW) & (XW_VIS - 1)) {
                const uint32_t v = vis[(h + lane) & (XW_VIS - 1)];
                const unsigned long long hit = __ballot(v == key), emp = __ballot(v == XW_EMPTY);
                if (!hit && !emp) continue;
                const uint32_t fh = hit ? (uint32_t)__ffsll((long long)hit) - 1 : XWW;
                const uint32_t fe = emp ? (uint32_t)__ffsll((long long)emp) - 1 : XWW;
                if (fh < fe) return true;
                if (2 * (vcount + 1) > XW_VIS) {  // table full: the fallback walks this root
                    fail = true;
                    return false;
                }
                if (lane == fe) vis[(h + fe) & (XW_VIS - 1)] = key;
                vcount++;
                return false;
            }
        };
        if (!(root & VIRT_BIT)) {
            uint32_t key = root;
            if (s.vkey && ri_shared(node_ri(s, root))) key = s.vkey[root];
            visit(key);  // the root is visited (:69-72)
            uint32_t b, e;
            row_span(s.all_off, s.reloc, root, b, e);
            rows++;
            if (b != e && e - b >= XR_UNION) fail = true;  // (a row past 2^31 tuples: the fallback)
            if (b != e && !fail) {  // no tuples on the first page -> nil (:97-99)
                if (lane == 0) priv[0] = walk_rec(SKEY_SET | root, d > 1, e - b);  // :101-104
                cnt = 1;
                uint4 top = make_uint4(b, e, (uint32_t)d, 0);
                while (d > 1 && !fail) {
                    if (top.x == top.y) {
                        if (sp == 0) break;
                        top = stk[--sp];
                        continue;
                    }
                    // the next (up to) 64 entries of the row, and each entry's own loads, together
                    const uint32_t m = std::min<uint32_t>(XWW, top.y - top.x);
                    const bool in = lane < m;
                    const uint32_t sk = in ? s.all_subj[top.x + lane] : 0u;
                    const bool set = in && (sk & SKEY_SET);
                    uint32_t ck = 0, cb = 0, ce = 0;
                    const uint2 nd = walk_rec(sk, false, 0);
                    if (set) {
                        const uint32_t c = sk & ~SKEY_SET;
                        ck = c;
                        if (s.vkey && ri_shared(node_ri(s, c))) ck = s.vkey[c];
                        row_span(s.all_off, s.reloc, c, cb, ce);
                    }
                    const unsigned long long setm = __ballot(set);
                    uint32_t pos = 0;
                    for (;;) {
                        const unsigned long long rest = pos < XWW ? setm & (~0ull << pos) : 0ull;
                        const uint32_t j = rest ? (uint32_t)__ffsll((long long)rest) - 1 : m;
                        // subject ids before the next subject set: leaves (:60-67), written together
                        const uint32_t nl = j - pos;
                        if (lane >= pos && lane < j && cnt + (lane - pos) < P.priv_cap) priv[cnt + (lane - pos)] = nd;
                        cnt += nl;
                        edges += nl;
                        if (cnt > P.priv_cap) {
                            fail = true;
                            break;
                        }
                        if (j >= m) {
                            top.x += m;
                            break;
                        }
                        // the subject set at j, in walk order
                        const uint32_t ckj = wave_at(ck, j), cbj = wave_at(cb, j), cej = wave_at(ce, j);  // (j is uniform)
                        edges++;
                        pos = j + 1;
                        bool expand = false;
                        if (!visit(ckj)) {  // a revisit is nil -> a leaf (:112-117)
                            if (fail) break;
                            rows++;
                            expand = cbj != cej && top.z - 1 > 1;
                            if (expand && cej - cbj >= XR_UNION) {
                                fail = true;
                                break;
                            }
                        }
                        if (lane == j && cnt < P.priv_cap) priv[cnt] = walk_rec(nd.x, expand, cej - cbj);
                        if (++cnt > P.priv_cap) {
                            fail = true;
                            break;
                        }
                        if (expand) {  // the child's subtree before the next sibling
                            if (sp >= XW_STACK) {
                                fail = true;
                                break;
                            }
                            if (lane == 0) stk[sp] = make_uint4(top.x + pos, top.y, top.z, 0);
                            sp++;
                            top = make_uint4(cbj, cej, top.z - 1, 0);
                            break;
                        }
                    }
                }
            }
        }
        __syncthreads();  // (the wave's LDS writes before the next root clears them)
        unsigned long long off = 0;
        if (P.dout && !fail) {  // span output: the tree's run of the output, written now
            if (lane == 0 && cnt) off = atomicAdd(P.dtop, (unsigned long long)cnt);
            off = __shfl(off, 0);
            if (off + cnt <= P.dcap)  // (past the capacity: only counted -- the caller learns the size it needs)
                for (uint32_t i0 = 0; i0 < cnt; i0 += 4 * XWW) {  // four records per lane in flight
                    uint2 r[4];
#pragma unroll
                    for (uint32_t u = 0; u < 4; u++) {
                        const uint32_t i = i0 + u * XWW + lane;
                        r[u] = i < cnt ? priv[i] : make_uint2(0, 0);
                    }
#pragma unroll
                    for (uint32_t u = 0; u < 4; u++) {
                        const uint32_t i = i0 + u * XWW + lane;
                        const bool un = (r[u].y & XR_UNION) != 0u;
                        if (i < cnt) P.dout[off + i] = api_node(s, un ? 1u : 4u, r[u].x, un ? r[u].y & ~XR_UNION : 0u);
                    }
                }
            if (lane == 0) {
                P.sizes[q] = cnt;
                P.first[q] = off;
                P.soff[q] = 0;
                P.err[q] = 0;
            }
            c_rows += rows;
            c_edges += edges;
            c_out += cnt;
            continue;
        }
        if (!fail && cnt) {
            if (lane == 0) off = atomicAdd(P.stage_top, (unsigned long long)cnt);
            off = __shfl(off, 0);
            if (off + cnt > P.stage_cap) fail = true;
        }
        if (fail) {
            if (lane == 0) {
                P.soff[q] = ~0ull;
                P.fb_list[atomicAdd(P.fb_count, 1u)] = q;
            }
            continue;
        }
        for (uint32_t i = lane; i < cnt; i += XWW) P.stage[off + i] = priv[i];
        if (lane == 0) {
            P.sizes[q] = cnt;
            P.soff[q] = off;
            P.err[q] = 0;
        }
        c_rows += rows;
        c_edges += edges;
        c_out += cnt;
    }
    if (P.counters && lane == 0) {
        atomicAdd(&P.counters[0], c_rows);
        atomicAdd(&P.counters[1], c_edges);
        atomicAdd(&P.counters[3], c_out);
    }
}

// trees from the stage into their root-order positions of the output, each walk record made into
// its API form on the way (Mapper.ToTree, uuid_mapping.go:356-385)
__global__ __launch_bounds__(256) void expand_place(DevSnapshot s, const uint2 *stage, const unsigned long long *soff,
                                                    const unsigned long long *sizes, const uint64_t *offsets, uint32_t n,
                                                    keto_tree_node *out) {
    for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
        const unsigned long long so = soff[q];
        if (so == ~0ull) continue;  // a fallback root: expand_kernel's emit pass writes it
        const unsigned long long c = sizes[q];
        for (unsigned long long i = threadIdx.x; i < c; i += blockDim.x) {
            const uint2 r = stage[so + i];
            const bool un = (r.y & XR_UNION) != 0u;
            out[offsets[q] + i] = api_node(s, un ? 1u : 4u, r.x, un ? r.y & ~XR_UNION : 0u);
        }
    }
}

// span output: the runs of the fallback roots (expand_kernel's count pass sized them), taken from
// the same counter as the wave kernel's trees; an errored root gets none
__global__ __launch_bounds__(256) void expand_fb_spans(const uint32_t *fb_list, const uint32_t *fb_count, uint32_t n,
                                                       const unsigned long long *sizes, const int32_t *err, unsigned long long *dtop,
                                                       uint64_t *first) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (fb_list ? j >= *fb_count : j >= n) return;  // (no list: every root is a fallback root)
    const uint32_t q = fb_list ? fb_list[j] : j;
    first[q] = err[q] ? 0ull : atomicAdd(dtop, sizes[q]);
}

// root-order offsets of the trees on the device: offsets[i + 1] = offsets[i] + (err[i] ? 0 :
// sizes[i]) -- one block, chunks of XO_RUN * blockDim roots with a carried sum (a batch is a few
// thousand roots), so the host reads offsets and errors back in one copy
constexpr uint32_t XO_BLOCK = 1024, XO_RUN = 4;
__global__ __launch_bounds__(XO_BLOCK) void expand_offsets(const unsigned long long *sizes, const int32_t *err, uint32_t n,
                                                         unsigned long long *offsets) {
    __shared__ unsigned long long wsum[XO_BLOCK / 64 + 1];
    const uint32_t t = threadIdx.x, lane = __lane_id(), w = t >> 6, nw = (blockDim.x + 63) >> 6;
    unsigned long long carry = 0;
    if (t == 0) offsets[0] = 0;
    for (uint32_t b = 0; b < n; b += blockDim.x * XO_RUN) {
        unsigned long long x[XO_RUN], acc = 0;
        const uint32_t i0 = b + t * XO_RUN;
        for (uint32_t k = 0; k < XO_RUN; k++) {
            const uint32_t i = i0 + k;
            x[k] = (i < n && !err[i]) ? sizes[i] : 0ull;
            acc += x[k];
        }
        unsigned long long v = acc;
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const unsigned long long y = __shfl_up(v, off);
            if (lane >= off) v += y;
        }
        if (lane == 63 || t == blockDim.x - 1) wsum[w] = v;  // (the wave's last lane)
        __syncthreads();
        if (t == 0) {
            unsigned long long s = 0;
            for (uint32_t k = 0; k < nw; k++) {
                const unsigned long long y = wsum[k];
                wsum[k] = s;
                s += y;
            }
            wsum[nw] = s;
        }
        __syncthreads();
        unsigned long long o = carry + wsum[w] + v - acc;
        for (uint32_t k = 0; k < XO_RUN; k++) {
            o += x[k];
            if (i0 + k < n) offsets[i0 + k + 1] = o;
        }
        carry += wsum[nw];
        __syncthreads();
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
        P.qlist = tier == 0 ? L.list : list[tier - 1];
        P.qlist_count = tier == 0 ? L.list_count : &sc.ctrl[3 + tier - 1];
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
            const uint64_t waves = lanes / 64, nr = L.list ? L.nl : L.n;
            P.live_lanes = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, (nr + waves - 1) / waves));
            lanes = (uint32_t)std::max<uint64_t>(64, std::min<uint64_t>(lanes, (nr + P.live_lanes - 1) / P.live_lanes * 64));
        }
        const uint32_t bs = std::min<uint32_t>(tier == 0 ? 64 : BLOCK, lanes);  // every launched lane owns scratch
        hipLaunchKernelGGL(expand_kernel, dim3(lanes / bs), dim3(bs), 0, st.stream, P);
        KETO_HIP(hipGetLastError());
    }
}

static size_t xal(size_t b) { return (b + 255) / 256 * 256; }

namespace {
// the wave kernel's buffers for n roots (grown as needed), its parameters, the heavy-first queue,
// and the fallback pass's launch: what both output forms share
struct XwRun {
    ExpandWaveParams P;
    ExpandLaunch F;
    bool wave;
};
XwRun xw_prepare(const Snapshot &s, Stream &st, const keto_subject_set *d_roots, uint64_t n, int32_t max_depth, size_t host_extra) {
    if (n >= (1ull << 31)) throw Error(KETO_E_LIMIT, "batch too large");
    auto &X = st.xw;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    // one-wave blocks of 9 KB LDS each, KETO_XW_BPC per CU (default 4).  C4, 4,096 roots (round 5):
    // 2 per CU 0.665 ms, 3-5 per CU 0.605-0.616 ms, 6 0.619, 8 0.633, 12 0.659 (round 4: 16 per CU,
    // every root at once, 0.73 ms): fewer waves in flight wait less on the rows they share
    static const uint64_t bpc = [] {
        const char *e = getenv("KETO_XW_BPC");
        return e ? (uint64_t)std::max(1, std::min(atoi(e), 17)) : 4ull;
    }();
    const uint64_t grid = (uint64_t)cus * bpc;
    if (!X.mem || X.ncap < n || X.grid < grid) {
        if (X.mem) KETO_HIP(hipFree(X.mem));
        X.mem = nullptr;
        uint64_t nc = 1;
        while (nc < n) nc <<= 1;
        const uint64_t sc = std::max<uint64_t>(X.stage_cap, 1u << 22);
        const size_t bytes = xal(64) + xal(grid * XW_PRIV * sizeof(uint2)) + xal(sc * sizeof(uint2)) +
                             2 * xal(nc * 8) + xal((nc + 1) * 8) + 3 * xal(nc * 4);
        KETO_HIP(hipMalloc(&X.mem, bytes));
        char *p = static_cast<char *>(X.mem);
        X.ctrl = reinterpret_cast<unsigned long long *>(p);
        p += xal(64);
        X.priv = reinterpret_cast<uint2 *>(p);
        p += xal(grid * XW_PRIV * sizeof(uint2));
        X.stage = reinterpret_cast<uint2 *>(p);
        p += xal(sc * sizeof(uint2));
        X.sizes = reinterpret_cast<unsigned long long *>(p);
        p += xal(nc * 8);
        X.soff = reinterpret_cast<unsigned long long *>(p);
        p += xal(nc * 8);
        X.offsets = reinterpret_cast<uint64_t *>(p);
        p += xal((nc + 1) * 8);
        X.err = reinterpret_cast<int32_t *>(p);
        p += xal(nc * 4);
        X.fb_list = reinterpret_cast<uint32_t *>(p);
        p += xal(nc * 4);
        X.order = reinterpret_cast<uint32_t *>(p);
        X.grid = grid;
        X.stage_cap = sc;
        X.ncap = nc;
    }
    // pinned read-back: ctrl (stage top, fallback count), offsets[n + 1], errors[n]
    const size_t hb = 64 + (n + 1) * 8 + n * 4 + host_extra;
    if (X.hpin_bytes < hb) {
        if (X.hpin) KETO_HIP(hipHostFree(X.hpin));
        X.hpin = nullptr;
        X.hpin_bytes = 0;
        KETO_HIP(hipHostMalloc(&X.hpin, 2 * hb, 0));
        X.hpin_bytes = 2 * hb;
    }
    KETO_HIP(hipMemsetAsync(X.ctrl, 0, 64, st.stream));
    // KETO_EXPAND_WAVE=0 (A/B, tests): every root through the lane kernel
    const char *ew = getenv("KETO_EXPAND_WAVE");
    const bool wave = !(ew && ew[0] == '0');
    ExpandWaveParams P{};
    P.s = s.dev;
    P.roots = d_roots;
    P.n = (uint32_t)n;
    P.max_depth = max_depth;
    const char *pc = getenv("KETO_XW_PRIV");
    P.priv_cap = pc ? (uint32_t)std::max(1, std::min(atoi(pc), (int)XW_PRIV)) : XW_PRIV;
    P.priv = X.priv;
    P.stage = X.stage;
    P.stage_cap = X.stage_cap;
    P.stage_top = X.ctrl;
    P.next = reinterpret_cast<uint32_t *>(X.ctrl + 1);
    P.fb_count = reinterpret_cast<uint32_t *>(X.ctrl + 2);
    P.fb_list = X.fb_list;
    P.sizes = X.sizes;
    P.soff = X.soff;
    P.err = X.err;
    P.counters = st.counters;
    if (!X.ev[0]) {
        for (hipEvent_t &e : X.ev) KETO_HIP(hipEventCreate(&e));
    }
    KETO_HIP(hipEventRecord(X.ev[0], st.stream));
    // heavy roots first (KETO_XW_HEAVY: the weight threshold, 0 = batch order)
    const char *xh = getenv("KETO_XW_HEAVY");
    const uint32_t heavy = xh ? (uint32_t)atoi(xh) : HEAVY_WEIGHT;
    if (wave && heavy && s.dev.weight) {
        hipLaunchKernelGGL(expand_order, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st.stream, s.dev, d_roots, (uint32_t)n, heavy,
                           X.order, reinterpret_cast<uint32_t *>(X.ctrl + 3));
        KETO_HIP(hipGetLastError());
        P.order = X.order;
    }
    ExpandLaunch F{};
    F.roots = d_roots;
    F.n = n;
    F.max_depth = max_depth;
    F.sizes = reinterpret_cast<uint64_t *>(X.sizes);
    F.offsets = X.offsets;  // (root i's first node: offsets[i], read by the emit pass)
    F.err = X.err;
    F.list = wave ? X.fb_list : nullptr;
    F.list_count = wave ? P.fb_count : nullptr;
    F.nl = n;
    F.emit = false;
    return XwRun{P, F, wave};
}
// the wave kernel (or, KETO_EXPAND_WAVE=0, a memset sending every root to the fallback), then the
// fallback's count pass over the roots it left -- reading their count from the device (no host
// round trip; with none its launches end at once)
void xw_walk(const Snapshot &s, Stream &st, XwRun &R, uint64_t n) {
    auto &X = st.xw;
    if (R.wave) {
        hipLaunchKernelGGL(expand_wave, dim3((uint32_t)std::min<uint64_t>(X.grid, n)), dim3(XWW), 0, st.stream, R.P);
        KETO_HIP(hipGetLastError());
    } else {
        KETO_HIP(hipMemsetAsync(X.soff, 0xFF, n * 8, st.stream));
    }
    run_expand(s, st, R.F);
}
}  // namespace

bool expand_batch(const Snapshot &s, Stream &st, const keto_subject_set *d_roots, uint64_t n, int32_t max_depth,
                  keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_offsets, int32_t *out_err) {
    out_offsets[0] = 0;
    if (n == 0) return true;
    auto &X = st.xw;
    const uint32_t cus = (uint32_t)num_cus(s.device);
    XwRun R = xw_prepare(s, st, d_roots, n, max_depth, 0);
    ExpandLaunch &F = R.F;
    const bool wave = R.wave;
    xw_walk(s, st, R, n);
    KETO_HIP(hipEventRecord(X.ev[1], st.stream));
    hipLaunchKernelGGL(expand_offsets, dim3(1), dim3(XO_BLOCK), 0, st.stream, X.sizes, X.err, (uint32_t)n,
                       reinterpret_cast<unsigned long long *>(X.offsets));
    KETO_HIP(hipGetLastError());
    char *hp = static_cast<char *>(X.hpin);
    unsigned long long *h = reinterpret_cast<unsigned long long *>(hp);
    uint64_t *hoff = reinterpret_cast<uint64_t *>(hp + 64);
    int32_t *herr = reinterpret_cast<int32_t *>(hp + 64 + (n + 1) * 8);
    KETO_HIP(hipMemcpyAsync(h, X.ctrl, 24, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(hoff, X.offsets, (n + 1) * 8, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(herr, X.err, n * 4, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    float ms = 0;
    if (hipEventElapsedTime(&ms, X.ev[0], X.ev[1]) == hipSuccess) {  // traversal time: the walk
        X.ms_sum += ms;
        X.batches++;
    }
    std::memcpy(out_offsets, hoff, (n + 1) * 8);
    std::memcpy(out_err, herr, n * 4);
    const uint32_t nfb = wave ? (uint32_t)h[2] : (uint32_t)n;
    const uint64_t total = out_offsets[n];
    if (h[0] > X.stage_cap / 2) X.stage_cap = std::max<uint64_t>(X.stage_cap, 2 * h[0]), X.ncap = 0;  // (regrown next batch)
    if (total > out_cap || (total && !out_nodes)) return false;
    if (total == 0) return true;
    if (X.out_cap < total) {
        if (X.outbuf) KETO_HIP(hipFree(X.outbuf));
        X.outbuf = nullptr;
        X.out_cap = 0;
        KETO_HIP(hipMalloc(&X.outbuf, total * sizeof(keto_tree_node)));
        X.out_cap = total;
    }
    hipLaunchKernelGGL(expand_place, dim3((uint32_t)std::min<uint64_t>(n, cus * 16)), dim3(256), 0, st.stream, s.dev, X.stage,
                       X.soff, X.sizes, X.offsets, (uint32_t)n, X.outbuf);
    KETO_HIP(hipGetLastError());
    if (nfb) {
        F.emit = true;
        F.nl = nfb;
        F.out = X.outbuf;
        run_expand(s, st, F);
    }
    // one copy of the trees in root order (caller memory from keto_host_alloc: straight DMA).
    // (Writing them from expand_place straight into mapped pinned memory instead, over PCIe,
    // measured the same: 1.38 / 1.40 vs 1.37 / 1.38 ms API -- the copy runs at PCIe speed either way.)
    KETO_HIP(hipMemcpyAsync(out_nodes, X.outbuf, total * sizeof(keto_tree_node), hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    return true;
}

// keto_expand_batch_spans: every tree written the moment its wave finishes it, at the run the
// output's counter hands it -- straight into the caller's buffer over PCIe when it is pinned
// (keto_host_alloc), so the copy-out overlaps the other roots' walks; else into a device buffer
// copied once at the end.  The fallback roots follow (count pass, runs, emit pass).  false with
// *out_total = the nodes required when out_cap is too small (nothing of the batch is usable then).
bool expand_batch_spans(const Snapshot &s, Stream &st, const keto_subject_set *d_roots, uint64_t n, int32_t max_depth,
                        keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_first, uint32_t *out_count,
                        int32_t *out_err, uint64_t *out_total) {
    *out_total = 0;
    if (n == 0) return true;
    auto &X = st.xw;
    // the caller's buffer, as the device sees it: pinned host memory is written in place
    keto_tree_node *dout = nullptr;
    hipPointerAttribute_t pa{};
    if (out_nodes && out_cap && hipPointerGetAttributes(&pa, out_nodes) == hipSuccess && pa.type == hipMemoryTypeHost &&
        pa.devicePointer && pa.hostPointer)
        dout = reinterpret_cast<keto_tree_node *>(static_cast<char *>(pa.devicePointer) +
                                                  (reinterpret_cast<char *>(out_nodes) - static_cast<char *>(pa.hostPointer)));
    else
        (void)hipGetLastError();  // (pageable memory: not a HIP allocation)
    uint64_t dcap = out_cap;
    if (!dout) {  // a device buffer of the last batch's size (at least 1Mi nodes); a larger batch runs again
        const uint64_t want = std::min<uint64_t>(out_cap, std::max<uint64_t>({X.out_cap, X.span_hint, 1ull << 20}));
        if (X.out_cap < want) {
            if (X.outbuf) KETO_HIP(hipFree(X.outbuf));
            X.outbuf = nullptr;
            X.out_cap = 0;
            KETO_HIP(hipMalloc(&X.outbuf, std::max<uint64_t>(1, want) * sizeof(keto_tree_node)));
            X.out_cap = want;
        }
        dout = X.outbuf;
        dcap = std::min<uint64_t>(out_cap, X.out_cap);
    }
    XwRun R = xw_prepare(s, st, d_roots, n, max_depth, n * 8);
    unsigned long long *dtop = X.ctrl + 4;
    R.P.dout = dout;
    R.P.dcap = dcap;
    R.P.dtop = dtop;
    R.P.first = X.offsets;
    R.F.offsets = X.offsets;  // (the emit pass writes root q at first[q])
    xw_walk(s, st, R, n);
    KETO_HIP(hipEventRecord(X.ev[1], st.stream));
    if (R.wave) {
        hipLaunchKernelGGL(expand_fb_spans, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st.stream, X.fb_list, R.P.fb_count,
                           (uint32_t)n, X.sizes, X.err, dtop, X.offsets);
    } else {
        hipLaunchKernelGGL(expand_fb_spans, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st.stream, nullptr, nullptr,
                           (uint32_t)n, X.sizes, X.err, dtop, X.offsets);
    }
    KETO_HIP(hipGetLastError());
    char *hp = static_cast<char *>(X.hpin);
    unsigned long long *h = reinterpret_cast<unsigned long long *>(hp);
    uint64_t *hfirst = reinterpret_cast<uint64_t *>(hp + 64);
    int32_t *herr = reinterpret_cast<int32_t *>(hp + 64 + (n + 1) * 8);
    unsigned long long *hsize = reinterpret_cast<unsigned long long *>(hp + 64 + (n + 1) * 8 + ((n * 4 + 7) & ~7ull));
    KETO_HIP(hipMemcpyAsync(h, X.ctrl, 40, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(hfirst, X.offsets, n * 8, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(herr, X.err, n * 4, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipMemcpyAsync(hsize, X.sizes, n * 8, hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    float ms = 0;
    if (hipEventElapsedTime(&ms, X.ev[0], X.ev[1]) == hipSuccess) {
        X.ms_sum += ms;
        X.batches++;
    }
    const uint64_t total = h[4];
    const uint32_t nfb = R.wave ? (uint32_t)h[2] : (uint32_t)n;
    *out_total = total;
    X.span_hint = std::max<uint64_t>(X.span_hint, total + total / 4);
    if (total > out_cap || (total && !out_nodes)) return false;
    if (total > dcap) {  // past the device buffer (pageable output): once more into one of the right size
        X.span_hint = total + total / 4;
        return expand_batch_spans(s, st, d_roots, n, max_depth, out_nodes, out_cap, out_first, out_count, out_err, out_total);
    }
    for (uint64_t i = 0; i < n; i++) {
        out_err[i] = herr[i];
        out_first[i] = herr[i] ? 0 : hfirst[i];
        out_count[i] = herr[i] ? 0u : (uint32_t)hsize[i];
    }
    if (nfb) {  // the fallback roots' trees at their runs
        R.F.emit = true;
        R.F.nl = nfb;
        R.F.out = dout;
        run_expand(s, st, R.F);
    }
    if (dout == X.outbuf && total)
        KETO_HIP(hipMemcpyAsync(out_nodes, X.outbuf, total * sizeof(keto_tree_node), hipMemcpyDeviceToHost, st.stream));
    KETO_HIP(hipStreamSynchronize(st.stream));
    return true;
}

}  // namespace keto
