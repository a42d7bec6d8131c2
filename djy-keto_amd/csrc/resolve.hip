// gfx950 batch pre-pass shared by both Check kernels: resolve every query once, then order
// the batch longest-first.
//
// Per query (one lane each, no persistent loop -- every step is a fixed handful of
// independent loads, so plain oversubscription hides the latency):
//   * root node of (namespace, object, relation): entity rank table, phantom entity for objects
//     that hold no tuple, virtual node for unconfigured namespaces / relations
//     (engine.go:76-100 resolution of the request tuple);
//   * subject index: subject id, or the node of a subject set (no phantom: a set that holds
//     no tuple is a subject of nothing);
//   * the subject's reverse row: length, and its entries when short (<= PROBE_K) so the
//     interpreter answers membership from registers;
//   * the effective depth (engine.go:82-84: request depth if 0 < d <= global max);
//   * a cost class from the root's path-count weight.
// Records are written in work order (heavy class first), so the interpreters start a query
// from ONE 32-byte record at their queue position instead of 4-6 dependent round trips, and
// the longest walks start at the beginning of the batch instead of forming its tail.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"

namespace keto {
namespace {

struct ResolveParams {
    DevSnapshot s;
    const keto_query *queries;
    uint32_t n;
    int32_t max_depth;
    uint4 *resolved;  // [2n], in work order: heavy from the front, light from the back
    uint32_t *ctrl;   // [0] heavy count, [1] light count; null: batch order (the frontier engine)
};

__device__ __forceinline__ uint32_t w8(const uint4 &v0, const uint4 &v1, uint32_t j) {
    return j < 4 ? wword(v0, j) : wword(v1, j - 4);
}

__global__ __launch_bounds__(256) void resolve_kernel(ResolveParams P) {
    const DevSnapshot &s = P.s;
    const Tables T = global_tables(s);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = __lane_id();
    const bool valid = i < P.n;
    bool heavy_cls = false;
    uint4 r0 = make_uint4(0, 0, 0, 0), R = make_uint4(NONE32, NONE32, NONE32, NONE32);
    if (valid) {
        const uint4 *qr = reinterpret_cast<const uint4 *>(P.queries + i);
        const uint4 a = qr[0], b = qr[1];
        const uint32_t qns = a.x, qobj = a.y, qrel = a.z, qkind = a.w;
        const uint32_t qsobj = b.x, qsns = b.y, qsrel = b.z;
        int32_t d0 = (int32_t)b.w;
        if (d0 <= 0 || P.max_depth < d0) d0 = P.max_depth;
        const uint32_t d = (uint32_t)std::min<int32_t>(d0, 0xFFFF);  // deeper walks overflow every scratch tier
        // root and subject-set entities: two independent rank-table loads
        const bool want_r = qns < s.n_ns;
        const uint32_t er0 = ent_lookup(s, qns, qobj);
        const uint32_t es = qkind == 1 ? ent_lookup(s, qsns, qsobj) : NONE32;
        uint32_t er = er0;
        uint32_t root = VIRT_BIT | (0x7FFFu << 16) | 0xFFFFu;  // unknown namespace
        if (want_r) {
            if (er == NONE32) er = T.ns[qns + 1].ent_base - 1;  // phantom entity: holds no tuple
            root = t_node(T, qns, er, qrel);
        }
        uint32_t sidx = NONE32;
        if (qkind == 1) {
            if (es != NONE32) {
                const uint32_t sn = t_node(T, qsns, es, qsrel);
                if (!(sn & VIRT_BIT)) sidx = s.n_uuids + sn;
            }
        } else if (qsobj < s.n_uuids) {
            sidx = qsobj;
        }
        // reverse-row offsets and the root weight: independent loads
        uint32_t rb = 0, re = 0, wgt = 0;
        if (sidx != NONE32) {
            rb = s.rev_off[sidx];
            re = s.rev_off[sidx + 1];
        }
        if (P.ctrl && !(root & VIRT_BIT)) wgt = s.weight[root];  // (the work order's cost class)
        const uint32_t len = re - rb;
        const bool heavy = len > PROBE_K;
        if (!heavy && len > 0) {
            const uint4 *w0 = win(s.rev_nodes, rb);
            const uint4 v0 = w0[0], v1 = w0[1];  // PROBE_K = 4 entries span at most two windows
            const uint32_t o = (uint32_t)((reinterpret_cast<uintptr_t>(s.rev_nodes + rb) >> 2) & 3);
            R.x = w8(v0, v1, o);
            R.y = len > 1 ? w8(v0, v1, o + 1) : NONE32;
            R.z = len > 2 ? w8(v0, v1, o + 2) : NONE32;
            R.w = len > 3 ? w8(v0, v1, o + 3) : NONE32;
        }
        // the second record is the whole subject test: its reverse row, or {subject, START_R_HEAVY,
        // filter of the row} (layout.hpp subj_filter_bits)
        if (heavy) {
            uint64_t f = ~0ull;
            if (len <= FILTER_MAX_LEN) {  // 16-byte windows of the row, two loads in flight
                f = 0;
                const uint32_t w0 = rb & ~3u;
                for (uint32_t j = w0; j < re; j += 8) {
                    const uint4 a = *reinterpret_cast<const uint4 *>(s.rev_nodes + j);
                    const uint4 b = j + 4 < re ? *reinterpret_cast<const uint4 *>(s.rev_nodes + j + 4) : make_uint4(0, 0, 0, 0);
                    for (uint32_t k = 0; k < 8; k++) {
                        const uint32_t e = j + k;
                        if (e >= rb && e < re) f |= subj_filter_bits(k < 4 ? wword(a, k) : wword(b, k - 4));
                    }
                }
            }
            R = make_uint4(sidx, START_R_HEAVY, (uint32_t)f, (uint32_t)(f >> 32));
        }
        // x root, y subject index, z depth | hash-probe flag, w query index
        r0 = make_uint4(root, sidx, d | (heavy ? START_HEAVY : 0u), i);
        heavy_cls = wgt >= HEAVY_WEIGHT;
    }
    if (!P.ctrl) {  // the frontier engine needs no work order: position = query index, no atomics
        if (valid) {
            P.resolved[2 * (size_t)i] = r0;
            P.resolved[2 * (size_t)i + 1] = R;
        }
        return;
    }
    // order: one atomic per class per wavefront
    const unsigned long long mh = __ballot(valid && heavy_cls), ml = __ballot(valid && !heavy_cls);
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t bh = 0, bl = 0;
    const int leader = __ffsll((long long)(mh | ml)) - 1;
    if ((int)lane == leader) {
        if (mh) bh = atomicAdd(&P.ctrl[0], (uint32_t)__popcll(mh));
        if (ml) bl = atomicAdd(&P.ctrl[1], (uint32_t)__popcll(ml));
    }
    if (leader >= 0) {
        bh = __shfl(bh, leader);
        bl = __shfl(bl, leader);
    }
    if (valid) {
        const uint32_t pos = heavy_cls ? bh + (uint32_t)__popcll(mh & below) : P.n - 1 - (bl + (uint32_t)__popcll(ml & below));
        P.resolved[2 * (size_t)pos] = r0;
        P.resolved[2 * (size_t)pos + 1] = R;
    }
}

}  // namespace

void run_resolve(const Snapshot &s, Stream &st, const keto_query *queries, uint64_t n, int32_t max_depth, bool ordered) {
    ensure_lists(st, n);
    if (ordered) KETO_HIP(hipMemsetAsync(st.order_ctrl, 0, 8, st.stream));
    ResolveParams P{};
    P.s = s.dev;
    P.queries = queries;
    P.n = (uint32_t)n;
    P.max_depth = max_depth;
    P.resolved = st.resolved;
    P.ctrl = ordered ? st.order_ctrl : nullptr;
    constexpr uint32_t BLOCK = 256;
    hipLaunchKernelGGL(resolve_kernel, dim3((uint32_t)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st.stream, P);
    KETO_HIP(hipGetLastError());
}

}  // namespace keto
