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
    const void *queries;  // keto_query (32 B) or keto_query16 records
    uint32_t n;
    int32_t max_depth;
    uint4 *resolved;  // [2n], in work order: heavy from the front, light from the back
    uint32_t *ctrl;   // [0] heavy count, [1] light count; null: batch order (the frontier engine)
};

#include "resolve_query.inc"

// Q16: keto_query16 records (include/keto_mi355x.h: one 16-byte load per query)
template <bool Q16>
__global__ __launch_bounds__(256) void resolve_kernel(ResolveParams P) {
    const DevSnapshot &s = P.s;
    const Tables T = global_tables(s);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = __lane_id();
    const bool valid = i < P.n;
    bool heavy_cls = false;
    uint4 r0 = make_uint4(0, 0, 0, 0), R = make_uint4(NONE32, NONE32, NONE32, NONE32);
    if (valid) {
        uint32_t wgt = 0;
        if constexpr (Q16) {
            const uint4 a = reinterpret_cast<const uint4 *>(P.queries)[i];  // {obj, s_obj, ns | rel | s_rel, s_ns | kind | depth}
            resolve_query(s, T, a.z & 0xFFFu, a.x, (a.z >> 12) & 0x3FFu, (a.w >> 12) & 1u, a.y, a.w & 0xFFFu, a.z >> 22,
                          (int32_t)(int16_t)(a.w >> 16), P.max_depth, i, P.ctrl != nullptr, r0, R, wgt);
        } else {
            const uint4 *qr = reinterpret_cast<const uint4 *>(static_cast<const keto_query *>(P.queries) + i);
            const uint4 a = qr[0], b = qr[1];
            resolve_query(s, T, a.x, a.y, a.z, a.w, b.x, b.y, b.z, (int32_t)b.w, P.max_depth, i, P.ctrl != nullptr, r0, R, wgt);
        }
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

void run_resolve(const Snapshot &s, Stream &st, const void *queries, bool q16, uint64_t n, int32_t max_depth, bool ordered) {
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
    if (q16) hipLaunchKernelGGL(resolve_kernel<true>, dim3((uint32_t)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st.stream, P);
    else hipLaunchKernelGGL(resolve_kernel<false>, dim3((uint32_t)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st.stream, P);
    KETO_HIP(hipGetLastError());
}

}  // namespace keto
