// TEST/DEBUG TOOL ONLY: keto_partition_* in the CPU emulation.  The closure path (csrc/partition.hip,
// csrc/devprim.hip) is not emulated -- its kernels are written for 256-thread blocks of 64-lane
// waves (ballot ranks, one digit per thread), which the one-lane emulation cannot run.  A job of
// several ranks runs the distributed frontier (csrc/frontier_dist.hip) as the library does; the
// queries it routes to the closure path come back with out_err = -1 here, so a test can compare
// every other decision with the oracle.  Every other entry point fails loudly.
#include <algorithm>
#include <memory>
#include <vector>

#include "../../djy-keto_amd/csrc/engine.hpp"
#include "../../djy-keto_amd/csrc/frontier_dist.hpp"

namespace keto {
struct PartitionHandle {
    DistEngine *dist = nullptr;
    keto_partition_stats last{};
    std::vector<keto_partition_level> levels;
    std::vector<keto_partition_generation> gens;
    std::vector<keto_tree_node> xnodes;
    std::vector<uint64_t> xoffs;
    std::vector<int32_t> xerr;
    ~PartitionHandle() {
        if (dist) dist_free(dist);
    }
};
[[noreturn]] static void unavailable() { throw Error(KETO_E_DEVICE, "the closure path of keto_partition_* is not part of the CPU emulation"); }
PartitionHandle *partition_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, bool device_ptrs,
                                  const keto_collective *coll, const keto_limits *limits, bool force_dist, const Placement &place) {
    if (!coll || (coll->world < 2 && !force_dist)) unavailable();
    auto P = std::make_unique<PartitionHandle>();
    keto_limits lim = limits ? *limits : keto_limits{5, 100};
    P->dist = dist_create(cfg, tuples, n, device_ptrs, *coll, lim, place);
    return P.release();
}
void partition_check_many(PartitionHandle *P, uint32_t nb, const keto_query *const *q, const uint64_t *n, uint8_t *const *allowed,
                          int32_t *const *err, uint32_t flags) {
    if (flags & KETO_F_COUNT_WORK) unavailable();
    for (uint32_t k = 0; k < nb; k++) {
        std::vector<uint32_t> routed;
        DistStats ds{};
        dist_check(*P->dist, q[k], n[k], allowed[k], err[k], (flags & KETO_F_ERR_DETAIL) != 0, routed, ds);
        for (uint32_t i : routed) err[k][i] = -1;
        P->last = keto_partition_stats{};
        P->last.batches = 1;
        P->last.generations = ds.generations;
        P->last.goals = ds.goals;
        P->last.routed = ds.routed;
        P->last.exchange_bytes = ds.bytes_exchanged;
        P->last.device_s = ds.device_s;
        P->last.exchange_s = ds.exchange_s;
        P->last.run_s = ds.wall_s;
        P->levels.clear();
        P->gens.clear();
        for (const keto_partition_level &l : dist_levels(*P->dist))
            P->gens.push_back(keto_partition_generation{l.objects, l.request_bytes, l.tuples, l.tuple_bytes_sent, l.ms});
    }
}
void partition_check(PartitionHandle *P, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, uint32_t flags) {
    partition_check_many(P, 1, &q, &n, &allowed, &err, flags);
}
uint64_t partition_expand(PartitionHandle *P, const keto_subject_set *roots, uint64_t n) {
    DistExpandStats xs;
    dist_expand(*P->dist, roots, n, P->xnodes, P->xoffs, P->xerr, xs);
    P->last = keto_partition_stats{};
    P->last.batches = 1;
    P->last.levels = xs.levels;
    P->last.objects = xs.rows;
    P->last.tuples = xs.entries;
    P->last.bytes_sent = xs.bytes_sent;
    P->levels = xs.per_level;
    return P->xoffs[n];
}
void partition_expand_result(PartitionHandle *P, keto_tree_node *nodes, uint64_t cap, uint64_t *offsets, int32_t *err) {
    const uint64_t n = P->xoffs.empty() ? 0 : P->xoffs.size() - 1, total = n ? P->xoffs[n] : 0;
    if (total > cap) throw Error(KETO_E_CAPACITY, "expand output");
    std::copy(P->xoffs.begin(), P->xoffs.end(), offsets);
    std::copy(P->xerr.begin(), P->xerr.begin() + n, err);
    std::copy(P->xnodes.begin(), P->xnodes.begin() + total, nodes);
}
void partition_stats(PartitionHandle *P, keto_partition_stats *out) { *out = P->last; }
void partition_levels(PartitionHandle *P, keto_partition_level *out, uint32_t cap, uint32_t *n) {
    *n = (uint32_t)P->levels.size();
    for (uint32_t i = 0; i < cap && i < P->levels.size(); i++) out[i] = P->levels[i];
}
void partition_generations(PartitionHandle *P, keto_partition_generation *out, uint32_t cap, uint32_t *n) {
    *n = (uint32_t)P->gens.size();
    for (uint32_t i = 0; i < cap && i < P->gens.size(); i++) out[i] = P->gens[i];
}
void partition_free(PartitionHandle *P) { delete P; }
}  // namespace keto
