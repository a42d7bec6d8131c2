// Partitioned graphs' distributed frontier engine (frontier_dist.hip), as partition.hip uses it.
#pragma once

#include <vector>

#include "engine.hpp"

namespace keto {

struct DistEngine;
struct DistStats {
    uint64_t generations = 0, goals = 0, positions = 0, routed = 0, records_sent = 0, bytes_exchanged = 0, decisive = 0;
    double device_s = 0, exchange_s = 0, wall_s = 0;
};
// this rank's partition (the tuples keto_object_owner -- or the job's placement -- gives it) as a
// resident snapshot whose node arithmetic, relation flags and uuid ids agree with every other
// rank's (collective)
DistEngine *dist_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, bool device_ptrs,
                        const keto_collective &coll, const keto_limits &limits, const Placement &place);
// collective: this rank's n queries (host) -> decisions (host); `routed` = the queries the
// caller's exact path must answer (their outputs here are placeholders)
void dist_check(DistEngine &E, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, bool err_detail,
                std::vector<uint32_t> &routed, DistStats &st);
void dist_free(DistEngine *E);
const Snapshot &dist_snapshot(const DistEngine &E);
// the last batch per generation: goals here, goal-record bytes sent / records received, decision
// bytes returned, device ms
std::vector<keto_partition_level> dist_levels(const DistEngine &E);

// what expand_dist.hip needs of the engine: its rank, collective, stream, snapshot, limits
struct DistView {
    int device;
    uint32_t rank, world;
    const keto_collective *coll;
    hipStream_t hs;
    const Snapshot *snap;
    keto_limits limits;
    Placement place;
};
DistView dist_view(DistEngine &E);
// the collective (all ranks call in the same order): one u64 per rank; all-to-all-v of device
// bytes on the engine's stream (host-staged when the collective takes no device buffers); wait_s
// accumulates the time spent inside the collective
std::vector<uint64_t> dist_alltoall(const DistView &V, const std::vector<uint64_t> &send, double &wait_s);
void dist_alltoallv(const DistView &V, const void *src, const std::vector<uint64_t> &sb, void *dst,
                    const std::vector<uint64_t> &rb, double &wait_s);

// collective: Expand of this rank's n roots (host) over the resident partitions -- the rows the
// reference's DFS can read fetched level by level from their owners (no closure snapshot, no
// build), then one DFS per root on the device over the fetched rows.  Trees in root order into
// nodes / offsets[n+1] / err (as keto_expand_batch).
struct DistExpandStats {
    uint64_t levels = 0, rows = 0, entries = 0, bytes_sent = 0;
    double fetch_s = 0, walk_s = 0, exchange_s = 0;
    std::vector<keto_partition_level> per_level;
};
void dist_expand(DistEngine &E, const keto_subject_set *roots, uint64_t n, std::vector<keto_tree_node> &nodes,
                 std::vector<uint64_t> &offsets, std::vector<int32_t> &err, DistExpandStats &st);

}  // namespace keto
