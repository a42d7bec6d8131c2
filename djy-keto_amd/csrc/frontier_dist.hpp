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
// this rank's partition (the tuples keto_object_owner gives it) as a resident snapshot whose node
// arithmetic, relation flags and uuid ids agree with every other rank's (collective)
DistEngine *dist_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, bool device_ptrs,
                        const keto_collective &coll, const keto_limits &limits);
// collective: this rank's n queries (host) -> decisions (host); `routed` = the queries the
// caller's exact path must answer (their outputs here are placeholders)
void dist_check(DistEngine &E, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, bool err_detail,
                std::vector<uint32_t> &routed, DistStats &st);
void dist_free(DistEngine *E);
const Snapshot &dist_snapshot(const DistEngine &E);
// the last batch per generation: goals here, goal-record bytes sent / records received, decision
// bytes returned, device ms
std::vector<keto_partition_level> dist_levels(const DistEngine &E);

}  // namespace keto
