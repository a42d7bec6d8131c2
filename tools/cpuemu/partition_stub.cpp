// TEST/DEBUG TOOL ONLY: keto_partition_* (csrc/partition.hip, csrc/devprim.hip) is not emulated -- its
// kernels are written for 256-thread blocks of 64-lane waves (ballot ranks, one digit per thread),
// which the one-lane emulation cannot run; its entry points fail loudly here.
#include "../../djy-keto_amd/csrc/engine.hpp"

namespace keto {
struct PartitionHandle {};
[[noreturn]] static void unavailable() { throw Error(KETO_E_DEVICE, "keto_partition_* is not part of the CPU emulation"); }
PartitionHandle *partition_create(const keto_snapshot_config *, const keto_tuple *, uint64_t, bool, const keto_collective *,
                                  const keto_limits *) { unavailable(); }
void partition_check(PartitionHandle *, const keto_query *, uint64_t, uint8_t *, int32_t *, uint32_t) { unavailable(); }
void partition_check_many(PartitionHandle *, uint32_t, const keto_query *const *, const uint64_t *, uint8_t *const *, int32_t *const *,
                          uint32_t) {
    unavailable();
}
uint64_t partition_expand(PartitionHandle *, const keto_subject_set *, uint64_t) { unavailable(); }
void partition_expand_result(PartitionHandle *, keto_tree_node *, uint64_t, uint64_t *, int32_t *) { unavailable(); }
void partition_stats(PartitionHandle *, keto_partition_stats *) { unavailable(); }
void partition_levels(PartitionHandle *, keto_partition_level *, uint32_t, uint32_t *) { unavailable(); }
void partition_free(PartitionHandle *) {}
}  // namespace keto
