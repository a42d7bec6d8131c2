// Internal host-side types of libketo_mi355x (behind the C ABI in include/keto_mi355x.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/keto_mi355x.h"
#include "layout.hpp"

namespace keto {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define KETO_HIP(expr)                                                                              \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            throw ::keto::Error(KETO_E_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
    } while (0)

// Room a store snapshot keeps for objects created after it (keto_store_snapshot_patch): spare
// entities in every namespace, between its real entities and its phantom, handed out once across
// every snapshot patched from it (the family shares this record: no spare is given twice)
struct Spares {
    std::mutex mu;
    std::vector<uint32_t> first, count, used;  // per namespace
};
struct BuildOpts {
    uint32_t uuid_capacity = 0;  // id space (>= cfg n_uuids): ids past the caller's are unknown until written
    bool spares = false;         // spare entities per namespace (n_real / 16 + 256)
    bool room = false;           // in-place advance room (Snapshot::Room): row slack, relocation table, shard keys
    // A partitioned graph's snapshots (frontier_dist.hip) share one node arithmetic: the (ns, rel)
    // pairs the job's tuples use are agreed on (OR over the ranks) before slots are laid out
    std::function<void(std::vector<uint8_t> &used)> agree_used;
    bool no_leaf = false;     // no EDGE_LEAF marks (the bit is such a snapshot's EDGE_REMOTE)
    bool no_weights = false;  // no scheduling-weight array at all (DevSnapshot::weight null)
    // rank `part_rank` of a job of part_world > 1 ranks: subject-set objects another rank owns
    // (keto_object_owner) are entities of ghost namespaces -- every row array stops at them
    uint32_t part_rank = 0, part_world = 1;
    Placement place{};  // (which objects are this rank's: keto_placement; zeros: the hash)
};

// Host mirror of the snapshot + its device buffers.
struct Snapshot {
    int device = 0;
    uint32_t n_ns = 0, n_rel = 0, n_rel_caller = 0, n_uuids = 0;
    bool strict = false;
    std::vector<std::string> ns_names, rel_names;
    std::vector<NsDev> ns;          // [n_ns+1]
    std::vector<uint32_t> ent_obj;  // entity -> uuid id (NONE32 for phantoms)
    std::vector<uint32_t> slot_rel; // global slot -> relname
    std::vector<uint32_t> relinfo, nsrel;
    std::vector<Op> ops;
    std::vector<uint32_t> op_children;
    std::vector<uint32_t> op_items;  // flattened OR rewrites (layout.hpp IT_*)
    std::vector<uint2> or_items;
    DevSnapshot dev{};
    std::vector<void *> allocs;
    std::vector<size_t> alloc_bytes;  // (parallel to allocs: what keto_snapshot_save writes)
    std::vector<std::shared_ptr<void>> owned;  // (parallel to allocs: a patched snapshot shares its base's unchanged arrays)
    keto_snapshot_info info{};
    uint64_t store_id = 0;     // the keto_store it was cut from (0: built directly)
    uint64_t cfg_hash = 0;     // config_hash of the configuration it was compiled from (patches keep it)
    uint64_t probe_used = 0;   // probe-hash slots holding a key or a tombstone (patches keep the load bounded)
    std::shared_ptr<Spares> spares;  // (store snapshots: room for new objects)
    // reachability tables (reach.hip), host side: each global slot's first candidate (NONE32: not
    // tabled), the candidates and the pool entries in use -- what a patch's incremental rebuild
    // compares and extends (empty after keto_snapshot_load: a patch then rebuilds them whole)
    std::vector<uint32_t> reach_slots;
    uint64_t reach_cand = 0, reach_pool_n = 0;
    std::vector<uint4> ext;          // {obj, ns, entity, 0} of the objects placed on spares (dev.ext's entries)
    uint64_t reach_pool_cap = 0;     // reach_pool entries allocated (> reach_pool_n: room to append)
    uint64_t reach_pool_built = 0;   // reach_pool_n at the last full build (an advance declines past 2x + 1Mi)
    // in-place advance (advance in patch.hip; store snapshots only, BuildOpts::room): the row value
    // arrays' capacities and next free entries past the rows, the relocation table (dev.reloc), and
    // each all_subj entry's shard key -- the high 64 bits of its shard_id, the order of a row
    struct Room {
        uint64_t all_cap = 0, all_tail = 0, rev_cap = 0, rev_tail = 0, set_cap = 0, set_tail = 0;
        uint32_t reloc_cap = 0, reloc_used = 0;
        unsigned long long *all_shard = nullptr;
        bool moved = false;  // an advance ran: rows live outside their CSR extents (no save, no copy patch)
    } room;
    // (room snapshots) per global slot: subject-set edges into the slot's nodes (a reach "target"
    // slot when > 0) and the slot's nodes with a non-empty set row (RI_SETROWS when > 0) -- kept
    // by each advance from its own rows, where a scan of set_dst would read moved rows' old copies
    std::vector<uint64_t> slot_in, slot_rows;
    // an in-place advance failed after its first write (patch.hip advance_snapshot): rows may be
    // half-advanced, so the C ABI refuses every further use but keto_snapshot_free
    bool broken = false;

    // a device allocation of this snapshot (back to the pool with its last sharer)
    void own(void *p, size_t bytes);
    void *alloc(size_t bytes);  // own(pool_acquire(bytes))
    // the allocation of `o` holding p, shared (p must be one of o's arrays)
    void share(const Snapshot &o, const void *p);
    // this snapshot's own allocation p: no other snapshot shares it / let go of it (back to the
    // pool with its last sharer)
    bool sole(const void *p) const;
    void drop(const void *p);
    // node -> (ns, entity, slot) on the host (for Expand output conversion)
    uint32_t ns_of(uint32_t node) const;
};

Snapshot *build_snapshot(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, bool device_tuples,
                         bool sched_weights = true, const BuildOpts *opts = nullptr);
// reach.hip: the snapshot's reachability tables (s.dev.reach_*), or none
void build_reach(Snapshot &s);
// reach.hip: the tables of a patched snapshot s from its base's: only the tabled nodes whose
// reach can have changed -- the touched rows' nodes and their ancestors over subject-set rows
// within REACH_CAP - 1 hops -- are walked again; anything else (the tabled slots changed, the base
// has no host record) rebuilds them whole
// (&s == &B: an in-place advance -- the tables are updated where they lie)
void patch_reach(Snapshot &s, const Snapshot &B, const std::vector<uint32_t> &touched_nodes);
// patch.hip: Snapshot::slot_in / slot_rows of a room snapshot, counted over its rows (at its build)
void room_slot_counts(Snapshot &s);
// 64-bit FNV-1a of everything a snapshot compiles from its configuration (name tables, AST JSON,
// strict mode; not the device, not n_uuids): equal hashes = the same compiled tables
uint64_t config_hash(const keto_snapshot_config *cfg);
// snapshot.cpp: a built snapshot to a file and back (keto_snapshot_save / _load)
void save_snapshot(const Snapshot &s, const char *path);
Snapshot *load_snapshot(const char *path, int device);

// build.hip: device-side snapshot construction (one-thread-per-item kernels)
namespace build {
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    size_t cap = 0;  // the block's size (scratch_get may hand out a larger cached block)
    DevBuf() = default;
    explicit DevBuf(size_t b);  // hipMalloc(b + 16): 16-byte window loads past the end stay in bounds
    ~DevBuf();
    DevBuf(DevBuf &&o) noexcept;
    DevBuf &operator=(DevBuf &&o) noexcept;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    void reset();
    void *release();
    uint32_t *u32() const { return static_cast<uint32_t *>(p); }
};
// v[0..n) -> exclusive prefix sums, v[n] = total, on stream s (temporaries fenced by the calling
// thread's ScratchStream)
void scan_excl(uint32_t *v, uint64_t n, hipStream_t s = nullptr);
uint32_t read_u32(const uint32_t *d, uint64_t i);
void validate(const keto_tuple *t, uint64_t n, uint32_t n_ns, uint32_t n_rel_caller, uint32_t n_uuids, uint32_t n_rel,
              uint32_t *used, unsigned long long *bad);
void entity_bits(const keto_tuple *t, uint64_t n, uint64_t stride, unsigned long long *bits, uint64_t nblk,
                 uint32_t *rank, uint32_t n_ns = 0, uint32_t part_rank = 0, uint32_t part_world = 1,
                 const Placement &place = Placement{});
void entity_ids(const unsigned long long *bits, uint32_t *rank, uint64_t nblk, uint64_t bpn, uint64_t stride,
                const uint32_t *ent_base, const uint32_t *rank0, uint32_t *ent_obj, uint4 *table);
struct RowsIn {
    const keto_tuple *tuples;       // device copy
    const keto_tuple *host_tuples;  // caller's host array, or null (very long rows are sorted on the host)
    uint64_t n, n_nodes, n_subj;
    const unsigned long long *bits;
    const uint32_t *rank;
    const NsDev *ns;
    const uint32_t *slot_of;
    uint64_t stride;
    uint32_t n_rel, n_uuids;
    bool weights = true;            // scheduling weights (false: all 1, e.g. per-batch closure snapshots)
    uint32_t n_ns = 0, part_rank = 0, part_world = 1;  // (ghost namespaces: BuildOpts::part_world > 1)
    Placement place{};
};
struct RowsOut {
    uint32_t *all_off, *rev_off, *all_subj, *rev_nodes, *weight;  // caller-allocated
    uint4 *set_row;
    unsigned long long *all_shard = nullptr;  // caller-allocated or null: shard_hi of each all_subj entry
    uint64_t set_slack = 0;                   // set_dst entries allocated past the rows
    DevBuf set_dst, probe;
    uint64_t n_set = 0, probe_buckets = 0, probe_keys = 0;
};
void rows(const RowsIn &in, RowsOut &out);
void alias_mark(uint32_t *set_dst, uint64_t n, const uint32_t *vkey, uint4 *set_row, uint64_t n_rows);
void leaf_mark(uint32_t *set_dst, uint64_t n, uint4 *set_row, uint64_t n_rows);
// EDGE_REMOTE on every edge into a ghost node (>= n_owned: an object another rank owns); the
// inline copies in set_row follow
void remote_mark(uint32_t *set_dst, uint64_t n, uint4 *set_row, uint64_t n_rows, uint32_t n_owned);
// flag[global slot] |= 1 where a row of the slot holds a subject set (flag zeroed by the caller)
void slot_setrows(const uint4 *set_row, uint64_t n_rows, const NsDev *ns, uint32_t n_ns, uint32_t *flag, uint32_t n_slots);
void slot_idrows(const keto_tuple *t, uint64_t n, const uint32_t *slot_of, uint32_t n_rel, const NsDev *ns, uint32_t *flag,
                 uint32_t n_slots);
}  // namespace build

// scratch tier: per-lane visited capacity (slots, pow2) and stack frames
struct Tier {
    uint32_t lanes, vcap, scap;
};

// per-stream device scratch for one kernel family: disjoint per-tier regions so an
// epoch-tagged visited slot can only ever be read back by the lane that wrote it
struct Scratch {
    void *mem = nullptr;
    size_t bytes = 0;
    Tier t[3]{};
    uint32_t *ctrl = nullptr;
    uint32_t *epochs[3]{};
    unsigned long long *vis[3]{};
    uint4 *stack[3]{};
};

// per-stream arena of the frontier engine (frontier.hip)
struct FrontierScratch {
    void *mem = nullptr;
    uint64_t cap = 0, ncap = 0, dcap = 0, ocap = 0;  // goals, queries, decisive-key slots, occurrences per slice
    uint32_t *ctrl = nullptr;              // [gbase | gcount | fallback count]
    uint32_t *qrouted = nullptr, *fb_list = nullptr, *fb_count = nullptr;  // qrouted: a bit per query
    uint32_t *qspawn = nullptr;  // per query: goals spawned from generation KETO_FR_CAP_GEN on
    uint4 *g0 = nullptr;
    uint2 *gfn = nullptr;
    uint2 *gvs = nullptr;  // {value, goals below} per goal
    unsigned long long *dkeys = nullptr;
    uint32_t *dcnt = nullptr, *occ_count = nullptr, *dbits = nullptr;
    uint2 *occ = nullptr;
    uint32_t *host_ctrl = nullptr;  // pinned
    uint32_t last_gens = 0, last_goals = 0, last_routed = 0;
    // asynchronous passes: each one's generation count goes to pinned host memory at its end
    // (fr_gens_used + a 4-byte copy), and a later pass adopts it as its speculation depth once the
    // copy has landed -- a stream that only ever runs asynchronous batches learns its depth too
    uint32_t *host_gens = nullptr;  // pinned
    hipEvent_t gens_ev = nullptr;
    bool gens_pending = false;
    uint32_t epoch = 1;  // scope-table epoch of the next batch (frontier.hip TAB_EPOCHS)
    keto_frontier_stats stats{};
    // phase A's children of rewrite / tuple-to-userset goals, kept for the write-out (frontier_goal.inc
    // Stash): FR_STASH_K entries of 8 B per resident lane, a column per lane
    uint2 *stash = nullptr;
    uint32_t stash_stride = 0;
};

// per-stream workspace of the block frontier engine (frontier_block.hip)
struct FrontierBlockScratch {
    void *mem = nullptr, *gpool = nullptr, *opool = nullptr;
    uint32_t *ctrl = nullptr, *host = nullptr;  // host: pinned read-back of ctrl
    uint32_t gpool_cap = 0, opool_cap = 0;
    uint32_t *fb_list = nullptr, *fb_count = nullptr;
    uint64_t fb_cap = 0;
};

struct Stream {
    int device = 0;
    hipStream_t stream = nullptr;
    // main-kernel timing: HIP event pairs recorded around every batch's tier-0 launch on this
    // stream, harvested after synchronisation (a ring, so async batches can queue up)
    static constexpr int TIMER_SLOTS = 64;
    hipEvent_t ev_a[TIMER_SLOTS] = {}, ev_b[TIMER_SLOTS] = {};
    uint64_t timer_issued = 0, timer_harvested = 0, timer_count = 0;
    double timer_ms_sum = 0;
    void mark_begin();  // before the main kernel (stream-ordered)
    void mark_end();    // after it
    void harvest();     // accumulate every completed pair (call after a stream sync)
    // device workspace (allocated on first use, never inside a launch sequence)
    Scratch check_scratch, expand_scratch;
    // expand_wave workspace (expand.hip): per-wave staging, the batch's stage, per-root arrays
    struct {
        void *mem = nullptr, *roots_mem = nullptr;
        uint64_t grid = 0, stage_cap = 0, ncap = 0;
        uint2 *priv = nullptr, *stage = nullptr;  // walk records {subject key, n_children | union} (expand.hip)
        keto_tree_node *outbuf = nullptr;
        uint64_t out_cap = 0;
        uint64_t span_hint = 0;  // keto_expand_batch_spans into pageable memory: the device buffer it wants
        unsigned long long *sizes = nullptr, *soff = nullptr, *ctrl = nullptr;
        uint64_t *offsets = nullptr;
        int32_t *err = nullptr;
        uint32_t *fb_list = nullptr;
        uint32_t *order = nullptr;  // the wave kernel's queue: heavy roots first (expand_order)
        hipEvent_t ev[2] = {nullptr, nullptr};  // around the traversal (expand_wave + the fallback's count pass)
        void *hpin = nullptr;                   // pinned read-back of the offsets, errors and stage top
        size_t hpin_bytes = 0;
        double ms_sum = 0;
        uint64_t batches = 0;
    } xw;
    FrontierScratch frontier;
    FrontierBlockScratch frontier_block;
    // per-batch workspace of list_cap queries, one allocation:
    uint32_t *lists = nullptr;       // two overflow hand-off lists (of start-record positions)
    uint4 *resolved = nullptr;       // 2 x 16 B start record per query, longest-first (resolve.hip)
    uint32_t *order_ctrl = nullptr;  // [0] heavy, [1] light counts
    uint64_t list_cap = 0;
    void *qbuf = nullptr, *obuf = nullptr;  // staging for host-pointer batches
    size_t qbuf_bytes = 0, obuf_bytes = 0;
    // KETO_F_ASYNC host-pointer batches: their copies run on two copy streams beside the compute
    // stream, through two staging slots, so batch k+1's H2D and batch k-1's D2H overlap batch k's
    // kernels (events order each slot's H2D -> kernels -> D2H -> next H2D)
    hipStream_t h2d = nullptr, d2h = nullptr;
    struct Slot {
        void *q = nullptr, *o = nullptr;
        size_t qb = 0, ob = 0;
        hipEvent_t in = nullptr, out = nullptr, free = nullptr;
    } slot[2];
    uint64_t slot_seq = 0;
    // One copy stream (default; KETO_COPY_STREAMS=2: the two above): batch k's D2H is enqueued
    // behind batch k+1's H2D -- or by keto_stream_sync -- on the h2d stream, so the two directions
    // never run at once.  Concurrent H2D + D2H moved 17 GB/s together on the box, against 54-55 GB/s
    // for either alone (tools/pcie_probe.py, round 6).
    bool one_copy = true;
    struct PendingD2H {
        bool on = false;
        uint8_t *allowed = nullptr;
        int32_t *err = nullptr;
        const void *src = nullptr;  // the slot's outputs: n decisions, then (64-aligned) n errors
        uint64_t n = 0;
        uint32_t slot = 0;
    } pend;
    void flush_d2h();  // (capi.cpp) enqueue the pending D2H, if any
    unsigned long long *counters = nullptr;  // device [3 tiers][8]
    keto_work_counters host_counters{};
    double last_kernel_ms = 0;
    uint32_t fr_budget = 1024;  // KETO_FR_BUDGET, read once when the stream is created (tests lower it)
    ~Stream();
};

// scratch.cpp
int num_cus(int device);
// snapshot arrays: a block of >= bytes from the device's pool of released arrays, else hipMalloc
// (*got: the block's size); release returns it (after a device sync) or frees it; reserve makes
// sure a free block of each size exists (allocated and touched now)
void *pool_acquire(int device, size_t bytes, size_t *got);
void pool_release(int device, void *p, size_t bytes);
void pool_reserve(int device, const std::vector<size_t> &sizes);
void pool_trim(int device);
void pool_shutdown();  // keto_shutdown: every device's pool and scratch cache back to the runtime
// builder temporaries (DevBuf): a per-device cache of freed blocks (scratch.cpp).  A block
// returned by a thread is fenced by an event on that thread's stream (scratch_stream sets it;
// returns the previous one), which its next user waits for.
void *scratch_get(size_t bytes, size_t *got);
void scratch_put(void *p, size_t bytes);
hipStream_t scratch_stream(hipStream_t s);
void scratch_forget_stream(hipStream_t s);  // call before destroying a stream scratch_stream named
struct ScratchStream {  // the calling thread's DevBufs live on stream s for this scope
    hipStream_t old;
    explicit ScratchStream(hipStream_t s) : old(scratch_stream(s)) {}
    ~ScratchStream() { scratch_stream(old); }
};  // every pooled block freed (any allocation that runs out of memory calls it)
void ensure_scratch(Scratch &sc, const Tier t[3]);
void ensure_lists(Stream &st, uint64_t n);

// check.hip / expand.hip
struct CheckLaunch {
    const void *queries;  // keto_query records, or keto_query16 (q16)
    bool q16 = false;
    uint64_t n;
    uint8_t *out_allowed;
    int32_t *out_err;
    int32_t max_depth, max_width;
    bool count;
    bool err_detail;  // KETO_F_ERR_DETAIL: out_err carries the failing relation name id << 8
    uint32_t budget;  // frontier goals per query before it is routed to the DFS interpreter (Stream::fr_budget)
    bool async;       // KETO_F_ASYNC: enqueue only, no host read-back inside the batch
};
// resolve.hip: per-query start records, longest-first, into st.resolved
// ordered: heavy-first work order for the DFS interpreters (two atomics per wave); else batch order
void run_resolve(const Snapshot &s, Stream &st, const void *queries, bool q16, uint64_t n, int32_t max_depth,
                 bool ordered = true);
void run_check(const Snapshot &s, Stream &st, const CheckLaunch &L);        // rewrite interpreter
uint2 *frontier_stash(Stream &st, uint32_t cus);  // frontier.hip: the frontier engines' phase-A stash
// frontier.hip: L.n resolved queries from batch position pos_base on, breadth-first; returns the
// number of queries routed to the DFS interpreter (batch positions in st.frontier.fb_list).
// Batches above FR_MAX_BATCH run as several passes: the arena's goal indices stay in range.
constexpr uint64_t FR_MAX_BATCH = 1ull << 21;
constexpr uint32_t FR_ROUTED_ON_DEVICE = 0xFFFFFFFFu;  // run_frontier, asynchronous: the count stays on the device
uint32_t run_frontier(const Snapshot &s, Stream &st, const CheckLaunch &L, uint64_t pos_base);
// frontier_block.hip: the same evaluation with a workgroup per chunk of queries (the default
// engine); routed batch positions in st.frontier_block.fb_list
uint32_t run_frontier_block(const Snapshot &s, Stream &st, const CheckLaunch &L, uint64_t pos_base);

struct ExpandLaunch {
    const keto_subject_set *roots;  // device
    uint64_t n;
    int32_t max_depth;
    uint64_t *sizes;    // device [n] (count pass output)
    const uint64_t *offsets; // device [n] (emit pass input)
    keto_tree_node *out;  // device nodes in API form (emit pass)
    int32_t *err;       // device [n]
    bool emit;
    const uint32_t *list = nullptr, *list_count = nullptr;  // only these roots (device list + count; nl roots at most)
    uint64_t nl = 0;
};
// the lane-per-root two-pass kernel (expand_kernel): expand_batch's fallback
void run_expand(const Snapshot &s, Stream &st, const ExpandLaunch &L);
// keto_expand_batch's device path (expand_wave, fallback expand_kernel): the trees of the n
// device roots into out_nodes (host, root order) with out_offsets / out_err; false (and the
// offsets filled) when out_cap is too small
bool expand_batch(const Snapshot &s, Stream &st, const keto_subject_set *d_roots, uint64_t n, int32_t max_depth,
                  keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_offsets, int32_t *out_err);

// keto_expand_batch_spans' device path: root i's tree at out_nodes[out_first[i]], out_count[i]
// nodes, written as the walks finish; false (*out_total = the nodes required) when out_cap is too small
bool expand_batch_spans(const Snapshot &s, Stream &st, const keto_subject_set *d_roots, uint64_t n, int32_t max_depth,
                        keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_first, uint32_t *out_count,
                        int32_t *out_err, uint64_t *out_total);

// treefmt.cpp: Expand trees -> API form (Mapper.ToTree + JSON / Tree.ToProto), host only
void trees_to_json(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                   const keto_name_tables *names, char *out, uint64_t cap, uint64_t *out_offsets);
void trees_to_proto(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                    const keto_name_tables *names, uint8_t *out, uint64_t cap, uint64_t *out_offsets);

// dispatcher.cpp: request coalescing (keto_dispatcher_*)
void dispatcher_create(keto_snapshot *snap, const keto_dispatcher_config *cfg, keto_dispatcher **out);
void dispatcher_destroy(keto_dispatcher *d);
int dispatcher_check(keto_dispatcher *d, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err,
                     std::string &msg);
void dispatcher_set_snapshot(keto_dispatcher *d, keto_snapshot *snap);
int dispatcher_expand(keto_dispatcher *d, const keto_subject_set *roots, uint64_t n, keto_tree_node *nodes, uint64_t cap,
                      uint64_t *offsets, int32_t *err, std::string &msg);
void dispatcher_stats(keto_dispatcher *d, keto_dispatcher_stats *out);

// store.hip: device tuple store with TransactRelationTuples deltas (keto_store_*)
struct TupleStore;
TupleStore *store_create(int device, const keto_tuple *tuples, uint64_t n, bool device_ptrs);
void store_transact(TupleStore &st, const keto_tuple *ins, uint64_t n_ins, const keto_tuple *del, uint64_t n_del,
                    bool device_ptrs);
Snapshot *store_snapshot(const TupleStore &st, const keto_snapshot_config *cfg);
// the store's current content by patching `base` (cut from this store earlier); *patched = false
// when the full device build ran instead
Snapshot *store_snapshot_patch(const TupleStore &st, const Snapshot &base, const keto_snapshot_config *cfg, bool *patched);
// patch.hip: base + the rows the touched tuples name, rebuilt from the store's content (nullptr:
// base has no node for some touched tuple, or its probe hash is too full -- build in full)
Snapshot *patch_snapshot(const Snapshot &base, const keto_tuple *store_rows, uint64_t n_store, const keto_tuple *touched,
                         const uint8_t *touched_is_ins, uint64_t n_touched);
// the store's current content in `snap` itself (cut from this store, no batch in flight on it):
// false when the delta needs a full build -- snap is then unchanged
bool store_snapshot_advance(const TupleStore &st, Snapshot &snap);
// patch.hip: snap + the touched tuples applied to its rows where they lie (false: nothing changed)
bool advance_snapshot(Snapshot &snap, const keto_tuple *touched, const uint8_t *touched_is_ins, uint64_t n_touched,
                      uint64_t n_store);
void store_free(TupleStore *st);
void store_info(const TupleStore &st, uint64_t *n, uint64_t *version);

// devprim.hip: stream-ordered primitives of the partition path (hand-written gfx950 kernels)
namespace prim {
// stable LSD radix sort of n pairs on the low `bits` bits of the keys, ping-ponging between
// (k0, v0) and (k1, v1); true when the result ends in (k1, v1)
bool sort_pairs(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t bits, hipStream_t s);
bool sort_pairs(uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, uint32_t bits, hipStream_t s);
// the distinct values of sorted a[0..n) into out; returns their count (synchronises s)
uint64_t unique_sorted(const uint32_t *a, uint64_t n, uint32_t *out, hipStream_t s);
// flag[i] = a[i] != a[i-1] (flag[0] = 1), flag[n] = 0: n + 1 slots, ready for build::scan_excl
void run_flags(const uint64_t *a, uint64_t n, uint32_t *flag, hipStream_t s);
void run_flags(const uint32_t *a, uint64_t n, uint32_t *flag, hipStream_t s);
void sum_u32(const uint32_t *v, uint64_t n, unsigned long long *out, hipStream_t s);  // *out = sum (device)
}  // namespace prim

// partition.hip: graphs partitioned by object over the ranks of a job (keto_partition_*)
struct PartitionHandle;
PartitionHandle *partition_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n,
                                  bool device_ptrs, const keto_collective *coll, const keto_limits *limits,
                                  bool force_dist = false, const Placement &place = Placement{});
void partition_check(PartitionHandle *p, const keto_query *q, uint64_t n, uint8_t *allowed, int32_t *err, uint32_t flags);
void partition_check_many(PartitionHandle *p, uint32_t nb, const keto_query *const *q, const uint64_t *n,
                          uint8_t *const *allowed, int32_t *const *err, uint32_t flags);
uint64_t partition_expand(PartitionHandle *p, const keto_subject_set *roots, uint64_t n);
void partition_expand_result(PartitionHandle *p, keto_tree_node *nodes, uint64_t cap, uint64_t *offsets, int32_t *err);
void partition_stats(PartitionHandle *p, keto_partition_stats *out);
void partition_levels(PartitionHandle *p, keto_partition_level *out, uint32_t cap, uint32_t *n);
void partition_generations(PartitionHandle *p, keto_partition_generation *out, uint32_t cap, uint32_t *n);
void partition_free(PartitionHandle *p);

}  // namespace keto
