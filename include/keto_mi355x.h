/*
 * keto_mi355x.h -- C ABI of the MI355X batched Check / Expand engine.
 *
 * This is the drop-in boundary for Keto's permission hot path.  It replaces
 * everything BELOW these reference entry points (paths relative to the
 * reference repository):
 *
 *   check.Engine.CheckIsMember / CheckRelationTuple   internal/check/engine.go:65-95
 *   expand.Engine.BuildTree                            internal/expand/engine.go:43-52
 *   relationtuple.Traverser / Manager read ops          internal/relationtuple/definitions.go:22-33
 *     (TraverseSubjectSetExpansion   persistence/sql/traverser.go:53-121,
 *      TraverseSubjectSetRewrite     persistence/sql/traverser.go:123-191,
 *      GetRelationTuples             persistence/sql/relationtuples.go:207-247,
 *      ExistsRelationTuples          persistence/sql/relationtuples.go:249-261)
 *
 * A Go cgo shim keeps the check.Engine / expand.Engine API
 * and does the Mapper work on the host (internal/relationtuple/uuid_mapping.go):
 * strings/UUIDs are interned to dense uint32 ids before they cross this ABI.
 *
 * Conventions: every entry point returns KETO_OK (0) or a negative KETO_E_*
 * status; keto_last_error() gives the message (thread-local).  Plain pointers
 * and sizes only.  The caller owns every buffer it passes; the library owns
 * device memory of snapshots and streams.  A snapshot is immutable after build
 * and may be shared by many streams/threads; a stream is used by one thread
 * at a time.
 */
#ifndef KETO_MI355X_H
#define KETO_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KETO_ABI_VERSION 7

/* status codes */
#define KETO_OK 0
#define KETO_E_INVALID (-1)   /* bad argument / malformed namespace JSON */
#define KETO_E_DEVICE (-2)    /* HIP runtime error */
#define KETO_E_CAPACITY (-3)  /* output buffer too small (required size reported) */
#define KETO_E_LIMIT (-4)     /* id space exceeds the snapshot format */

/* per-query error codes (out_err[i]); 0 = no error.
 * 1 -> herodot.ErrBadRequest "relation %q does not exist"
 *      (internal/namespace/definitions.go:61, surfaced by engine.go:228-232)
 * 2 -> internal: evaluation exceeded every scratch tier (only reachable with a
 *      cyclic zero-depth-cost rewrite, on which the reference never returns)
 * 3 -> "not implemented" rewrite operator (internal/check/rewrites.go:18-20) */
#define KETO_QERR_NONE 0
#define KETO_QERR_NO_RELATION 1
#define KETO_QERR_INTERNAL 2
#define KETO_QERR_NOT_IMPLEMENTED 3

/* Relation tuple as stored in keto_relation_tuples (schema:
 * persistence/sql/migrations/sql/20230228091200000000_add-on-delete-cascade-to-relationship.sqlite.up.sql:14-49).
 * ns/rel index the name tables of keto_snapshot_config; obj/s_obj are interned
 * UUIDs (< n_uuids).  subj_kind 0 = SubjectID(s_obj); 1 = SubjectSet(s_ns:s_obj#s_rel).
 * shard_id = the tuple's shard_id UUID bytes: it defines every iteration order
 * (ORDER BY shard_id, traverser.go:88 / relationtuples.go:216). */
typedef struct keto_tuple {
    uint32_t ns, obj, rel;
    uint32_t subj_kind;
    uint32_t s_obj, s_ns, s_rel;
    uint32_t reserved;
    uint8_t shard_id[16];
} keto_tuple;

/* One Check: ns:obj#rel@subject; max_depth = request max-depth
 * (<= 0 or > global -> global, engine.go:82-84). */
typedef struct keto_query {
    uint32_t ns, obj, rel;
    uint32_t subj_kind;
    uint32_t s_obj, s_ns, s_rel;
    int32_t max_depth;
} keto_query;

/* ABI 7: the same Check in 16 bytes (SURVEY 8.1 A1's request record), for keto_check_batch16:
 * half the H2D bytes of a host batch.  Holds namespace ids < 4096, relation ids < 1024 and request
 * depths in [-32768, 32767] (keto_pack_query16 refuses anything else); the decisions are
 * keto_check_batch's on the unpacked request.
 *   word 0: obj                 word 1: s_obj (the subject id, or the subject set's object)
 *   word 2: ns | rel << 12 | s_rel << 22
 *   word 3: s_ns | subj_kind << 12 | (uint16_t)max_depth << 16 */
typedef struct keto_query16 {
    uint32_t obj, s_obj, ns_rel, s_ns_depth;
} keto_query16;

/* Expand root: a subject set ns:obj#rel (a SubjectID root is answered by the
 * shim itself as a leaf, expand/handler.go:119-126 / expand/engine.go:60-67). */
typedef struct keto_subject_set {
    uint32_t ns, obj, rel;
    int32_t max_depth;
} keto_subject_set;

/* Expand output, pre-order.  type: 1 = union, 4 = leaf (ketoapi/enc_proto.go:164-176
 * numbering).  Each node's tuple carries only its subject (uuid_mapping.go:356-385). */
typedef struct keto_tree_node {
    uint32_t type;
    uint32_t subj_kind;
    uint32_t s_obj, s_ns, s_rel;
    uint32_t n_children;
} keto_tree_node;

typedef struct keto_snapshot_config {
    uint32_t n_namespaces;
    const char *const *namespace_names; /* id -> name */
    uint32_t n_relations;
    const char *const *relation_names;  /* id -> name ("" allowed) */
    uint32_t n_uuids;                   /* every obj / s_obj is < n_uuids */
    /* Namespace configuration as AST JSON, the format of
     * internal/schema/.snapshots/TestParser-*.json: {"Ns": [relation, ...]} with
     * relation = {"name", "types": [{"namespace", "relation"?}], "rewrite"?}.
     * A namespace mapped to [] is a legacy namespace without relation config. */
    const char *namespaces_json;
    int32_t strict_mode;                /* namespaces.experimental_strict_mode */
    int32_t device;                     /* HIP device ordinal */
} keto_snapshot_config;

typedef struct keto_snapshot_info {
    uint64_t n_tuples, n_nodes, n_entities, n_set_edges, n_rev_entries;
    uint64_t device_bytes;
    double build_seconds;
    uint64_t version; /* keto_store version it was cut from (the snaptoken); 0 if built directly */
    uint64_t n_reach; /* nodes with a reachability table (the frontier's spawn-time NotMember) */
} keto_snapshot_info;

/* limit.max_read_depth / limit.max_read_width (internal/driver/config/provider.go:180-185) */
typedef struct keto_limits {
    int32_t max_read_depth; /* default 5 */
    int32_t max_read_width; /* default 100 */
} keto_limits;

/* Algorithmic work counters (BASELINE.md byte model), per scratch tier t = 0..2:
 * rows opened, subject-set edges read, membership probes, Expand nodes emitted and
 * queries completed by the kernels of tier t; plus the Check interpreters' load-slot
 * iterations summed over wavefronts (wave_steps) and over lanes holding a live query
 * (lane_steps): lane_steps / (64 * wave_steps) is the SIMD-lane utilisation. */
typedef struct keto_work_counters {
    uint64_t rows[3], edges[3], probes[3], out_nodes[3], queries[3];
    uint64_t wave_steps[3], lane_steps[3];
} keto_work_counters;

typedef struct keto_snapshot keto_snapshot;
typedef struct keto_stream keto_stream;

/* flags for keto_check_batch / keto_expand_batch */
#define KETO_F_DEVICE_PTRS 0x1u  /* query / output pointers are device memory */
/* KETO_F_ASYNC: enqueue only, no host synchronisation inside the call; pair with
 * keto_stream_sync before reading the outputs.  With host buffers the copies in and out are
 * enqueued on the stream too (pinned memory, keto_host_alloc, makes them truly asynchronous);
 * the buffers must stay valid until the stream is synchronised.  (A host-buffer batch's copy
 * out is enqueued behind the next batch's copy in, or by keto_stream_sync: synchronise before
 * destroying the stream.)  The frontier engine launches
 * the generations the stream's last synchronous batch needed plus a margin; a query deeper than
 * that is answered by the DFS interpreter (same answers).  keto_frontier_stats counts these
 * batches in async_batches only. */
#define KETO_F_ASYNC 0x2u
#define KETO_F_COUNT_WORK 0x4u   /* accumulate keto_work_counters on the stream */
/* keto_check_batch: for KETO_QERR_NO_RELATION, out_err[i] = 1 | (relation name id << 8), the
 * relation ASTRelationFor rejected -- not always the query's own (a subject set deeper in the
 * walk can name it) -- so the shim can return the reference's exact
 * `relation %q does not exist` (internal/namespace/definitions.go:61).  Without the flag
 * out_err[i] is the bare code. */
#define KETO_F_ERR_DETAIL 0x8u
/* keto_partition_create (ABI 7): run the distributed frontier even for a job of one rank -- every
 * goal record, subject table and decision goes to the rank itself through the collective's
 * exchanges (alltoallv_device included) instead of the resident-snapshot shortcut.  For a host
 * that wants to check its collective (an RCCL communicator) on one GPU before it scales out. */
#define KETO_F_PART_DIST 0x10u

int keto_abi_version(void);
/* copies the thread's last error message; returns its full length */
size_t keto_last_error(char *buf, size_t len);
/* Returns every device block and event the library caches between calls (its snapshot-array
 * pool and builder scratch cache, on every device it used) to the HIP runtime.  Call it at
 * process exit after freeing the library's objects, before the runtime's own teardown (a Go
 * host: after the last keto_*_free, e.g. from the server's shutdown hook; the Python mirror
 * registers it with atexit).  The library stays usable afterwards: the caches refill on
 * demand.  No reference counterpart. */
int keto_shutdown(void);

int keto_snapshot_build(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n_tuples,
                        keto_snapshot **out);
/* Same, from tuples already resident in device memory of cfg->device (for example a
 * replica broadcast over RCCL/xGMI from the rank that read the store); the caller
 * keeps them alive for the duration of the call only. */
int keto_snapshot_build_device(const keto_snapshot_config *cfg, const keto_tuple *device_tuples, uint64_t n_tuples,
                               keto_snapshot **out);
/* A built snapshot to a file and back: the restart artefact (checkpoint).
 * The reference's state is its SQL database (internal/driver/registry_default.go:247-292) and a
 * restart re-reads it; here a restart can load the snapshot of the last snaptoken instead of
 * rebuilding it.  The file holds the compiled namespace tables and every device array of this
 * library's layout (its ABI version is checked on load); load onto any device.  The store
 * version (info.version) travels with it; build_seconds of a loaded snapshot = the load time. */
int keto_snapshot_save(const keto_snapshot *snap, const char *path);
int keto_snapshot_load(const char *path, int32_t device, keto_snapshot **out);
int keto_snapshot_free(keto_snapshot *snap);
int keto_snapshot_info_get(const keto_snapshot *snap, keto_snapshot_info *out);

int keto_stream_create(int32_t device, keto_stream **out);
int keto_stream_destroy(keto_stream *s);
int keto_stream_sync(keto_stream *s);
int keto_stream_counters(keto_stream *s, keto_work_counters *out, int32_t reset);
/* average device time (ms) of the last batch's main check kernel, measured with
 * HIP events on the stream the kernel ran on */
int keto_stream_last_kernel_ms(keto_stream *s, double *ms);
/* Frontier-engine activity on the stream (check batches of rewrite snapshots): batches, the
 * queries they held, the queries routed to the DFS interpreter (a repeated visited key with a
 * decisive occurrence, the goal budget, the generation cap or the arena), goals spawned and
 * generations run (sum and max).  reset != 0 zeroes them afterwards. */
typedef struct keto_frontier_stats {
    uint64_t batches, queries, routed, goals, generations, max_generations;  /* synchronous batches */
    uint64_t async_batches;  /* KETO_F_ASYNC batches (their counts stay on the device) */
} keto_frontier_stats;
int keto_stream_frontier_stats(keto_stream *s, keto_frontier_stats *out, int32_t reset);
/* Synchronises the stream, then reports the summed device time (ms) and count of the main
 * check kernel launches timed on it (HIP events around every batch's launch, async batches
 * included); reset != 0 zeroes the sums afterwards. */
int keto_stream_kernel_time(keto_stream *s, double *ms_sum, uint64_t *launches, int32_t reset);

/* Device time (ms, HIP events on the stream) of the Expand traversals since the last reset:
 * the wave-per-root kernel plus, for roots it hands on, the fallback's count pass -- not the
 * copies placing the trees in root order. */
int keto_stream_expand_time(keto_stream *s, double *ms_sum, uint64_t *batches, int32_t reset);

/* Check n queries: out_allowed[i] = CheckIsMember's bool, out_err[i] = error code.
 * Replaces check.Engine.CheckIsMember (engine.go:65-71) for a whole batch. */
int keto_check_batch(keto_snapshot *snap, keto_stream *s, const keto_query *queries, uint64_t n,
                     const keto_limits *limits, uint8_t *out_allowed, int32_t *out_err, uint32_t flags);
/* ABI 7: keto_check_batch over 16-byte records (same flags, outputs and errors). */
int keto_check_batch16(keto_snapshot *snap, keto_stream *stream, const keto_query16 *queries, uint64_t n,
                       const keto_limits *limits, uint8_t *out_allowed, int32_t *out_err, uint32_t flags);
/* n keto_query records -> keto_query16 (host); KETO_E_LIMIT when one does not fit the 16-byte form */
int keto_pack_query16(const keto_query *in, uint64_t n, keto_query16 *out);

/* Expand n roots into one pre-order node buffer; out_offsets[i]..out_offsets[i+1]
 * delimit root i's tree (empty range = nil tree, expand/handler.go:141-143).
 * If out_cap is too small returns KETO_E_CAPACITY with out_offsets[n] = required.
 * Replaces expand.Engine.BuildTree (expand/engine.go:43-124). */
int keto_expand_batch(keto_snapshot *snap, keto_stream *s, const keto_subject_set *roots, uint64_t n,
                      const keto_limits *limits, keto_tree_node *out_nodes, uint64_t out_cap,
                      uint64_t *out_offsets, int32_t *out_err);
/* ABI 7: keto_expand_batch with the trees in completion order instead of root order: root i's
 * tree is out_nodes[out_first[i] .. out_first[i] + out_count[i]) (count 0: nil tree, or out_err[i]
 * set), and *out_total = the nodes written.  Each tree is written the moment its walk ends -- into
 * out_nodes directly, over PCIe, when it is pinned (keto_host_alloc) -- so the copy-out overlaps
 * the other roots' walks.  If out_cap is too small returns KETO_E_CAPACITY with *out_total =
 * required (nothing of the batch is usable then).  Same trees as keto_expand_batch. */
int keto_expand_batch_spans(keto_snapshot *snap, keto_stream *s, const keto_subject_set *roots, uint64_t n,
                            const keto_limits *limits, keto_tree_node *out_nodes, uint64_t out_cap,
                            uint64_t *out_first, uint32_t *out_count, int32_t *out_err, uint64_t *out_total);

/* Incremental snapshots: a device-resident tuple store of one network that applies
 * TransactRelationTuples deltas (persistence/sql/relationtuples.go:277-287: insert every row
 * of ins -- the caller supplies their fresh shard_ids --, then delete every row matching a
 * row of del on (namespace, object, relation, subject), :168-189) and cuts snapshots of its
 * current content, stamped with its version.  flags: KETO_F_DEVICE_PTRS for device inputs. */
typedef struct keto_store keto_store;
int keto_store_create(int32_t device, const keto_tuple *tuples, uint64_t n, uint32_t flags, keto_store **out);
int keto_store_transact(keto_store *st, const keto_tuple *ins, uint64_t n_ins, const keto_tuple *del, uint64_t n_del,
                        uint32_t flags);
/* cfg->device must be the store's device; cfg->n_uuids must cover every id written so far */
int keto_store_snapshot(keto_store *st, const keto_snapshot_config *cfg, keto_snapshot **out);
/* The store's current content cut by patching `base`, a snapshot this store cut earlier (by
 * keto_store_snapshot or this call) whose version is still in the store's change log (the rows
 * of the last 4M inserted or deleted tuples).  Only the rows the transactions since base name
 * are rebuilt -- their nodes' set and Expand rows, their subjects' reverse rows and probe keys
 * (the reference's per-row write path: persistence/sql/relationtuples.go:104-126, 168-189,
 * 277-287) --; every other row is copied shifted, and node space, entities and the rewrite
 * program are shared with base.  Equal in every answer to keto_store_snapshot of the same
 * version.  When a transaction wrote something base has no node for (a new object, a new
 * (namespace, relation) pair, a uuid >= n_uuids), or base is not this store's or too old, the
 * full device build runs instead; *patched (optional) says which ran.  base stays valid. */
int keto_store_snapshot_patch(keto_store *st, const keto_snapshot *base, const keto_snapshot_config *cfg,
                              keto_snapshot **out, int32_t *patched);
/* ABI 6.  The store's current content in `snap` itself, advanced in place by the transactions
 * since its version -- work proportional to the rows they name, not to the graph (the
 * reference's write path touches only its rows: persistence/sql/relationtuples.go:104-126,
 * 168-189, 277-287).  snap must be a snapshot keto_store_snapshot cut from this store (advanced
 * any number of times since), with its version still in the change log, and NO batch may be in
 * flight on it: serve from a second snapshot meanwhile (keto_dispatcher_set_snapshot) and advance
 * the two in turn.  Rows that grow move into slack the snapshot keeps past its rows.
 * *advanced = 0 (snap unchanged, still at its version): the delta needs a full build -- a new
 * (namespace, relation) pair, a uuid past the id room, a namespace out of spare entities, a
 * shard-id tie in a row, the slack or relocation room spent, snap not this store's; cut a new one
 * with keto_store_snapshot.  An advanced snapshot is not saved (keto_snapshot_save refuses) nor
 * the base of keto_store_snapshot_patch (that call builds in full). */
int keto_store_snapshot_advance(keto_store *st, keto_snapshot *snap, int32_t *advanced);
int keto_store_info(keto_store *st, uint64_t *n_tuples, uint64_t *version);
int keto_store_free(keto_store *st);

/* Request coalescing for serving: concurrent callers, one batch per launch (the
 * dispatcher a Go shim puts behind CheckService, check/handler.go:304-331). */
typedef struct keto_dispatcher keto_dispatcher;
/* One finished dispatcher batch, for the caller's metrics (the reference's Prometheus / otel
 * hooks, internal/driver/registry_default.go:170-182, count requests above the engine; this is
 * what happens below it). */
typedef struct keto_batch_event {
    uint32_t kind;      /* 0 Check, 1 Expand */
    uint32_t requests;  /* callers coalesced into the batch */
    uint64_t queries;   /* queries / roots */
    double wall_ms;     /* the slot's copies + kernels + copies, host clock */
    double device_ms;   /* the check path / Expand traversal on the device (HIP events) */
    int32_t rc;         /* KETO_OK or the batch's error */
} keto_batch_event;
typedef void (*keto_batch_hook)(void *ctx, const keto_batch_event *ev);
typedef struct keto_dispatcher_config {
    keto_limits limits;
    uint32_t max_batch;   /* queries per launch (staging size); a larger request runs alone */
    uint32_t max_wait_us; /* 0: launch as soon as a slot is free with whatever is queued */
    uint32_t inflight;    /* batches in flight on their own streams (0 -> 4, at most 16) */
    uint32_t flags;       /* KETO_F_ERR_DETAIL: out_err as keto_check_batch with that flag */
    keto_batch_hook on_batch;  /* optional: called by the slot thread after each batch, callers released */
    void *hook_ctx;
} keto_dispatcher_config;
typedef struct keto_dispatcher_stats {
    uint64_t batches, requests, queries, max_batch_seen;
    double wall_ms_sum, device_ms_sum;  /* summed over the batches */
} keto_dispatcher_stats;

/* The snapshot must outlive the dispatcher (or be replaced with set_snapshot first). */
int keto_dispatcher_create(keto_snapshot *snap, const keto_dispatcher_config *cfg, keto_dispatcher **out);
int keto_dispatcher_destroy(keto_dispatcher *d);
/* Thread-safe; blocks until the n queries are decided.  Same outputs as keto_check_batch. */
int keto_dispatcher_check(keto_dispatcher *d, const keto_query *queries, uint64_t n, uint8_t *out_allowed,
                          int32_t *out_err);
/* Thread-safe Expand coalescing (expand.Engine.BuildTree behind ExpandService.Expand,
 * expand/handler.go:115-152): blocks until the n roots are expanded.  Same outputs as
 * keto_expand_batch for these roots (offsets relative to out_nodes; KETO_E_CAPACITY with
 * out_offsets[n] = required nodes if out_cap is too small). */
int keto_dispatcher_expand(keto_dispatcher *d, const keto_subject_set *roots, uint64_t n, keto_tree_node *out_nodes,
                           uint64_t out_cap, uint64_t *out_offsets, int32_t *out_err);
/* Switch to another snapshot (same device) between batches: batches taken after the call
 * use the new one; when this returns the previous snapshot is no longer in use and may be
 * freed (only batches taken before the swap are waited for, so sustained load cannot
 * starve it). */
int keto_dispatcher_set_snapshot(keto_dispatcher *d, keto_snapshot *snap);
int keto_dispatcher_stats_get(keto_dispatcher *d, keto_dispatcher_stats *out);

/* Name tables for the API form of a result (Mapper, uuid_mapping.go:199-399): id -> string
 * for namespaces, relations and interned UUIDs (the shim's MapUUIDsToStrings view of
 * keto_uuid_mappings, persistence/sql/uuid_mapping.go:19-33). */
typedef struct keto_name_tables {
    uint32_t n_namespaces;
    const char *const *namespace_names;
    uint32_t n_relations;
    const char *const *relation_names;
    uint64_t n_uuids;
    const char *const *uuid_strings;
} keto_name_tables;

/* Expand trees (keto_expand_batch output: nodes + offsets[n_trees+1]) -> API form, host
 * only.  Tree i becomes out[out_offsets[i] .. out_offsets[i+1]); a nil tree (empty range)
 * becomes zero bytes.  If cap is too small returns KETO_E_CAPACITY with
 * out_offsets[n_trees] = bytes required.
 *   json:  Mapper.ToTree (uuid_mapping.go:347-399) + encoding/json of ketoapi.Tree
 *          (ketoapi/public_api_definitions.go:217-229): the REST expand response body.
 *   proto: Mapper.ToTree + Tree.ToProto (ketoapi/enc_proto.go:119-133): serialized
 *          SubjectTree (expand_service.proto:77-92), the gRPC ExpandResponse.tree. */
int keto_trees_to_json(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                       const keto_name_tables *names, char *out, uint64_t cap, uint64_t *out_offsets);
int keto_trees_to_proto(const keto_tree_node *nodes, const uint64_t *offsets, uint64_t n_trees,
                        const keto_name_tables *names, uint8_t *out, uint64_t cap, uint64_t *out_offsets);

/* Owner of an object in a graph partitioned over nparts GPUs (BASELINE config 5,
 * SURVEY.md 8.1 (e)): every tuple of (ns, obj) lives on one rank, so all relation slots of
 * an object -- its direct rows, computed usersets and tuple-to-userset rows -- are local to
 * one partition.  A loader selects a rank's tuples with it; keto_partition_* routes object
 * requests with the same function. */
static inline uint32_t keto_object_owner(uint32_t ns, uint32_t obj, uint32_t nparts) {
    const uint64_t h = ((((uint64_t)ns) << 32) | obj) * 0x9E3779B97F4A7C15ull;
    return (uint32_t)((h >> 32) % nparts);
}

/* Graphs larger than one GPU: the job's ranks each hold the tuples they own
 * (keto_object_owner) and evaluate their own queries together.  There is no reference
 * counterpart (Keto never partitions); the decisions and trees are the whole graph's.
 *
 * A job of several ranks builds each rank's partition once, at creation, into a resident
 * snapshot (node arithmetic and relation flags agreed over the job).  A Check batch runs the
 * frontier engine on every rank at once: goals whose node another rank owns go to it as 32-byte
 * records, one all-to-all per generation, and their values come back, one all-to-all per
 * generation bottom-up.  The few queries whose answer could depend on
 * visited-set pruning (or that outgrow the goal budget) are routed to the closure path below, as
 * are Expand batches: a level-synchronous closure exchange (object requests to their owners,
 * their tuples back, max_read_depth + 1 levels), built into a device snapshot on which the
 * Check / Expand kernels run.  KETO_PART_CLOSURE=1 sends every batch down the closure path.
 *
 * A job of one rank (coll NULL or world 1) holds the whole graph: its partition is built once,
 * at creation, into a resident snapshot and every batch runs on it -- no closure, no per-batch
 * build.
 *
 * The exchange goes through the caller's collective, every rank calling in the same order (a Go
 * host wraps its RCCL communicator; the tests wrap gloo): the host-buffer alltoallv always, and
 * with alltoallv_device (optional, below) the library's device buffers on its stream: */
typedef struct keto_collective {
    void *ctx;
    int32_t rank, world;
    /* send[r] -> rank r; recv[r] <- rank r (one value per rank) */
    int (*alltoall_u64)(void *ctx, const uint64_t *send, uint64_t *recv);
    /* send: the bytes for rank 0, 1, ... back to back (send_bytes[r] each); recv likewise,
     * recv_bytes[r] from rank r (announced by the preceding alltoall_u64) */
    int (*alltoallv)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes);
    /* *value <- max over ranks */
    int (*allreduce_max_u64)(void *ctx, uint64_t *value);
    /* optional (NULL: alltoallv over host copies): the same all-to-all-v over DEVICE buffers of
     * the library's device, ordered on `stream` (the library's hipStream_t): the send bytes are
     * complete in stream order when it is called, and the library's later work on the stream
     * reads the received bytes.  An RCCL host enqueues ncclGroupStart, one ncclSend / ncclRecv
     * per peer and ncclGroupEnd on that stream -- the bytes move GPU to GPU over xGMI, no host
     * copy, no host synchronisation. */
    int (*alltoallv_device)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv,
                            const uint64_t *recv_bytes, void *stream);
} keto_collective;
typedef struct keto_partition_stats {
    /* the per-batch closure (a job of one rank on the closure path, Expand, and the queries the
     * distributed frontier routes): its levels, objects, tuples and bytes, and phase times */
    uint64_t batches, levels, objects, tuples, bytes_sent;
    double closure_s, build_s, run_s;
    /* a KETO_F_COUNT_WORK batch: the check kernels' work counters (keto_work_counters, tier 0) */
    uint64_t rows, edges, probes, queries;
    /* ABI 5, a job of several ranks over resident partitions (the distributed frontier): its
     * generations and goals on this rank, the queries it routed to the closure path, the goal
     * records and decisions this rank sent to the other ranks (bytes), its time on the device
     * (the generations' kernels, HIP events) and inside the collective */
    uint64_t generations, goals, routed, exchange_bytes;
    double device_s, exchange_s;
} keto_partition_stats;
typedef struct keto_partition keto_partition;
/* tuples: this rank's partition (host, or device memory of cfg->device with
 * KETO_F_DEVICE_PTRS); coll NULL = one rank, no exchange (KETO_F_PART_DIST with a one-rank
 * collective: the distributed frontier over the exchanges regardless).  The collective is kept
 * by value. */
int keto_partition_create(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, uint32_t flags,
                          const keto_collective *coll, const keto_limits *limits, keto_partition **out);
/* ABI 7: where the job's objects live, beside keto_object_owner's hash.  block[ns] > 0 puts
 * object obj of namespace ns (ns < 16) on rank (obj / block[ns]) % world: whole id ranges on one
 * rank -- a deployment whose objects of a hierarchy are numbered together (a folder tree under
 * its root) keeps a tuple-to-userset chain on one rank, so the distributed frontier walks it in
 * one goal instead of a record and a generation per hop.  KETO_PLACE_ALL replicates the
 * namespace: every rank loads all of its tuples and owns all of its objects (a group graph small
 * beside the rest: nested-group expand-subjects then run where they are spawned, with the
 * reachability tables).  0: the hash.  Every rank passes the same placement, and loads the
 * tuples whose keto_object_owner_placed is its rank or KETO_OWNER_ALL. */
#define KETO_PLACE_ALL 0xFFFFFFFFu
#define KETO_OWNER_ALL 0xFFFFFFFFu
typedef struct keto_placement {
    uint32_t block[16];
} keto_placement;
static inline uint32_t keto_object_owner_placed(const keto_placement *p, uint32_t ns, uint32_t obj, uint32_t nparts) {
    if (p && ns < 16 && p->block[ns] == KETO_PLACE_ALL) return KETO_OWNER_ALL;
    if (p && ns < 16 && p->block[ns]) return (obj / p->block[ns]) % nparts;
    return keto_object_owner(ns, obj, nparts);
}
/* keto_partition_create with a placement (NULL: keto_object_owner) */
int keto_partition_create_placed(const keto_snapshot_config *cfg, const keto_tuple *tuples, uint64_t n, uint32_t flags,
                                 const keto_collective *coll, const keto_limits *limits, const keto_placement *placement,
                                 keto_partition **out);
/* collective: this rank's queries (host) -> decisions, as keto_check_batch (flags: COUNT_WORK,
 * ERR_DETAIL).  Check closures ship subject-set tuples plus only the subject-id tuples that
 * name one of the batch's subjects: no other subject-id tuple is ever read by these queries. */
int keto_partition_check(keto_partition *p, const keto_query *queries, uint64_t n, uint8_t *out_allowed,
                         int32_t *out_err, uint32_t flags);
/* collective: n_batches batches in order, as keto_partition_check each, pipelined -- batch k+1's
 * closure exchange runs on a helper thread (which then calls the collective) while batch k is
 * built and checked (KETO_PART_SEQUENTIAL: one after another).  Every rank passes the same
 * n_batches.  Stats: the last batch's. */
int keto_partition_check_many(keto_partition *p, uint32_t n_batches, const keto_query *const *queries, const uint64_t *n,
                              uint8_t *const *out_allowed, int32_t *const *out_err, uint32_t flags);
/* collective: expands this rank's roots; *out_nodes_needed = nodes of all the trees.  Then
 * (local, no collective) keto_partition_expand_result copies them out, as keto_expand_batch. */
int keto_partition_expand(keto_partition *p, const keto_subject_set *roots, uint64_t n, uint64_t *out_nodes_needed);
int keto_partition_expand_result(keto_partition *p, keto_tree_node *out_nodes, uint64_t out_cap, uint64_t *out_offsets,
                                 int32_t *out_err);
/* the last batch's closure and phase times */
int keto_partition_stats_get(keto_partition *p, keto_partition_stats *out);
/* The last batch's exchange level by level (a job of one rank over its resident snapshot has
 * none): *n = the levels run; the first min(cap, *n) are copied to out.  Closure path: one level
 * per closure level.  Distributed frontier (several ranks): one level per generation, with the
 * fields as commented in brackets. */
typedef struct keto_partition_level {
    uint64_t objects;          /* objects this rank asked for at this level (new to its seen set)
                                  [the generation's goals on this rank] */
    uint64_t request_bytes;    /* object keys it sent to the other ranks [goal records it sent to them] */
    uint64_t tuples;           /* tuples it received: its closure grows by these [goal records it received] */
    uint64_t tuple_bytes_sent; /* tuples it shipped to the other ranks (as an owner) [values it returned to them] */
    double ms;                 /* the level's wall time on this rank (0 when the levels were enqueued at once)
                                  [device time of the generation's kernels, both passes: no collective wait] */
} keto_partition_level;
int keto_partition_levels_get(keto_partition *p, keto_partition_level *out, uint32_t cap, uint32_t *n);
/* ABI 7: the last distributed-frontier batch generation by generation, under its own names (a
 * job on the closure path or over one resident snapshot has none): *n = the generations run; the
 * first min(cap, *n) are copied to out.  A batch run in chunks sums its chunks per generation. */
typedef struct keto_partition_generation {
    uint64_t goals;            /* the generation's goals on this rank (proxies of remote children included) */
    uint64_t record_bytes_out; /* goal records this rank sent to the other ranks, wire bytes */
    uint64_t records_in;       /* goal records it received: goals of the next generation here */
    uint64_t value_bytes_back; /* values of received goals it returned to their senders, bytes */
    double ms;                 /* device time of the generation's kernels, both passes (no collective wait) */
} keto_partition_generation;
int keto_partition_generations_get(keto_partition *p, keto_partition_generation *out, uint32_t cap, uint32_t *n);
int keto_partition_free(keto_partition *p);

/* pinned host memory (hipHostMalloc) for the query / output buffers of KETO_F_ASYNC batches */
int keto_host_alloc(uint64_t bytes, void **out);
int keto_host_free(void *p);
/* device memory helpers (for callers without their own allocator) */
int keto_device_alloc(int32_t device, uint64_t bytes, void **out);
int keto_device_free(void *p);
int keto_memcpy_h2d(keto_stream *s, void *dst, const void *src, uint64_t bytes);
int keto_memcpy_d2h(keto_stream *s, void *dst, const void *src, uint64_t bytes);
int keto_device_count(int32_t *out);

#ifdef __cplusplus
}
#endif
#endif
