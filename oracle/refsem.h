/*
 * refsem.h -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * A plain-C, single-threaded-per-query restatement of the reference Keto
 * Check / Expand semantics (Go sources under /root/reference, cited per
 * function in refsem.c).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (djy-keto_amd/, libketo_mi355x.so) never links or calls it.
 *
 * Parity pinning: the oracle is checked against the known-answer vectors
 * transcribed from the reference's own tests into tests/golden/ (JSON fixtures)
 * (see tests/golden/make_golden.py for the file:line of every vector).
 * The reference itself (Go) cannot be built in this image (no Go
 * toolchain), so there is no oracle/_ref build.
 */
#ifndef KETO_REFSEM_H
#define KETO_REFSEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One relation tuple, ids interned by the caller.  kind 0 = SubjectID
 * (sid = subject id), kind 1 = SubjectSet (sns:sid#srel).  shard_hi/lo is
 * the tuple's shard_id UUID as two big-endian halves (or its raw bytes, see
 * rs_config.shard_bytes); it fixes every
 * iteration order (reference: persistence/sql/relationtuples.go:113). */
typedef struct {
    uint32_t ns, obj, rel;
    uint32_t kind;
    uint32_t sid;
    uint32_t sns, srel;
    uint32_t pad;
    uint64_t shard_hi, shard_lo;
} rs_tuple;

/* Check query: ns:obj#rel@subject with request max-depth (<=0 -> global). */
typedef struct {
    uint32_t ns, obj, rel;
    uint32_t kind, sid, sns, srel;
    int32_t depth;
} rs_query;

/* Flattened namespace AST (reference: internal/namespace/ast/ast_definitions.go:8-72). */
enum { RS_REWRITE = 0, RS_CSS = 1, RS_TTU = 2, RS_INVERT = 3 };
enum { RS_OP_OR = 0, RS_OP_AND = 1 };
typedef struct {
    int32_t type;        /* RS_REWRITE / RS_CSS / RS_TTU / RS_INVERT */
    int32_t op;          /* RS_REWRITE: RS_OP_OR / RS_OP_AND (others: not implemented) */
    uint32_t rel;        /* CSS: relation; TTU: tupleset relation */
    uint32_t computed;   /* TTU: computed subject-set relation */
    int32_t child_begin; /* REWRITE/INVERT: index into children[] */
    int32_t child_count;
} rs_ast;

typedef struct {
    uint32_t name;       /* relation-name id */
    int32_t rewrite;     /* ast index of the relation's SubjectSetRewrite, -1 = none */
    int32_t has_ss_type; /* a declared type carries a relation (containsSubjectSetExpand) */
    int32_t pad;
} rs_rel;

typedef struct {
    int32_t configured;  /* namespace known to the namespace manager */
    int32_t rel_begin;   /* index into rels[] */
    int32_t rel_count;   /* 0 = legacy namespace without relation config */
    int32_t pad;
} rs_ns;

typedef struct {
    uint32_t n_ns, n_relnames, empty_rel;
    const rs_ns *ns;
    const rs_rel *rels;
    uint32_t n_rels;
    const rs_ast *ast;
    uint32_t n_ast;
    const int32_t *children;
    uint32_t n_children;
    /* [n_ns * n_relnames]: equal ids <=> equal ns+"-"+rel strings
     * (visited key, relationtuple/definitions.go:114-116) */
    const uint32_t *vclass;
    int32_t strict, max_depth, max_width;
    /* 1: shard_hi/lo hold the shard_id's raw UUID bytes (the engine's keto_tuple layout),
     * 0: the two big-endian halves as numbers */
    int32_t shard_bytes;
} rs_config;

/* Work counters for the algorithmic-byte model:
 * B = 8*rows + 4*edges + 8*probes + 17 per check. */
typedef struct {
    uint64_t rows, edges, probes, out_nodes;
} rs_stats;

/* Membership codes (checkgroup/definitions.go:68-72) and error codes. */
enum { RS_UNKNOWN = 0, RS_IS_MEMBER = 1, RS_NOT_MEMBER = 2 };
enum { RS_OK = 0, RS_ERR_NO_RELATION = 1, RS_ERR_INTERNAL = 2, RS_ERR_NOT_IMPLEMENTED = 3 };

/* Expand tree node in pre-order; TREE_UNION = 1, TREE_LEAF = 4 (ketoapi enc_proto.go:164-176). */
typedef struct {
    uint32_t type, kind, sid, sns, srel, n_children;
} rs_tree_node;

typedef struct rs_db rs_db;

rs_db *rs_build(const rs_tuple *tuples, size_t n, const rs_config *cfg);
void rs_free(rs_db *db);
void rs_set_limits(rs_db *db, int32_t max_depth, int32_t max_width);
/* the frontier restatement's reachability rule (u_reach_prunes) on / off (default on, unless
 * RS_NO_REACH=1): the product's snapshots carry the tables unless KETO_NO_REACH=1 */
void rs_set_reach(rs_db *db, int on);

/* Returns membership; *err receives the error code. */
int rs_check(rs_db *db, const rs_query *q, int32_t *err, rs_stats *st);

/* Multi-threaded batch (CPU baseline): decision[i] = allowed, err[i]. */
void rs_check_batch(rs_db *db, const rs_query *q, size_t n, int threads,
                    uint8_t *decision, int32_t *err, rs_stats *st);

/* Schedule-sensitivity report.  The canonical (eager-marking) result,
 * plus flags: RS_F_SENSITIVE when some visited scope both pruned a sibling as already
 * visited and saw an order-sensitive event (depth or width truncation, an error, AND / NOT)
 * under either simulated schedule or in the maximal-exploration tree (the conservative
 * criterion); RS_F_SEQ_DIFFERS when the
 * sequential schedule (every child done before the next sibling is marked) decides
 * differently.  Runs each query three times (two schedules, the maximal-exploration tree). */
#define RS_F_SENSITIVE 1u
#define RS_F_SEQ_DIFFERS 2u
/* set (with RS_F_SENSITIVE) when the maximal-exploration criterion fired: the tree of every
 * check the reference's eager construction can start (refsem.c "Maximal exploration") */
#define RS_F_MAXEXP 4u
int rs_check_ex(rs_db *db, const rs_query *q, int32_t *err, rs_stats *st, uint32_t *flags);
void rs_check_batch_ex(rs_db *db, const rs_query *q, size_t n, int threads, uint8_t *decision,
                       int32_t *err, uint32_t *flags, rs_stats *st);

/* Frontier semantics (refsem.c "Frontier semantics"; the spec of csrc/frontier.hip): the
 * query evaluated without visited pruning.  *routed = 1 when a visited scope would receive a
 * key twice or the query spawns more than `budget` goals -- only then may the result differ
 * from rs_check's.  *goals = goals spawned, *gens = goal-tree generations. */
int rs_check_u(rs_db *db, const rs_query *q, uint32_t budget, int32_t *err, uint32_t *routed, uint32_t *goals,
               uint32_t *gens);
void rs_check_u_batch(rs_db *db, const rs_query *q, size_t n, int threads, uint32_t budget, uint8_t *decision,
                      int32_t *err, uint32_t *routed, uint32_t *goals, uint32_t *gens);

/* Rows of every object within `levels` subject-set hops of (ns[i], obj[i]) (the SQL-mode
 * baseline's store, oracle/refsql.py): pos = the row's rank in the index, which keeps every
 * (ns, obj, rel)'s shard order.  Returns the count; only the first cap are written. */
typedef struct {
    uint32_t ns, obj, rel, kind, sid, sns, srel, pad;
    uint64_t pos;
} rs_row;
size_t rs_closure(rs_db *db, const uint32_t *ns, const uint32_t *obj, size_t n, int levels, rs_row *out, size_t cap);

/* Expand: returns number of nodes written (0 = nil tree), -1 if cap too small. */
long rs_expand(rs_db *db, uint32_t kind, uint32_t sid, uint32_t sns, uint32_t srel,
               int32_t depth, rs_tree_node *out, size_t cap, rs_stats *st);

#ifdef __cplusplus
}
#endif
#endif
