// Device-resident snapshot layout shared by the host builder and the gfx950 kernels.
//
// Node space ("dense arithmetic layout"): every namespace ns owns a contiguous
// entity range [ent_base, ent_base + n_ent) (real objects sorted by uuid id,
// plus one phantom entity standing for every object the snapshot has never seen)
// and a fixed relation-slot count n_slots.  The node for (entity e, slot s) is
//     node = node_base[ns] + (e - ent_base[ns]) * n_slots[ns] + s
// so computed-userset and tuple-to-userset hops are pure arithmetic on the node id
// (rewrites.go:208-230, 242-293) and no per-node metadata is ever fetched.
// (ns, relname) pairs that own no slot are "virtual" nodes: they have no tuples,
// only a relation status (NIL / ERR), and are encoded as VIRT_BIT|ns<<16|relname.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace keto {

constexpr uint32_t VIRT_BIT = 0x80000000u;  // frame node id: virtual node

// Where a partitioned graph's objects live (keto_placement, include/keto_mi355x.h): block[ns] > 0
// puts object obj of namespace ns on rank (obj / block[ns]) % world -- whole id ranges on one
// rank, e.g. a folder tree on its root's; PLACE_ALL replicates the namespace (every rank holds all
// of its tuples: each owns it); 0 (and every ns >= PLACE_NS) hashes (keto_object_owner)
constexpr uint32_t PLACE_NS = 16, PLACE_ALL = 0xFFFFFFFFu;
struct Placement {
    uint32_t block[PLACE_NS];
};
// the owner rank, or PLACE_ALL for a replicated namespace
__host__ __device__ inline uint32_t place_owner(const Placement &p, uint32_t ns, uint32_t obj, uint32_t world) {
    const uint32_t b = ns < PLACE_NS ? p.block[ns] : 0u;
    if (b == PLACE_ALL) return PLACE_ALL;
    if (b) return (obj / b) % world;
    const uint64_t h = ((((uint64_t)ns) << 32) | obj) * 0x9E3779B97F4A7C15ull;
    return (uint32_t)((h >> 32) % world);
}
// an owner lookup's arguments, passed by value to the routing kernels (a replicated object is the
// asking rank's own)
struct Dest {
    uint32_t world, rank;
    Placement pl;
    __host__ __device__ uint32_t owner(uint32_t ns, uint32_t obj) const {
        const uint32_t o = place_owner(pl, ns, obj, world);
        return o == PLACE_ALL ? rank : o;
    }
};
constexpr uint32_t EDGE_ALIAS = 0x80000000u; // set_dst entry: visited key != node id
// set_dst entry (snapshots of < 2^30 nodes, DevSnapshot::edge_leaf): the child node holds no
// subject-set tuple, so its expand-subject finds nothing -- an ES child the frontier engine
// decides at spawn instead of spawning a goal that reads an empty row
constexpr uint32_t EDGE_LEAF = 0x40000000u;
// set_dst entry of a partitioned graph's snapshot (frontier_dist.hip; these snapshots carry no
// EDGE_LEAF): the child node belongs to an object another rank owns -- its rows are there
constexpr uint32_t EDGE_REMOTE = 0x40000000u;
constexpr uint32_t SKEY_SET = 0x80000000u;   // all-row entry: subject set (else subject id)
constexpr uint32_t NO_SLOT = 0xFFFFu;
constexpr uint32_t NO_OP = 0xFFFFu;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;

// relation status of (ns, relname) per namespace.ASTRelationFor
// (internal/namespace/definitions.go:37-62)
enum RelStatus : uint32_t { REL_NIL = 0, REL_DECLARED = 1, REL_ERROR = 2 };

// relinfo word (per (ns, slot)):  bits 0-15 rewrite op (NO_OP = none)
//   bit 16 has_rewrite, bit 17 can_have_subject_sets (engine.go:233-235), bits 18-19 status
//   bit 20 shared visited class (vkey array must be consulted), bit 21 some row of the slot holds
//   a subject set, bit 22 some row of the slot holds a subject id (both set by the snapshot
//   builder; virtual nodes never)
__host__ __device__ inline uint32_t ri_op(uint32_t ri) { return ri & 0xFFFFu; }
__host__ __device__ inline bool ri_rw(uint32_t ri) { return (ri >> 16) & 1u; }
__host__ __device__ inline bool ri_ss(uint32_t ri) { return (ri >> 17) & 1u; }
__host__ __device__ inline uint32_t ri_status(uint32_t ri) { return (ri >> 18) & 3u; }
__host__ __device__ inline bool ri_shared(uint32_t ri) { return (ri >> 20) & 1u; }
constexpr uint32_t RI_SETROWS = 1u << 21;
__host__ __device__ inline bool ri_setrows(uint32_t ri) { return (ri >> 21) & 1u; }
constexpr uint32_t RI_IDROWS = 1u << 22;
// bit 23: the slot's nodes have reachability tables (reach.hip; DevSnapshot::reach_base)
constexpr uint32_t RI_REACH = 1u << 23;
__host__ __device__ inline bool ri_idrows(uint32_t ri) { return (ri >> 22) & 1u; }
__host__ __device__ inline uint32_t make_ri(uint32_t op, bool rw, bool ss, uint32_t status, bool shared) {
    return (op & 0xFFFFu) | (uint32_t(rw) << 16) | (uint32_t(ss) << 17) | (status << 18) | (uint32_t(shared) << 20);
}
// nsrel word (per (ns, relname)): bits 0-15 slot (NO_SLOT = virtual), bits 16-17 status
__host__ __device__ inline uint32_t nr_slot(uint32_t w) { return w & 0xFFFFu; }
__host__ __device__ inline uint32_t nr_status(uint32_t w) { return (w >> 16) & 3u; }

// rewrite program op (flattened ast.SubjectSetRewrite / Child, ast_definitions.go:8-72)
enum OpType : uint32_t { OP_REWRITE = 0, OP_CSS = 1, OP_TTU = 2, OP_INVERT = 3 };
enum OpKind : uint32_t { OPK_OR = 0, OPK_AND = 1, OPK_BAD = 2 };
struct alignas(16) Op {
    uint32_t type_kind;    // type | kind << 8 | has_css << 16
    uint32_t child_begin;  // into op_children
    uint32_t child_count;
    uint32_t rel_computed; // CSS: rel | 0 ; TTU: tupleset rel | computed << 16
};

// OR rewrites flattened for the frontier engine (frontier.hip): an OR's items in add order --
// its IN shortcut, the shortcut candidates, its other children -- with nested OR rewrites spliced
// in (IT_NEST guards them: rest depth d - k <= 0 makes the nested OR Unknown; skip to `end`).
// item {x = kind | k << 4 | end << 16, y = arg}; k = nesting depth (each nested rewrite costs 1)
enum OrItemKind : uint32_t { IT_NEST = 0, IT_SHORT = 1, IT_CAND = 2, IT_TTU = 3, IT_INV = 4, IT_RW = 5 };
__host__ __device__ inline uint32_t it_kind(uint32_t x) { return x & 0xFu; }
__host__ __device__ inline uint32_t it_k(uint32_t x) { return (x >> 4) & 0xFFFu; }
__host__ __device__ inline uint32_t it_end(uint32_t x) { return x >> 16; }

struct alignas(16) NsDev {
    uint32_t ent_base, node_base, n_slots, slot_base;
};

// Device view (all pointers device memory).  Passed by value to kernels.
struct DevSnapshot {
    const uint4 *set_row;      // [n_nodes] {begin, end, edge 0, edge 1} of each subject-set row (ES + TTU):
                               // one 16 B load; rows of <= 2 edges need no set_dst load
    const uint32_t *set_dst;   // node | EDGE_ALIAS | EDGE_LEAF, shard order within a row
    uint32_t edge_mask;        // node bits of a set_dst entry (and of set_row's inline edges)
    uint32_t edge_leaf;        // set_dst entries carry EDGE_LEAF
    const uint32_t *weight;    // [n_nodes] capped path count below a node (longest-first scheduling)
    const uint32_t *ent_obj;   // [n_entities] entity -> uuid id (NONE32 for phantoms): Expand output
    const uint32_t *slot_rel;  // [total slots] global slot -> relation name id: Expand output
    const uint32_t *vkey;      // [n_nodes] visited representative (only read for aliased nodes)
    const uint32_t *vclass;    // [total slots] partitioned graphs: visited class of a slot (frontier_goal.inc gkey)
    const uint32_t *all_off;   // [n_nodes+1]  every tuple of a node, shard order (Expand)
    const uint32_t *all_subj;  // subject id, or SKEY_SET|node
    const uint32_t *rev_off;   // [n_uuids + n_nodes + 1]  subject -> the nodes holding it (a multiset)
    const uint32_t *rev_nodes;
    // rows an in-place advance (advance.hip) moved: an all_off / rev_off word with ROW_MOVED is
    // the index of the row's {begin, end, the word's original offset, 0} here; null on every
    // snapshot that cannot be advanced in place (read rows through row_span)
    const uint4 *reloc;
    const NsDev *ns;           // [n_ns + 1] (sentinel: node_base = n_nodes)
    const uint32_t *relinfo;   // [total slots]
    const uint32_t *nsrel;     // [n_ns * n_rel]
    const Op *ops;
    const uint32_t *op_children;
    const uint32_t *op_items;  // [ops] OR ops: first item | item count << 16 (0: not an OR)
    const uint2 *or_items;     // flattened OR items
    // (ns, obj) -> entity rank table: block b covers ids [64b, 64b+64) of ck = ns*ent_stride+obj,
    // {set bits lo, hi, entity of the block's first set bit, 0}; an unset bit = no entity
    const uint4 *ent_rank;
    uint64_t ent_stride;
    // objects a patched store snapshot created (keto_store_snapshot_patch): open addressing over
    // {obj, ns, entity, 0}, entity NONE32 = empty; consulted when the rank table has no entity
    const uint4 *ext;
    uint32_t ext_mask;
    // membership probe hash for "heavy" subjects (reverse row longer than probe_k):
    // 16-byte buckets of two keys ((subject_idx<<32)|node)+1, linear probing over buckets
    const uint4 *probe;
    uint32_t probe_mask;  // bucket count - 1
    uint32_t probe_k;     // reverse rows up to this length are kept in VGPRs instead
    uint32_t n_ns, n_rel, n_nodes, n_uuids;
    // partitioned graphs' snapshots (frontier_dist.hip): every namespace ns has a ghost namespace
    // n_ns + ns (same slots) holding the subject-set objects other ranks own; n_ns_x = the ns
    // table's entries (0 = n_ns), n_owned = the first ghost node (node-indexed row arrays -- set_row,
    // all_off -- cover [0, n_owned) only: ghosts hold no rows here)
    uint32_t n_ns_x, n_owned;
    // reachability tables (reach.hip): a tabled node's reach over subject-set rows, for the
    // frontier's spawn-time NotMember (frontier_goal.inc reach_prunes); null when none
    const uint32_t *reach_base;  // [total slots] first reach_idx entry of a tabled slot, NONE32
    const uint4 *reach_idx;      // [tabled slots' entities] {count | NONE32: not tabled, entry 0, entry 1,
                                 //  pool offset of entries 2.. (runs padded to 4 entries)}
    const uint32_t *reach_pool;  // the reaches past their first two entries (nodes; the node itself not listed)
    // [ns table entries] 1.0 / n_slots (0 for a namespace without slots): node -> entity without
    // an integer division (device_common.hpp t_div_slots)
    const double *ns_rcp;
    int32_t strict;
    // byte sizes (multiples of 16) of ns, relinfo, nsrel, ops, op_children, op_items, or_items,
    // ns_rcp: staged in LDS
    uint32_t tab_bytes[8];
    uint32_t lds_bytes;
};

constexpr uint32_t ROW_MOVED = 1u << 31;  // all_off / rev_off word of a moved row (DevSnapshot::reloc)
// row i of an offset array (all_off, rev_off): [off[i], off[i+1]) unless the advance moved row i
// (its own word flagged: the relocated extent) or row i+1 (the flagged next word's original
// offset ends row i)
__device__ __forceinline__ void row_span(const uint32_t *off, const uint4 *reloc, uint64_t i, uint32_t &b, uint32_t &e) {
    b = off[i];
    e = off[i + 1];
    if (reloc && ((b | e) & ROW_MOVED)) {
        if (b & ROW_MOVED) {
            const uint4 r = reloc[b & ~ROW_MOVED];
            b = r.x;
            e = r.y;
        } else {
            e = reloc[e & ~ROW_MOVED].z;
        }
    }
}

constexpr uint32_t REACH_CAP = 32;         // nodes of a tabled reach, the node itself included (oracle reach_cap;
                                           // KETO_REACH_CAP <= REACH_CAP_MAX for A/B builds)
constexpr uint32_t REACH_CAP_MAX = 128;
constexpr uint32_t WEIGHT_ROUNDS = 12;     // path-count relaxation rounds (> typical max depth)
constexpr uint32_t WEIGHT_CAP = 1u << 20;
constexpr uint32_t HEAVY_WEIGHT = 32;      // roots at or above this weight are scheduled first
constexpr uint32_t START_HEAVY = 1u << 31;  // start record: subject row answered by the probe hash
constexpr uint32_t START_R_HEAVY = 0xFFFFFFFEu;  // second start record of a heavy subject: {subject, this, filter lo, hi}
// A heavy subject's start record carries a 64-bit filter of its reverse row (two bits per node,
// subj_filter_bits): a membership test whose bits are not all set is answered NotMember without
// the probe-hash load.  Rows longer than FILTER_MAX_LEN get an all-ones filter (no filtering).
constexpr uint32_t FILTER_MAX_LEN = 96;
__host__ __device__ __forceinline__ uint64_t subj_filter_bits(uint32_t node) {
    const uint32_t h = node * 0x9E3779B1u;
    return (1ull << (h >> 26)) | (1ull << ((h >> 20) & 63u));
}
constexpr uint32_t PROBE_K = 4;           // VGPR-resident reverse row capacity (<= 4: two windows)
constexpr uint32_t LDS_TABLE_LIMIT = 48 * 1024;

}  // namespace keto
