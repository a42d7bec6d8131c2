// Device helpers shared by the check and expand kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "engine.hpp"

namespace keto {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// 16-byte aligned window holding element i of a u32 array
__device__ __forceinline__ const uint4 *win(const uint32_t *a, uint32_t i) {
    return reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(a + i) & ~uintptr_t(15));
}
__device__ __forceinline__ uint32_t wword(const uint4 &v, uint32_t k) {
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}
// element i of array a, given the window loaded for it
__device__ __forceinline__ uint32_t pick(const uint32_t *a, uint32_t i, const uint4 &v) {
    return wword(v, (uint32_t)((reinterpret_cast<uintptr_t>(a + i) >> 2) & 3));
}

// (ns, obj) -> entity id through the rank table (one 16-byte load); NONE32 if the object holds
// no tuple in ns (the caller then uses the namespace's phantom entity)
__device__ __forceinline__ uint32_t ent_lookup(const DevSnapshot &s, uint32_t ns, uint32_t obj, bool ghost = false) {
    if (ghost) ns += s.n_ns;  // (the caller checked that the snapshot has ghost namespaces)
    else if (ns >= s.n_ns) return NONE32;
    if (obj >= s.n_uuids) return NONE32;
    const uint64_t ck = (uint64_t)ns * s.ent_stride + obj;
    const uint4 b = s.ent_rank[ck >> 6];
    const uint64_t m = (uint64_t)b.x | ((uint64_t)b.y << 32);
    const uint32_t j = (uint32_t)(ck & 63);
    if (!((m >> j) & 1ull)) {
        if (!s.ext) return NONE32;
        for (uint32_t h = (uint32_t)mix64((((uint64_t)ns << 32) | obj) + 1) & s.ext_mask;; h = (h + 1) & s.ext_mask) {
            const uint4 x = s.ext[h];  // (at most half full: every walk ends at an empty slot)
            if (x.z == NONE32) return NONE32;
            if (x.x == obj && x.y == ns) return x.z;
        }
    }
    return b.z + (uint32_t)__popcll(m & ((1ull << j) - 1ull));
}

// Small per-snapshot tables (namespace table, relation info, rewrite program) staged in LDS.
struct Tables {
    const NsDev *ns;
    const uint32_t *relinfo;
    const uint32_t *nsrel;
    const Op *ops;
    const uint32_t *op_children;
    const uint32_t *op_items;
    const uint2 *or_items;
    const double *ns_rcp;
    uint32_t n_ns, n_rel;
    uint32_t n_ns_x;  // ns table entries (ghost namespaces of a partitioned graph's snapshot included)
};
__device__ __forceinline__ uint32_t ns_entries(const DevSnapshot &s) { return s.n_ns_x ? s.n_ns_x : s.n_ns; }
// a ghost namespace's namespace (partitioned graphs; identity otherwise)
__device__ __forceinline__ uint32_t t_real_ns(const Tables &T, uint32_t ns) { return ns >= T.n_ns ? ns - T.n_ns : ns; }

// (o / n_slots of namespace ns) for an offset o = node - node_base: ((double)o + 0.5) * (1 / n) lies
// within 3 * 2^-53 * o / n of (o + 0.5) / n, whose distance to the next integers is >= 0.5 / n;
// exact for o < 2^32 and n < 2^16 (3 * 2^-21 < 0.5 / 65535)
__device__ __forceinline__ uint32_t t_div_slots(const Tables &T, uint32_t ns, uint32_t o) {
    return (uint32_t)(((double)o + 0.5) * T.ns_rcp[ns]);
}

__device__ __forceinline__ uint32_t t_ns_of(const Tables &T, uint32_t node) {
    uint32_t lo = 0, hi = T.n_ns_x;  // last namespace whose node_base <= node
    while (hi - lo > 1) {
        uint32_t m = (lo + hi) >> 1;
        if (T.ns[m].node_base <= node) lo = m;
        else hi = m;
    }
    return lo;
}

struct NodeInfo {
    uint32_t ns, slot, ri;
};

__device__ __forceinline__ NodeInfo t_node_info(const Tables &T, uint32_t node) {
    NodeInfo r;
    if (node & VIRT_BIT) {
        r.ns = (node >> 16) & 0x7FFFu;
        r.slot = NO_SLOT;
        const uint32_t rel = node & 0xFFFFu;
        uint32_t st = (r.ns < T.n_ns && rel < T.n_rel) ? nr_status(T.nsrel[(size_t)r.ns * T.n_rel + rel]) : REL_NIL;
        r.ri = make_ri(NO_OP, false, true, st, false);  // no rewrite: direct + expand of an empty row
        return r;
    }
    r.ns = t_ns_of(T, node);
    const NsDev nd = T.ns[r.ns];
    const uint32_t o = node - nd.node_base;
    r.slot = o - t_div_slots(T, r.ns, o) * nd.n_slots;
    r.ri = T.relinfo[nd.slot_base + r.slot];
    return r;
}

// relation name id of a node (error detail: the relation ASTRelationFor rejects)
__device__ __forceinline__ uint32_t t_relname(const DevSnapshot &s, const Tables &T, uint32_t node, const NodeInfo &ni) {
    if (node & VIRT_BIT) return node & 0xFFFFu;
    return s.slot_rel[T.ns[ni.ns].slot_base + ni.slot];
}

// node of (same entity as `node`, relation `rel`): computed usersets / tuple-to-userset hops
// Relation ids past the snapshot's name table (a caller-side id the snapshot never saw) are
// clamped to the reserved last name, which no namespace declares: ASTRelationFor's
// "relation does not exist" for a configured namespace, nil otherwise (definitions.go:37-62).
__device__ __forceinline__ uint32_t t_rel(const Tables &T, uint32_t rel) { return rel < T.n_rel ? rel : T.n_rel - 1; }

__device__ __forceinline__ uint32_t t_sibling(const Tables &T, uint32_t node, const NodeInfo &ni, uint32_t rel) {
    rel = t_rel(T, rel);
    const uint32_t w = T.nsrel[(size_t)ni.ns * T.n_rel + rel];
    uint32_t slot = nr_slot(w);
    if (slot == NO_SLOT || (node & VIRT_BIT)) return VIRT_BIT | (t_real_ns(T, ni.ns) << 16) | (rel & 0xFFFFu);
    return node - ni.slot + slot;
}

// t_sibling and the sibling's node info (= t_node_info of the result) from the node's own: the
// sibling shares the entity, so its namespace and slot need no search or division
__device__ __forceinline__ uint32_t t_sibling_ni(const Tables &T, uint32_t node, const NodeInfo &ni, uint32_t rel, NodeInfo &out) {
    rel = t_rel(T, rel);
    const uint32_t w = T.nsrel[(size_t)ni.ns * T.n_rel + rel];
    const uint32_t slot = nr_slot(w);
    if (slot == NO_SLOT || (node & VIRT_BIT)) {
        const uint32_t v = VIRT_BIT | (t_real_ns(T, ni.ns) << 16) | (rel & 0xFFFFu);
        out = t_node_info(T, v);
        return v;
    }
    out.ns = ni.ns;
    out.slot = slot;
    out.ri = T.relinfo[T.ns[ni.ns].slot_base + slot];
    return node - ni.slot + slot;
}

// node of (ns, entity e, rel) given e; virtual if ns has no slot for rel
__device__ __forceinline__ uint32_t t_node(const Tables &T, uint32_t ns, uint32_t e, uint32_t rel) {
    rel = t_rel(T, rel);
    const uint32_t w = T.nsrel[(size_t)ns * T.n_rel + rel];
    if (nr_slot(w) == NO_SLOT) return VIRT_BIT | (ns << 16) | (rel & 0xFFFFu);
    const NsDev nd = T.ns[ns];
    return nd.node_base + (e - nd.ent_base) * nd.n_slots + nr_slot(w);
}

// Copy the small tables into dynamic LDS (whole block cooperates); returns LDS views.
__device__ __forceinline__ Tables stage_tables(const DevSnapshot &s, char *lds) {
    Tables T;
    T.n_ns = s.n_ns;
    T.n_rel = s.n_rel;
    T.n_ns_x = ns_entries(s);
    const uint4 *src[8] = {reinterpret_cast<const uint4 *>(s.ns), reinterpret_cast<const uint4 *>(s.relinfo),
                           reinterpret_cast<const uint4 *>(s.nsrel), reinterpret_cast<const uint4 *>(s.ops),
                           reinterpret_cast<const uint4 *>(s.op_children), reinterpret_cast<const uint4 *>(s.op_items),
                           reinterpret_cast<const uint4 *>(s.or_items), reinterpret_cast<const uint4 *>(s.ns_rcp)};
    uint32_t off = 0;
    char *dst[8];
    for (int i = 0; i < 8; i++) {
        dst[i] = lds + off;
        const uint32_t n16 = s.tab_bytes[i] / 16;
        for (uint32_t k = threadIdx.x; k < n16; k += blockDim.x) reinterpret_cast<uint4 *>(dst[i])[k] = src[i][k];
        off += s.tab_bytes[i];
    }
    __syncthreads();
    T.ns = reinterpret_cast<const NsDev *>(dst[0]);
    T.relinfo = reinterpret_cast<const uint32_t *>(dst[1]);
    T.nsrel = reinterpret_cast<const uint32_t *>(dst[2]);
    T.ops = reinterpret_cast<const Op *>(dst[3]);
    T.op_children = reinterpret_cast<const uint32_t *>(dst[4]);
    T.op_items = reinterpret_cast<const uint32_t *>(dst[5]);
    T.or_items = reinterpret_cast<const uint2 *>(dst[6]);
    T.ns_rcp = reinterpret_cast<const double *>(dst[7]);
    return T;
}

__device__ __forceinline__ Tables global_tables(const DevSnapshot &s) {
    return Tables{s.ns, s.relinfo, s.nsrel, s.ops, s.op_children, s.op_items, s.or_items, s.ns_rcp, s.n_ns, s.n_rel, ns_entries(s)};
}

}  // namespace keto
