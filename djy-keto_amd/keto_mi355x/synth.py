"""Seeded synthetic workloads of BASELINE.json.

C2  nested groups: Group{members: (User | SubjectSet<Group,"members">)[]}, 1M groups in
    5 levels (group->subgroup edges only level l -> l+1), 8M user tuples (Zipf s=1.1
    over 2M users) + 2M group->subgroup tuples = 10M; max_read_depth 8; 2^20 queries,
    50% random-walk positives, 50% uniform, plus a 1% sub-batch at request depth 1-4.
C3  Drive: File/Folder{parents, viewers, editors, owners, banned; view, edit} as the OPL
    parser builds it (left-deep, internal/schema/parser.go:300-417 + simplifyExpression
    :519-537), a fanout-5 depth-10 folder forest, ~6 ACL tuples per node, 1M groups x
    ~20 members; max_read_depth 16.

Every generator is a pure function of (scale, seed) via numpy PCG64, so every rank of a
multi-GPU run rebuilds the identical replica.  shard_id = seeded UUIDv4 bytes per tuple.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._abi import QUERY_DT, TUPLE_DT


@dataclass
class Workload:
    name: str
    namespaces: dict
    ns_names: list
    rel_names: list
    n_uuids: int
    tuples: np.ndarray  # TUPLE_DT
    max_depth: int
    max_width: int = 100
    strict: bool = False
    meta: dict = None


def _shards(rng, n):
    b = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    b[:, 6] = (b[:, 6] & 0x0F) | 0x40  # UUIDv4 version
    b[:, 8] = (b[:, 8] & 0x3F) | 0x80  # RFC 4122 variant
    return b


def _zipf_ranks(rng, n_items, s, size):
    """Zipf(s) over [0, n_items) by inverse CDF on the exact finite distribution."""
    w = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = rng.random(size)
    return np.minimum(np.searchsorted(cdf, u, side="right"), n_items - 1)


def _dedupe(cols):
    """drop duplicate tuples (the relation-tuple table holds each tuple once)."""
    key = np.stack(cols, axis=1)
    _, idx = np.unique(key, axis=0, return_index=True)
    idx.sort()
    return idx


# --------------------------------------------------------------------------------------
# C2 nested groups

GROUPS_NS = {"Group": [{"name": "members", "types": [{"namespace": "User"},
                                                     {"namespace": "Group", "relation": "members"}]}],
             "User": []}


def nested_groups(n_tuples: int = 10_000_000, seed: int = 1, levels: int = 5) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    n_groups = max(levels, n_tuples // 10)            # 1M at 10M tuples
    n_users = max(1, n_tuples // 5)                   # 2M
    n_sub = n_tuples // 5                             # 2M group->subgroup
    n_user_t = n_tuples - n_sub                       # 8M
    lvl_size = n_groups // levels
    # group id g: level = g // lvl_size (last level absorbs the remainder)
    lvl_base = np.arange(levels) * lvl_size
    lvl_len = np.full(levels, lvl_size)
    lvl_len[-1] = n_groups - lvl_base[-1]
    # subgroup edges: parent level uniform over 0..levels-2, child in next level
    pl = rng.integers(0, levels - 1, size=n_sub)
    parent = lvl_base[pl] + (rng.random(n_sub) * lvl_len[pl]).astype(np.int64)
    child = lvl_base[pl + 1] + (rng.random(n_sub) * lvl_len[pl + 1]).astype(np.int64)
    ug = rng.integers(0, n_groups, size=n_user_t)
    uu = _zipf_ranks(rng, n_users, 1.1, n_user_t)
    # dedupe
    ks = _dedupe([parent, child])
    parent, child = parent[ks], child[ks]
    ku = _dedupe([ug, uu])
    ug, uu = ug[ku], uu[ku]
    n = len(parent) + len(ug)
    t = np.zeros(n, dtype=TUPLE_DT)
    # ids: ns Group=0 User=1; rel members=0; uuids: groups [0, G), users [G, G+U)
    t["ns"] = 0
    t["rel"] = 0
    m = len(parent)
    t["obj"][:m] = parent
    t["subj_kind"][:m] = 1
    t["s_obj"][:m] = child
    t["s_ns"][:m] = 0
    t["s_rel"][:m] = 0
    t["obj"][m:] = ug
    t["s_obj"][m:] = n_groups + uu
    t["shard_id"] = _shards(rng, n)
    perm = rng.permutation(n)  # insertion order is irrelevant; shard_id fixes iteration order
    t = t[perm]
    meta = {"n_groups": n_groups, "n_users": n_users, "levels": levels, "lvl_size": lvl_size, "seed": seed}
    return Workload("nested_groups", GROUPS_NS, ["Group", "User"], ["members", ""], n_groups + n_users, t, 8,
                    meta=meta)


def nested_groups_queries(w: Workload, n: int, seed: int = 7, trunc_frac: float = 0.01) -> np.ndarray:
    """50% random-walk positives, 50% uniform; a trunc_frac sub-batch uses request depth 1-4."""
    rng = np.random.Generator(np.random.PCG64(seed))
    G, U = w.meta["n_groups"], w.meta["n_users"]
    t = w.tuples
    sub = t[t["subj_kind"] == 1]
    usr = t[t["subj_kind"] == 0]
    # CSR of subgroup edges and of direct members (host-side, for the walk only)
    so = np.argsort(sub["obj"], kind="stable")
    s_obj, s_dst = sub["obj"][so], sub["s_obj"][so]
    s_off = np.searchsorted(s_obj, np.arange(G + 1))
    uo = np.argsort(usr["obj"], kind="stable")
    u_obj, u_dst = usr["obj"][uo], usr["s_obj"][uo]
    u_off = np.searchsorted(u_obj, np.arange(G + 1))
    q = np.zeros(n, dtype=QUERY_DT)
    q["ns"] = 0
    q["rel"] = 0
    q["s_ns"] = 0
    q["s_rel"] = 0
    npos = n // 2
    start = rng.integers(0, G, size=npos)
    cur = start.copy()
    steps = rng.integers(0, w.meta["levels"], size=npos)
    for k in range(w.meta["levels"]):
        deg = s_off[cur + 1] - s_off[cur]
        go = (steps > k) & (deg > 0)
        pick = s_off[cur] + (rng.random(npos) * np.maximum(deg, 1)).astype(np.int64)
        cur = np.where(go, s_dst[np.minimum(pick, len(s_dst) - 1)], cur)
    mdeg = u_off[cur + 1] - u_off[cur]
    mpick = u_off[cur] + (rng.random(npos) * np.maximum(mdeg, 1)).astype(np.int64)
    user = np.where(mdeg > 0, u_dst[np.minimum(mpick, len(u_dst) - 1)], G + rng.integers(0, U, size=npos))
    q["obj"][:npos] = start
    q["s_obj"][:npos] = user
    q["obj"][npos:] = rng.integers(0, G, size=n - npos)
    q["s_obj"][npos:] = G + rng.integers(0, U, size=n - npos)
    perm = rng.permutation(n)
    q = q[perm]
    ntr = int(n * trunc_frac)
    q["max_depth"][:ntr] = rng.integers(1, 5, size=ntr)
    return q


# --------------------------------------------------------------------------------------
# C3 Drive (folder hierarchy, parents.traverse + AND/NOT)

def _css(r):
    return {"relation": r}


def _ttu(r, c):
    return {"relation": r, "computed_subject_set_relation": c}


def _or(*c):
    return {"operator": "or", "children": list(c)}


def _and(*c):
    return {"operator": "and", "children": list(c)}


def _leftdeep_or(items):
    """parser.go: `a || b || c` -> {or,[{or,[{or,[a]},b]},c]} (no simplification below a group)"""
    root = {"operator": "or", "children": [items[0]]}
    for it in items[1:]:
        root = {"operator": "or", "children": [root, it]}
    return root


def drive_namespaces():
    acl_types = [{"namespace": "User"}, {"namespace": "Group", "relation": "members"}]
    # view: (viewers || editors || owners || parents.traverse(p => p.permits.view(ctx))) && !banned
    group = _leftdeep_or([_css("viewers"), _css("editors"), _css("owners"), _ttu("parents", "view")])
    # the parenthesised group becomes the AND's first child unsimplified (parser.go:330-345, 519-537)
    view = _and(group, {"inverted": _css("banned")})
    # edit: owners || parents.traverse(p => p.permits.edit(ctx))  -> simplified single OR
    edit = _or(_css("owners"), _ttu("parents", "edit"))
    rels = [{"name": "parents", "types": [{"namespace": "File"}, {"namespace": "Folder"}]},
            {"name": "viewers", "types": acl_types}, {"name": "editors", "types": acl_types},
            {"name": "owners", "types": acl_types}, {"name": "banned", "types": [{"namespace": "User"}]},
            {"name": "view", "rewrite": view}, {"name": "edit", "rewrite": edit}]
    return {"User": [],
            "Group": [{"name": "members", "types": [{"namespace": "User"}, {"namespace": "Group", "relation": "members"}]}],
            "Folder": rels, "File": rels}


def drive(depth: int = 10, fanout: int = 5, acl_per_node: int = 6, n_groups: int = 1_000_000,
          members_per_group: int = 20, n_users: int = 10_000_000, seed: int = 3) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    # nodes in BFS order: level sizes fanout^k; parent(i) = (i - 1) // fanout
    n_nodes = (fanout ** (depth + 1) - 1) // (fanout - 1)
    n_folders = (fanout ** depth - 1) // (fanout - 1)  # levels 0..depth-1
    NS_USER, NS_GROUP, NS_FOLDER, NS_FILE = 0, 1, 2, 3
    rel_names = ["parents", "viewers", "editors", "owners", "banned", "view", "edit", "members", ""]
    R = {r: i for i, r in enumerate(rel_names)}
    # uuid space: nodes [0, n_nodes), groups [n_nodes, +G), users after
    gbase, ubase = n_nodes, n_nodes + n_groups
    node_ns = np.where(np.arange(n_nodes) < n_folders, NS_FOLDER, NS_FILE).astype(np.uint32)
    parts = []
    # parent tuples: node#parents@Folder:parent (subject set, empty relation)
    child = np.arange(1, n_nodes, dtype=np.int64)
    par = (child - 1) // fanout
    pt = np.zeros(len(child), dtype=TUPLE_DT)
    pt["ns"] = node_ns[child]
    pt["obj"] = child
    pt["rel"] = R["parents"]
    pt["subj_kind"] = 1
    pt["s_obj"] = par
    pt["s_ns"] = NS_FOLDER
    pt["s_rel"] = R[""]
    parts.append(pt)
    # ACL tuples
    na = n_nodes * acl_per_node
    an = np.repeat(np.arange(n_nodes, dtype=np.int64), acl_per_node)
    rr = rng.random(na)
    arel = np.where(rr < 0.5, R["viewers"], np.where(rr < 0.7, R["editors"], np.where(rr < 0.9, R["owners"], R["banned"])))
    is_grp = (rng.random(na) < 0.3) & (arel != R["banned"])
    at = np.zeros(na, dtype=TUPLE_DT)
    at["ns"] = node_ns[an]
    at["obj"] = an
    at["rel"] = arel
    at["subj_kind"] = is_grp
    at["s_obj"] = np.where(is_grp, gbase + rng.integers(0, n_groups, size=na), ubase + rng.integers(0, n_users, size=na))
    at["s_ns"] = np.where(is_grp, NS_GROUP, 0)
    at["s_rel"] = np.where(is_grp, R["members"], 0)
    parts.append(at)
    # group members: mostly users, ~1 nested group each (acyclic: subgroup id > group id)
    ng = n_groups * members_per_group
    gg = np.repeat(np.arange(n_groups, dtype=np.int64), members_per_group)
    nested = (rng.random(ng) < 1.0 / members_per_group) & (gg < n_groups - 1)
    sub = gg + 1 + (rng.random(ng) * np.maximum(n_groups - gg - 1, 1)).astype(np.int64)
    gt = np.zeros(ng, dtype=TUPLE_DT)
    gt["ns"] = NS_GROUP
    gt["obj"] = gbase + gg
    gt["rel"] = R["members"]
    gt["subj_kind"] = nested
    gt["s_obj"] = np.where(nested, gbase + np.minimum(sub, n_groups - 1), ubase + rng.integers(0, n_users, size=ng))
    gt["s_ns"] = np.where(nested, NS_GROUP, 0)
    gt["s_rel"] = np.where(nested, R["members"], 0)
    parts.append(gt)
    t = np.concatenate(parts)
    t["shard_id"] = _shards(rng, len(t))
    meta = {"n_nodes": n_nodes, "n_folders": n_folders, "gbase": gbase, "ubase": ubase, "n_users": n_users,
            "n_groups": n_groups, "fanout": fanout, "depth": depth, "seed": seed}
    return Workload("drive", drive_namespaces(), ["User", "Group", "Folder", "File"], rel_names, ubase + n_users, t,
                    16, meta=meta)


def drive_queries(w: Workload, n: int, seed: int = 11) -> np.ndarray:
    """view/edit checks on random nodes; half the subjects are taken from the node's own
    or an ancestor's ACL (likely positives), half uniform users."""
    rng = np.random.Generator(np.random.PCG64(seed))
    m = w.meta
    t = w.tuples
    acl = t[(t["rel"] >= 1) & (t["rel"] <= 3) & (t["subj_kind"] == 0) & (t["obj"] < m["n_nodes"])]
    q = np.zeros(n, dtype=QUERY_DT)
    node = rng.integers(0, m["n_nodes"], size=n)
    q["ns"] = np.where(node < m["n_folders"], 2, 3)
    q["obj"] = node
    q["rel"] = np.where(rng.random(n) < 0.8, 5, 6)  # view / edit
    half = n // 2
    pick = rng.integers(0, len(acl), size=half)
    q["s_obj"][:half] = acl["s_obj"][pick]
    # place the ACL'd subject's node as the queried node or a descendant of it
    q["obj"][:half] = acl["obj"][pick]
    q["ns"][:half] = np.where(acl["obj"][pick] < m["n_folders"], 2, 3)
    q["s_obj"][half:] = m["ubase"] + rng.integers(0, m["n_users"], size=n - half)
    return q[rng.permutation(n)]
