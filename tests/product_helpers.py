"""Bridges between the oracle's World (test-side Mapper) and the product's C ABI records."""
import json

import numpy as np

import keto_mi355x as km
import refsem


def tuples_to_product(t_rs: np.ndarray) -> np.ndarray:
    out = np.zeros(len(t_rs), dtype=km.TUPLE_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("subj_kind", "kind"), ("s_obj", "sid"),
                 ("s_ns", "sns"), ("s_rel", "srel")):
        out[a] = t_rs[b]
    out["shard_id"] = km.shard_bytes(t_rs["shard_hi"], t_rs["shard_lo"])
    return out


def queries_to_product(q_rs: np.ndarray) -> np.ndarray:
    out = np.zeros(len(q_rs), dtype=km.QUERY_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("subj_kind", "kind"), ("s_obj", "sid"),
                 ("s_ns", "sns"), ("s_rel", "srel"), ("max_depth", "depth")):
        out[a] = q_rs[b]
    return out


def product_snapshot(world: refsem.World, t_rs: np.ndarray, device: int = 0) -> km.Snapshot:
    return km.Snapshot(json.dumps(world.namespaces), tuples_to_product(t_rs), world.ns_names.names,
                       world.rel_names.names, max(1, len(world.uuids.names)), strict=world.strict, device=device)


def product_tree_to_nested(world: refsem.World, nodes: np.ndarray):
    """product pre-order TREE_DT -> the same nested dict shape as refsem.tree_to_nested"""
    conv = np.zeros(len(nodes), dtype=refsem.TREE_DT)
    conv["type"] = nodes["type"]
    conv["kind"] = nodes["subj_kind"]
    conv["sid"] = nodes["s_obj"]
    conv["sns"] = nodes["s_ns"]
    conv["srel"] = nodes["s_rel"]
    conv["n_children"] = nodes["n_children"]
    return refsem.tree_to_nested(world, conv)


def world_from_workload(wl, with_tuples: bool = True):
    """oracle World over a synth Workload (same ids as the product snapshot); with the
    tuples converted to the oracle's record layout unless with_tuples=False (then t is None:
    give the oracle wl.tuples.view(refsem.TUPLE_DT) with shard_bytes=True instead)"""
    w = refsem.World(namespaces=wl.namespaces, strict=wl.strict, max_depth=wl.max_depth, max_width=wl.max_width)
    w.ns_names = refsem.Interner()
    w.rel_names = refsem.Interner()
    w.uuids = refsem.Interner()
    for n in wl.ns_names:
        w.ns_names(n)
    for r in wl.rel_names:
        w.rel_names(r)
    w._walk_names()
    if not with_tuples:
        return w, None
    t = np.zeros(len(wl.tuples), dtype=refsem.TUPLE_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("kind", "subj_kind"), ("sid", "s_obj"),
                 ("sns", "s_ns"), ("srel", "s_rel")):
        t[a] = wl.tuples[b]
    sb = wl.tuples["shard_id"]
    t["shard_hi"] = sb[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
    t["shard_lo"] = sb[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)
    return w, t


def queries_to_oracle(q):
    o = np.zeros(len(q), dtype=refsem.QUERY_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("kind", "subj_kind"), ("sid", "s_obj"),
                 ("sns", "s_ns"), ("srel", "s_rel"), ("depth", "max_depth")):
        o[a] = q[b]
    return o
