"""Seeded random namespaces / tuples / queries that exercise every branch of the
Check and Expand semantics: OR shortcuts, AND/NOT, tuple-to-userset, computed
usersets, undeclared relations (errors), legacy and unconfigured namespaces,
subject sets with empty relations, cycles, depth and width truncation, strict mode."""
import numpy as np

import refsem


def _rewrite(rng, rels, depth):
    kind = rng.random()
    if depth <= 0 or kind < 0.35:
        if rng.random() < 0.55:
            return {"relation": rng.choice(rels)}
        return {"relation": rng.choice(rels), "computed_subject_set_relation": rng.choice(rels)}
    if kind < 0.5:
        return {"inverted": _rewrite(rng, rels, depth - 1)}
    op = "or" if rng.random() < 0.6 else "and"
    n = int(rng.integers(1, 4))
    return {"operator": op, "children": [_rewrite(rng, rels, depth - 1) for _ in range(n)]}


def random_world(seed: int, n_obj=10, n_users=6, n_tuples=70, rewrites: bool = True):
    rng = np.random.Generator(np.random.PCG64(seed))
    base_rels = ["a", "b", "c", "d"]
    namespaces = {}
    for ns in ["x", "y"]:
        rels = []
        for r in base_rels:
            rel = {"name": r}
            if rng.random() < 0.5:
                rel["types"] = [{"namespace": "x", "relation": str(rng.choice(base_rels))}] if rng.random() < 0.5 \
                    else [{"namespace": "u"}]
            if rewrites and rng.random() < 0.45:
                # mostly declared relations; occasionally an undeclared one ("zz") -> error path
                pool = base_rels + (["zz"] if rng.random() < 0.15 else [])
                rel["rewrite"] = _rewrite(rng, pool, 3)
                if "operator" not in rel["rewrite"]:
                    rel["rewrite"] = {"operator": "or", "children": [rel["rewrite"]]}
            rels.append(rel)
        namespaces[ns] = rels
    namespaces["leg"] = []  # legacy namespace without relation config
    # "free" is never configured (ASTRelationFor -> nil, no error)
    strict = bool(rng.random() < 0.3)
    w = refsem.World(namespaces=namespaces, strict=strict, max_depth=int(rng.integers(1, 8)),
                     max_width=int(rng.integers(1, 6)))
    nss = ["x", "y", "leg", "free"]
    rels_all = base_rels + ["", "zz", "..."]
    objs = [f"o{i}" for i in range(n_obj)]
    users = [f"u{i}" for i in range(n_users)]
    tuples = []
    for _ in range(n_tuples):
        ns = str(rng.choice(nss, p=[0.4, 0.3, 0.2, 0.1]))
        obj = str(rng.choice(objs))
        rel = str(rng.choice(base_rels)) if rng.random() < 0.9 else str(rng.choice(rels_all))
        if rng.random() < 0.45:
            subj = str(rng.choice(users))
        else:
            sns = str(rng.choice(nss, p=[0.4, 0.3, 0.2, 0.1]))
            srel = str(rng.choice(base_rels)) if rng.random() < 0.8 else str(rng.choice(rels_all))
            subj = f"{sns}:{rng.choice(objs)}#{srel}"
        tuples.append(f"{ns}:{obj}#{rel}@{subj}")
    tuples = sorted(set(tuples), key=tuples.index)
    hi, lo = refsem.seeded_shard_ids(len(tuples), seed + 1000)
    t = w.tuple_array(tuples, hi, lo)
    queries = []
    for _ in range(120):
        ns = str(rng.choice(nss, p=[0.45, 0.35, 0.15, 0.05]))
        obj = str(rng.choice(objs + ["unknown_obj"]))
        rel = str(rng.choice(base_rels)) if rng.random() < 0.9 else str(rng.choice(rels_all))
        if rng.random() < 0.7:
            subj = str(rng.choice(users + ["nobody"]))
        else:
            subj = f"{rng.choice(nss)}:{rng.choice(objs)}#{rng.choice(base_rels + [''])}"
        queries.append((f"{ns}:{obj}#{rel}@{subj}", int(rng.integers(-1, 8))))
    q = w.query_array(queries)
    expands = []
    for _ in range(12):
        expands.append((str(rng.choice(nss[:3])), str(rng.choice(objs)), str(rng.choice(base_rels)),
                        int(rng.integers(0, 7))))
    for ns, obj, rel, _ in expands:
        w.ns_names(ns), w.uuids(obj), w.rel_names(rel)
    return w, t, q, expands
