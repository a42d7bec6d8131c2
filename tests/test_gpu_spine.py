"""The spine (csrc/frontier_goal.inc spine_inner; oracle/refsem.c u_spine) against the oracle.

A rewrite goal whose last OR item is a one-parent tuple-to-userset, whose parent's check would be
another rewrite goal of an OR or and-merge shape, walks the parent's items itself, level after
level up the ancestors.  These worlds are folder chains built to hit every place the walk can
stop or change shape: a banned user at an ancestor (the and-merge fails there, and that level's
AND is an ordinary goal), an ancestor with two parents, a plain-OR spine (view2), a spine that
switches relation (edit -> view), an undeclared computed relation at the top of a chain (an
error leaf), group members (expand-subject goals at every level), request depths 1-16 and a
width limit that truncates rows.  Decisions and errors must equal the canonical DFS (rs_check);
routed counts and, with nothing routed, goal counts must equal rs_check_u's -- so the spine's
spawn rules are pinned goal for goal (internal/check/rewrites.go:33-134, 242-293, binop.go)."""
import numpy as np
import pytest

import keto_mi355x as km
import refsem
from product_helpers import product_snapshot, queries_to_product

pytestmark = pytest.mark.gpu


def _view(and_banned: bool, rel: str, computed: str):
    items = {"operator": "or", "children": [{"relation": "viewers"}, {"relation": "editors"},
                                            {"relation": "parents", "computed_subject_set_relation": computed}]}
    if not and_banned:
        return items
    return {"operator": "and", "children": [items, {"inverted": {"relation": "banned"}}]}


def spine_world(seed: int, max_width: int):
    rng = np.random.default_rng(seed)
    acl = [{"namespace": "User"}, {"namespace": "Group", "relation": "members"}]
    folder = [{"name": "parents", "types": [{"namespace": "Folder"}]},
              {"name": "viewers", "types": acl}, {"name": "editors", "types": acl},
              {"name": "banned", "types": [{"namespace": "User"}]},
              {"name": "view", "rewrite": _view(True, "view", "view")},
              {"name": "view2", "rewrite": _view(False, "view2", "view2")},
              {"name": "edit", "rewrite": {"operator": "or", "children": [
                  {"relation": "editors"}, {"relation": "parents", "computed_subject_set_relation": "view"}]}},
              {"name": "bad", "rewrite": {"operator": "or", "children": [
                  {"relation": "viewers"}, {"relation": "parents", "computed_subject_set_relation": "nope"}]}}]
    namespaces = {"User": [], "Group": [{"name": "members", "types": [{"namespace": "User"},
                                                                       {"namespace": "Group", "relation": "members"}]}],
                  "Folder": folder}
    w = refsem.World(namespaces=namespaces, strict=False, max_depth=16, max_width=max_width)
    users = [f"u{i}" for i in range(8)]
    groups = [f"g{i}" for i in range(6)]
    tuples = []
    for g in range(6):  # group members: users and nested groups
        for u in rng.choice(users, 2, replace=False):
            tuples.append(f"Group:g{g}#members@{u}")
        for h in range(g):  # nested groups (a DAG): rows past a small width limit get truncated
            if rng.random() < 0.5:
                tuples.append(f"Group:g{g}#members@Group:g{h}#members")
    chains, depth = 6, 14
    for c in range(chains):
        for i in range(depth):
            f = f"f{c}_{i}"
            if i > 0:
                tuples.append(f"Folder:{f}#parents@Folder:f{c}_{i - 1}#")
            if c == 3 and i == 6:  # a second parent: the spine stops here
                tuples.append(f"Folder:{f}#parents@Folder:f{(c + 1) % chains}_{i - 2}#")
            for rel in ("viewers", "editors"):
                if rng.random() < 0.25:
                    if rng.random() < 0.5:
                        tuples.append(f"Folder:{f}#{rel}@{rng.choice(users)}")
                    else:
                        tuples.append(f"Folder:{f}#{rel}@Group:{rng.choice(groups)}#members")
            if (c == 2 and i == 7) or rng.random() < 0.05:  # banned: the and-merge fails at this level
                tuples.append(f"Folder:{f}#banned@{rng.choice(users[:3])}")
    tuples = sorted(set(tuples), key=tuples.index)
    hi, lo = refsem.seeded_shard_ids(len(tuples), seed + 7)
    t = w.tuple_array(tuples, hi, lo)
    queries = []
    for c in range(chains):
        for i in range(0, depth, 2):
            for rel in ("view", "view2", "edit", "bad"):
                for u in users[:5]:
                    queries.append((f"Folder:f{c}_{i}#{rel}@{u}", int(rng.choice([0, 0, 1, 2, 3, 5, 9, 16]))))
            queries.append((f"Folder:f{c}_{i}#view@Group:{rng.choice(groups)}#members", 0))
    return w, t, w.query_array(queries)


@pytest.mark.parametrize("max_width", [10, 2, 1])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_spine_worlds_match_oracle(seed, max_width):
    w, t, q = spine_world(seed, max_width)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    dec, err, _ = orc.check_batch(q, threads=4)
    udec, uerr, routed, goals, _ = orc.check_u_batch(q, threads=4, budget=1024)
    ok = routed == 0
    np.testing.assert_array_equal(udec[ok], dec[ok])
    np.testing.assert_array_equal(uerr[ok], err[ok])
    assert (err != 0).any() and dec.any() and not dec.all()  # errors, members and non-members all occur
    stream = km.Stream(0)
    try:
        snap = product_snapshot(w, t)
        eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
        stream.frontier_stats(reset=True)
        allowed, gerr = eng.check_batch(queries_to_product(q))
        fs = stream.frontier_stats(reset=True)
        np.testing.assert_array_equal(gerr, err)
        np.testing.assert_array_equal(allowed, dec)
        assert fs["routed"] == int(routed.sum())
        if not routed.any():
            assert fs["goals"] == int(goals.sum())
        snap.close()
    finally:
        stream.close()


def test_async_speculation_learns_depth_and_routes_deeper(monkeypatch):
    """The generation engine's asynchronous batches speculate last-depth + 2 generations, the depth
    learned from the device after earlier batches (frontier.hip fr_gens_used).  A stream that ran
    shallow batches (request depths 1-2) then gets a deep one (the whole spine world at depth 16):
    what lies past the speculated generations is routed and the DFS interpreter answers it -- the
    decisions are the oracle's either way"""
    monkeypatch.setenv("KETO_FR_ENGINE", "gen")  # (small batches would run the block engine)
    w, t, q = spine_world(5, 10)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    shallow = q.copy()
    shallow["depth"] = 2
    deep = q.copy()
    deep["depth"] = 16
    stream = km.Stream(0)
    try:
        snap = product_snapshot(w, t)
        eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
        for batch in (shallow, shallow, shallow, deep, deep):
            dec, err, _ = orc.check_batch(batch, threads=4)
            qa = km.PinnedArray(len(batch), km.QUERY_DT)
            qa.array[:] = queries_to_product(batch)
            out = (km.PinnedArray(len(batch), np.uint8), km.PinnedArray(len(batch), np.int32))
            eng.check_batch_async(qa.array, out[0].array, out[1].array)
            stream.sync()
            np.testing.assert_array_equal(out[1].array, err)
            np.testing.assert_array_equal(out[0].array, dec)
            for a in (qa, *out):
                a.free()
        assert stream.frontier_stats()["async_batches"] == 5
        snap.close()
    finally:
        stream.close()
