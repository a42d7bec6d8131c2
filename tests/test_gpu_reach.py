"""Reachability tables (csrc/reach.hip; frontier_goal.inc reach_prunes; oracle/refsem.c
u_reach_prunes) against the oracle.

The expand-subject of a "tabled" node n -- a pure relation (no rewrite, no ASTRelationFor
error) whose every reachable node over subject-set rows is pure, at most REACH_CAP of them -- is
NotMember when no node of that reach below n holds the subject in its own row, and the
frontier's expand-subject goal decides so at once: no scope, no children.  These worlds are nested groups built to hit every
place the rule must not fire or must stop: reaches past the cap (a group with 140 subgroups),
an impure node inside a reach (a Team whose members relation has a rewrite, an undeclared
relation that is an error), cycles, strict mode, request depths 1-12, width truncation and
subject-set subjects.  Decisions and errors must equal the canonical DFS (rs_check); routed and
goal counts must equal rs_check_u's with the rule on -- and the rule must actually prune: with it
off the same queries spawn more goals (internal/check/engine.go:102-164, 214-249)."""
import numpy as np
import pytest

import keto_mi355x as km
import refsem
from product_helpers import product_snapshot, queries_to_product

pytestmark = pytest.mark.gpu


def reach_world(seed: int, strict: bool, max_width: int):
    rng = np.random.default_rng(seed)
    member_types = [{"namespace": "User"}, {"namespace": "Group", "relation": "members"},
                    {"namespace": "Team", "relation": "members"}]
    namespaces = {
        "User": [],
        "Group": [{"name": "members", "types": member_types}, {"name": "owners", "types": member_types}],
        # Team#members has a rewrite: a group whose reach holds a team is never tabled
        "Team": [{"name": "leads", "types": [{"namespace": "User"}]},
                 {"name": "members", "types": member_types,
                  "rewrite": {"operator": "or", "children": [{"relation": "leads"}]}}],
        "Folder": [{"name": "viewers", "types": member_types},
                   {"name": "view", "rewrite": {"operator": "or", "children": [{"relation": "viewers"}]}}],
    }
    w = refsem.World(namespaces=namespaces, strict=strict, max_depth=12, max_width=max_width)
    users = [f"u{i}" for i in range(40)]
    n_groups = 220
    tuples = []
    for g in range(n_groups):
        for u in rng.choice(users, 3, replace=False):
            tuples.append(f"Group:g{g}#members@{u}")
        # nested groups: mostly a forward DAG of long chains, a few back edges (cycles)
        for _ in range(int(rng.integers(0, 3))):
            h = int(rng.integers(g + 1, n_groups)) if g + 1 < n_groups and rng.random() < 0.9 else int(rng.integers(0, n_groups))
            tuples.append(f"Group:g{g}#members@Group:g{h}#members")
        if rng.random() < 0.05:  # an impure node in the reach
            tuples.append(f"Group:g{g}#members@Team:t{g % 7}#members")
        if rng.random() < 0.03:  # a relation the Group namespace does not declare: an error node
            tuples.append(f"Group:g{g}#members@Group:g{(g + 5) % n_groups}#nope")
        if rng.random() < 0.2:
            tuples.append(f"Group:g{g}#owners@Group:g{int(rng.integers(0, n_groups))}#members")
    for k in range(140):  # a reach past REACH_CAP
        tuples.append(f"Group:big#members@Group:g{k}#members")
    for t in range(7):
        tuples.append(f"Team:t{t}#leads@{users[t]}")
        tuples.append(f"Team:t{t}#members@Group:g{t * 3}#members")
    for f in range(60):
        for _ in range(3):
            tuples.append(f"Folder:f{f}#viewers@Group:g{int(rng.integers(0, n_groups))}#members")
        if f % 10 == 0:
            tuples.append(f"Folder:f{f}#viewers@Group:big#members")
    tuples = sorted(set(tuples), key=tuples.index)
    hi, lo = refsem.seeded_shard_ids(len(tuples), seed + 11)
    t = w.tuple_array(tuples, hi, lo)
    queries = []
    for _ in range(900):
        u = users[int(rng.integers(0, len(users)))]
        d = int(rng.choice([0, 0, 0, 1, 2, 3, 5, 8, 12]))
        r = rng.random()
        if r < 0.4:
            queries.append((f"Group:g{int(rng.integers(0, n_groups))}#members@{u}", d))
        elif r < 0.55:
            queries.append((f"Group:g{int(rng.integers(0, n_groups))}#owners@{u}", d))
        elif r < 0.65:
            queries.append((f"Group:big#members@{u}", d))
        elif r < 0.75:
            queries.append((f"Group:g{int(rng.integers(0, n_groups))}#members@Group:g{int(rng.integers(0, n_groups))}#members", d))
        else:
            queries.append((f"Folder:f{int(rng.integers(0, 60))}#view@{u}", d))
    return w, t, w.query_array(queries)


@pytest.mark.parametrize("strict,max_width", [(False, 100), (False, 2), (True, 100)])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_reach_worlds_match_oracle(seed, strict, max_width):
    w, t, q = reach_world(seed, strict, max_width)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    dec, err, _ = orc.check_batch(q, threads=4)
    udec, uerr, routed, goals, _ = orc.check_u_batch(q, threads=4, budget=1024)
    orc.set_reach(False)
    _, _, routed0, goals0, _ = orc.check_u_batch(q, threads=4, budget=1024)
    orc.set_reach(True)
    ok = routed == 0
    np.testing.assert_array_equal(udec[ok], dec[ok])
    np.testing.assert_array_equal(uerr[ok], err[ok])
    assert dec.any() and not dec.all()
    assert int(goals.sum()) < int(goals0.sum())  # the rule prunes
    assert int(routed.sum()) <= int(routed0.sum())
    stream = km.Stream(0)
    try:
        snap = product_snapshot(w, t)
        assert snap.info()["n_reach"] > 0
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


def test_reach_tables_follow_in_place_advances():
    """keto_store_snapshot_advance keeps the tables exact where the set of tabled slots changes and
    where reaches cross the cap: transactions on a reach world cut the 140-child group under the
    cap, make Team#members a target of Folder viewers and then no target at all, grow and break
    nested-group chains, make Group#owners a target (a newly tabled slot: the tables rebuilt over
    the moved rows) and no target again -- after each, one store snapshot advanced in place answers, spawns and
    tables (n_reach) exactly as a full build of the same version (the decisions also as the oracle's)"""
    import json

    from product_helpers import tuples_to_product
    from store_ref import transact

    w, t, q = reach_world(4, False, 100)
    rng = np.random.default_rng(40)
    names = (json.dumps(w.namespaces), w.ns_names.names, w.rel_names.names)
    host = tuples_to_product(t)
    st = km.TupleStore(host)
    n_uuids = max(1, len(w.uuids.names))
    snap = km.Snapshot(names[0], None, names[1], names[2], n_uuids, store=st)
    qp = queries_to_product(q)

    def rows(lines):
        hi, lo = refsem.seeded_shard_ids(len(lines), int(rng.integers(1 << 30)))
        return tuples_to_product(w.tuple_array(lines, hi, lo))

    def _rs(p):  # product records back to the oracle's layout
        out = np.zeros(len(p), dtype=refsem.TUPLE_DT)
        for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("subj_kind", "kind"), ("s_obj", "sid"),
                     ("s_ns", "sns"), ("s_rel", "srel")):
            out[b] = p[a]
        sb = p["shard_id"].astype(np.uint64)
        out["shard_hi"] = sum(sb[:, k] << np.uint64(8 * (7 - k)) for k in range(8))
        out["shard_lo"] = sum(sb[:, 8 + k] << np.uint64(8 * (7 - k)) for k in range(8))
        return out

    steps = [
        (None, [f"Group:big#members@Group:g{k}#members" for k in range(120)]),  # the big group falls under the cap
        ([f"Folder:f{f}#viewers@Team:t{f % 7}#members" for f in range(20)]  # Team#members: a target of viewers
         + [f"Group:g{g}#members@Group:g{g + 1}#members" for g in range(30, 60)]
         + ["Folder:f3#viewers@Group:g5#owners"], None),  # Group#owners a target: a newly tabled slot
        (None, [f"Folder:f{f}#viewers@Team:t{f % 7}#members" for f in range(20)]  # ... and none again
         + [f"Group:g{g}#members@Team:t{g % 7}#members" for g in range(220)]
         + ["Folder:f3#viewers@Group:g5#owners"]),  # Group#owners untabled again
        ([f"Group:big#members@Group:g{k}#members" for k in range(150, 219)], [f"Group:g{g}#members@Group:g{g + 1}#members"
                                                                            for g in range(40, 50)]),
    ]
    for i, (ins, dele) in enumerate(steps):
        ins_p = rows(ins) if ins else host[:0]
        del_p = rows(dele) if dele else host[:0]
        st.transact(ins_p, del_p)
        host = transact(host, ins_p, del_p)
        assert snap.advance(st), i
        full = km.Snapshot(names[0], None, names[1], names[2], n_uuids, store=st)  # (spares alike: n_reach counts them)
        out = []
        for s in (snap, full):
            stream = km.Stream(0)
            eng = km.CheckEngine(s, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
            stream.frontier_stats(reset=True)
            a, e = eng.check_batch(qp)
            fs = stream.frontier_stats(reset=True)
            out.append((a, e, fs["goals"], fs["routed"], s.info()["n_reach"]))
            stream.close()
        (a1, e1, g1, r1, n1), (a2, e2, g2, r2, n2) = out
        np.testing.assert_array_equal(a1, a2)
        np.testing.assert_array_equal(e1, e2)
        assert n1 == n2, (i, n1, n2)
        assert r1 == r2
        if r1 == 0:
            assert g1 == g2, (i, g1, g2)
        orc = refsem.Oracle(w, _rs(host))
        orc.set_limits(w.max_depth, w.max_width)
        dec, err, _ = orc.check_batch(q, threads=4)
        np.testing.assert_array_equal(a1, dec)
        np.testing.assert_array_equal(e1, err)
        full.close()
    snap.close()
    st.close()
