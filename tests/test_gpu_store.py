"""Incremental snapshots (keto_store_*): TransactRelationTuples deltas applied on the device
give exactly the snapshot a full rebuild from the host-side transaction result gives, and
the oracle agrees on it; versions count transactions; a dispatcher picks the new snapshot
up between batches."""
import os

import numpy as np
import pytest

import keto_mi355x as km
import refsem
from keto_mi355x import synth
from product_helpers import queries_to_oracle, world_from_workload
from store_ref import transact

pytestmark = pytest.mark.gpu


def _delta(wl, rng, n_ins=3000, n_del=2000):
    t = wl.tuples
    ins = t[rng.choice(len(t), n_ins, replace=False)].copy()
    # new ACL rows: the same objects, other users (and a few exact duplicates of stored rows)
    users = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], n_ins)
    acl = (ins["rel"] != 0) & (ins["ns"] >= 2)
    ins["subj_kind"][acl], ins["s_obj"][acl], ins["s_ns"][acl], ins["s_rel"][acl] = 0, users[acl], 0, 0
    ins["shard_id"] = rng.integers(0, 256, (n_ins, 16), dtype=np.uint8)
    dele = t[rng.choice(len(t), n_del, replace=False)].copy()
    dele["shard_id"] = 0  # deletes match on content only
    dele = np.concatenate([dele, ins[:50]])  # rows inserted by the same transaction go too
    return ins, dele


def test_device_transactions_equal_host_rebuild():
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    rng = np.random.default_rng(0)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    for step in range(3):
        ins, dele = _delta(wl, rng)
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        n, version = st.info()
        assert n == len(host) and version == step + 1
    q = synth.drive_queries(wl, 20_000, seed=6)
    inc = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    assert inc.info()["version"] == 3 and inc.info()["n_tuples"] == len(host)
    full = km.Snapshot(wl.namespaces, host, wl.ns_names, wl.rel_names, wl.n_uuids)
    a1, e1 = km.CheckEngine(inc, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    a2, e2 = km.CheckEngine(full, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(e1, e2)
    w, _ = world_from_workload(wl)
    orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
    np.testing.assert_array_equal(a1, dec)
    # the deltas changed answers (the test is not vacuous)
    base = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    a0, _ = km.CheckEngine(base, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    assert (a0 != a1).any()
    st.close()


def test_delete_everything_and_duplicates():
    wl = synth.drive(depth=3, n_groups=100, n_users=300, seed=2)
    st = km.TupleStore(wl.tuples[:10])
    dup = wl.tuples[:2].copy()
    dup["shard_id"][:, 0] ^= 0xFF
    st.transact(dup, None)  # the same content twice: both rows stored
    assert st.info() == (12, 1)
    st.transact(None, wl.tuples[:1])  # removes both copies of row 0
    assert st.info() == (10, 2)
    st.transact(None, wl.tuples[:10])
    assert st.info() == (0, 3)
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 256, seed=1)
    a, _ = km.CheckEngine(snap, max_read_depth=wl.max_depth).check_batch(q)
    assert a.sum() == 0


def test_snapshot_save_load_round_trip(tmp_path):
    """keto_snapshot_save / _load (the snapshot file is the restart artefact):
    a Drive snapshot with rewrites and a cut store version, saved and loaded back, answers every
    Check and Expand exactly as the built one; a file of another kind is refused"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    st = km.TupleStore(wl.tuples)
    rng = np.random.default_rng(4)
    ins, dele = _delta(wl, rng, 500, 300)
    st.transact(ins, dele)
    built = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    path = tmp_path / "drive.ketosnap"
    built.save(path)
    loaded = km.Snapshot.load(path, wl.ns_names, wl.rel_names)
    bi, li = built.info(), loaded.info()
    for k in ("n_tuples", "n_nodes", "n_entities", "n_set_edges", "version", "device_bytes"):
        assert bi[k] == li[k], k
    q = synth.drive_queries(wl, 20_000, seed=6)
    q["max_depth"][:500] = rng.integers(1, 5, 500)
    a1, e1 = km.CheckEngine(built, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    a2, e2 = km.CheckEngine(loaded, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(e1, e2)
    roots = np.zeros(64, dtype=km.SUBJSET_DT)
    roots["ns"], roots["rel"] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    roots["obj"] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 64)
    n1, o1, x1 = km.ExpandEngine(built, max_read_depth=wl.max_depth).build_trees(roots)
    n2, o2, x2 = km.ExpandEngine(loaded, max_read_depth=wl.max_depth).build_trees(roots)
    np.testing.assert_array_equal(o1, o2)
    assert n1.tobytes() == n2.tobytes()
    bad = tmp_path / "bad.ketosnap"
    bad.write_bytes(b"not a snapshot" * 10)
    with pytest.raises(km.KetoError):
        km.Snapshot.load(bad, wl.ns_names, wl.rel_names)
    st.close()


def _edge_delta(wl, rng, t_now):
    """subject-set edges in and out: nested-group rows emptied (their parents' edges become
    leaves) and leaf groups given a nested group (their parents' edges stop being leaves), one
    user made heavy (> 4 reverse entries: probe keys) and a heavy subject made light again"""
    g_ns, mem = wl.ns_names.index("Group"), wl.rel_names.index("members")
    nested = t_now[(t_now["ns"] == g_ns) & (t_now["rel"] == mem) & (t_now["subj_kind"] == 1)]
    dele = nested[rng.choice(len(nested), min(40, len(nested)), replace=False)].copy()
    groups = wl.meta["gbase"] + rng.choice(wl.meta["n_groups"], 40, replace=False)
    ins = np.zeros(80, dtype=t_now.dtype)
    ins["ns"][:40], ins["obj"][:40], ins["rel"][:40] = g_ns, groups, mem
    ins["subj_kind"][:40], ins["s_ns"][:40], ins["s_rel"][:40] = 1, g_ns, mem
    ins["s_obj"][:40] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 40)
    acl = t_now[(t_now["ns"] >= 2) & (t_now["rel"] != wl.rel_names.index("parents"))]
    pick = acl[rng.choice(len(acl), 40, replace=False)].copy()
    pick["subj_kind"], pick["s_obj"], pick["s_ns"], pick["s_rel"] = 0, wl.meta["ubase"] + 7, 0, 0
    ins[40:] = pick
    ins["shard_id"] = rng.integers(0, 256, (80, 16), dtype=np.uint8)
    # a subject with many reverse entries loses all of them but two
    subj, cnt = np.unique(t_now["s_obj"][t_now["subj_kind"] == 0], return_counts=True)
    heavy = subj[np.argmax(cnt)]
    rows = t_now[(t_now["subj_kind"] == 0) & (t_now["s_obj"] == heavy)]
    dele = np.concatenate([dele, rows[2:]])
    dele["shard_id"] = 0
    return ins, dele


def _compare(wl, a, b, q, roots):
    """every Check answer (and the frontier's routed count, and its goal count -- the flags it
    reads: RI_SETROWS, EDGE_LEAF -- when no query is routed: a routed query stops spawning when
    its bit is seen, so its goals vary with timing on the GPU; the CPU emulation, one lane at a
    time, compares them exactly: tests/test_kernel_emulation.py) and every Expand tree of
    snapshot a equal b's"""
    out = []
    for snap in (a, b):
        stream = km.Stream(0)
        eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
        stream.frontier_stats(reset=True)
        al, er = eng.check_batch(q)
        fs = stream.frontier_stats(reset=True)
        nodes, offs, xerr = km.ExpandEngine(snap, stream, max_read_depth=wl.max_depth).build_trees(roots)
        out.append((al, er, fs["goals"], fs["routed"], nodes.tobytes(), offs, xerr))
        stream.close()
    (a1, e1, g1, r1, n1, o1, x1), (a2, e2, g2, r2, n2, o2, x2) = out
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(e1, e2)
    assert r1 == r2
    if r1 == 0 or os.environ.get("KETO_MI355X_LIB_OVERRIDE"):
        assert g1 == g2
    np.testing.assert_array_equal(o1, o2)
    np.testing.assert_array_equal(x1, x2)
    assert n1 == n2
    return a1


def _roots(wl, rng, n=256):
    r = np.zeros(n, dtype=km.SUBJSET_DT)
    h = n // 2
    r["ns"][:h], r["rel"][:h] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    r["obj"][:h] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], h)
    r["ns"][h:], r["rel"][h:] = wl.ns_names.index("Folder"), wl.rel_names.index("viewers")
    r["obj"][h:] = rng.integers(0, wl.meta["folders_per_root"], n - h)
    return r


def test_patched_snapshots_equal_full_builds():
    """keto_store_snapshot_patch: a chain of transactions -- ACL rows in and out, duplicates,
    nested-group edges in and out (leaf flags), subjects crossing the heavy threshold (probe keys
    and tombstones) -- each cut by patching the previous snapshot: every Check (with depth
    truncation), frontier goal count and Expand tree equals a full build of the same store
    version, and the oracle over the host-side transaction result agrees"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    rng = np.random.default_rng(3)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 20_000, seed=6)
    q["max_depth"][:500] = rng.integers(1, 5, 500)
    roots = _roots(wl, rng)
    w, _ = world_from_workload(wl)
    for step in range(4):
        ins, dele = _delta(wl, rng, 1500, 1000) if step % 2 == 0 else _edge_delta(wl, rng, host)
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        prev = snap
        snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=prev)
        assert snap.patched, f"step {step}: the full build ran"
        full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
        pi, fi = snap.info(), full.info()
        for k in ("n_tuples", "n_set_edges", "version", "n_reach"):
            assert pi[k] == fi[k], (step, k)
        allowed = _compare(wl, snap, full, q, roots)
        orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
        np.testing.assert_array_equal(allowed, dec)
        full.close()
        prev.close()
    # the patch is not a no-op: answers moved since the first version
    base = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    a0, _ = km.CheckEngine(base, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    assert (a0 != allowed).any()
    st.close()


def test_patch_falls_back_when_base_has_no_node():
    """a transaction creating more objects than the base snapshot kept spare entities for (half
    the graph at once) cannot be patched in: the full build runs (patched = False) and the result
    is still the store's content; a snapshot of another store is never patched"""
    wl = synth.drive(depth=4, n_groups=300, n_users=1000, seed=5)
    st = km.TupleStore(wl.tuples[: len(wl.tuples) // 2])
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    rest = wl.tuples[len(wl.tuples) // 2:]
    st.transact(rest, None)
    nxt = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=snap)
    assert not nxt.patched
    full = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    q = synth.drive_queries(wl, 4096, seed=2)
    rng = np.random.default_rng(0)
    _compare(wl, nxt, full, q, _roots(wl, rng, 64))
    other = km.TupleStore(wl.tuples)
    o2 = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=other, base=nxt)
    assert not o2.patched
    st.close()
    other.close()


def _first_edges(rows):
    """a row's tuples in shard order (traverser.go:88)"""
    key = [bytes(r) for r in rows["shard_id"]]
    return rows[np.argsort(np.array(key, dtype=object), kind="stable")]


def test_patch_two_sibling_leaf_flips_under_one_parent():
    """one transaction gives two leaf child groups -- the first two edges of an
    untouched parent's row, i.e. both of its inline edge copies -- their first nested group.
    Both flips rewrite the parent's inline words; the patched snapshot must still equal the full
    build (EDGE_LEAF read through set_row .z/.w for rows of <= 2 edges) and the oracle"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    t = wl.tuples
    g_ns, mem = wl.ns_names.index("Group"), wl.rel_names.index("members")
    nested = t[(t["ns"] == g_ns) & (t["rel"] == mem) & (t["subj_kind"] == 1)]
    has_rows = set(nested["obj"].tolist())
    parent, kids = None, None
    for p in np.unique(nested["obj"]):
        row = _first_edges(nested[nested["obj"] == p])
        if len(row) >= 2 and row["s_obj"][0] not in has_rows and row["s_obj"][1] not in has_rows \
                and row["s_obj"][0] != row["s_obj"][1]:
            parent, kids = int(p), [int(row["s_obj"][0]), int(row["s_obj"][1])]
            break
    assert parent is not None, "no parent with two leaf children first in shard order"
    st = km.TupleStore(t)
    host = t.copy()
    base = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    donor = int(nested["obj"][0])  # a group that has members of its own
    ins = np.zeros(2, dtype=t.dtype)
    ins["ns"], ins["obj"], ins["rel"] = g_ns, kids, mem
    ins["subj_kind"], ins["s_ns"], ins["s_obj"], ins["s_rel"] = 1, g_ns, donor, mem
    ins["shard_id"] = np.random.default_rng(1).integers(0, 256, (2, 16), dtype=np.uint8)
    st.transact(ins, None)
    host = transact(host, ins, ins[:0])
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=base)
    assert snap.patched
    full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    rng = np.random.default_rng(5)
    q = synth.drive_queries(wl, 4096, seed=3)
    # the parent's membership of every member of the donor group: through a flipped child only
    members = t[(t["ns"] == g_ns) & (t["obj"] == donor) & (t["rel"] == mem) & (t["subj_kind"] == 0)]
    k = min(len(members), 256)
    q["ns"][:k], q["obj"][:k], q["rel"][:k] = g_ns, parent, mem
    q["subj_kind"][:k], q["s_obj"][:k], q["s_ns"][:k], q["s_rel"][:k] = 0, members["s_obj"][:k], 0, 0
    q["max_depth"][:k] = 0
    roots = _roots(wl, rng, 64)
    roots["ns"][0], roots["obj"][0], roots["rel"][0] = g_ns, parent, mem
    allowed = _compare(wl, snap, full, q, roots)
    assert allowed[:k].any()
    w, _ = world_from_workload(wl)
    orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, _, _ = orc.check_batch(queries_to_oracle(q), threads=8)
    np.testing.assert_array_equal(allowed, dec)
    st.close()


def test_patch_with_changed_namespace_config_builds_in_full():
    """a patch reuses its base's compiled rewrites only for the same configuration.
    After a namespace reload (here: File/Folder `view` becomes `!banned` alone) the call builds in full
    (patched = False) and answers with the new rewrites; with the new configuration on both sides
    the next patch runs again"""
    import copy
    wl = synth.drive(depth=4, n_groups=300, n_users=1000, seed=5)
    st = km.TupleStore(wl.tuples)
    base = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    ns2 = copy.deepcopy(wl.namespaces)
    for name in ("File", "Folder"):
        for r in ns2[name]:
            if r["name"] == "view" and r["rewrite"]["operator"] == "and":  # (File and Folder share one list)
                r["rewrite"] = {"operator": "or", "children": [r["rewrite"]["children"][1]]}  # {!banned}
    ins = wl.tuples[:1].copy()
    ins["shard_id"][:, 0] ^= 0x5A
    st.transact(ins, None)
    nxt = km.Snapshot(ns2, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=base)
    assert not nxt.patched
    full = km.Snapshot(ns2, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 4096, seed=2)
    a_new = _compare(wl, nxt, full, q, _roots(wl, np.random.default_rng(0), 64))
    a_old, _ = km.CheckEngine(base, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    assert (a_new != a_old).any()  # non-viewers are allowed now: the old rewrites were not kept
    st.transact(ins, None)
    again = km.Snapshot(ns2, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=nxt)
    assert again.patched
    st.close()


def test_patch_creates_objects():
    """verdict r3: the reference's insert creates rows for any object (persistence/sql/
    relationtuples.go:104-126, 277-287).  A transaction of 1,000 rows creating 100 new files (a
    parent tuple + 9 ACL rows each, ids past the base's) is patched in -- the new objects go on
    the base's spare entities -- and then a second one creating a new folder and files under it
    (a new subject-set object): every Check (goal counts too) and Expand tree equals a full build
    of the same version, and the oracle agrees; the new files' answers are not the phantom's"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    rng = np.random.default_rng(11)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    base = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    w, _ = world_from_workload(wl)
    folders = rng.integers(0, wl.meta["n_folders"], 100)
    n_uuids = wl.n_uuids
    new_ids = n_uuids + np.arange(100)
    ins = synth.drive_new_files(wl, new_ids, folders, rng)
    assert len(ins) == 1000
    snaps = [base]
    for step in range(2):
        if step == 1:  # a new folder (under an existing one) and 20 files in it
            fo_ns = wl.ns_names.index("Folder")
            new_folder = n_uuids
            files = n_uuids + 1 + np.arange(20)
            ins = synth.drive_new_files(wl, files, np.full(20, new_folder), rng)
            up = ins[:1].copy()
            up["ns"], up["obj"], up["s_obj"] = fo_ns, new_folder, int(folders[0])
            ins = np.concatenate([up, ins])
            new_ids = np.concatenate([[new_folder], files])
        n_uuids = int(new_ids.max()) + 1
        st.transact(ins, None)
        host = transact(host, ins, ins[:0])
        snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, n_uuids, store=st, base=snaps[-1])
        assert snap.patched, f"step {step}: the full build ran"
        full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, n_uuids, store=st)
        q = synth.drive_queries(wl, 8192, seed=20 + step)
        k = 4096  # view / edit of the new objects for random users (ids past the workload's included)
        f_ns = wl.ns_names.index("File") if step == 0 else np.where(np.arange(k) % 21 == 0, wl.ns_names.index("Folder"),
                                                                        wl.ns_names.index("File"))
        q["ns"][:k] = f_ns
        q["obj"][:k] = rng.choice(new_ids, k)
        q["rel"][:k] = rng.choice([wl.rel_names.index("view"), wl.rel_names.index("edit")], k)
        q["subj_kind"][:k], q["s_ns"][:k], q["s_rel"][:k] = 0, 0, 0
        q["s_obj"][:k] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], k)
        q["max_depth"][:k] = 0
        roots = _roots(wl, rng, 64)
        roots["ns"][:32], roots["obj"][:32] = wl.ns_names.index("File"), rng.choice(new_ids, 32)
        roots["rel"][:32] = wl.rel_names.index("viewers")
        allowed = _compare(wl, snap, full, q, roots)
        assert allowed[:k].any()  # the new files are found, not the phantom
        orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
        np.testing.assert_array_equal(allowed, dec)
        full.close()
        snaps.append(snap)
    st.close()


def test_advanced_snapshots_equal_full_builds():
    """keto_store_snapshot_advance: the same chain of transactions as the patch test -- ACL rows in
    and out, duplicates, nested-group edges in and out (leaf flags), subjects crossing the heavy
    threshold -- applied to ONE store snapshot in place, rows moved into its slack: after each,
    every Check (depth truncation included), goal count and Expand tree equals a full build of the
    same store version, and the oracle over the host-side transaction result agrees"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    rng = np.random.default_rng(3)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 20_000, seed=6)
    q["max_depth"][:500] = rng.integers(1, 5, 500)
    roots = _roots(wl, rng)
    w, _ = world_from_workload(wl)
    for step in range(4):
        ins, dele = _delta(wl, rng, 1500, 1000) if step % 2 == 0 else _edge_delta(wl, rng, host)
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        if step == 2:  # two transactions behind: both applied in one advance, in order
            ins2, dele2 = _delta(wl, rng, 200, 100)
            st.transact(ins2, dele2)
            host = transact(host, ins2, dele2)
        assert snap.advance(st), f"step {step}: declined"
        full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
        pi, fi = snap.info(), full.info()
        for k in ("n_tuples", "n_set_edges", "version", "n_reach"):
            assert pi[k] == fi[k], (step, k)
        allowed = _compare(wl, snap, full, q, roots)
        orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
        np.testing.assert_array_equal(allowed, dec)
        full.close()
    assert snap.advance(st)  # (already at the store's version: nothing to do)
    base = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    a0, _ = km.CheckEngine(base, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    assert (a0 != allowed).any()
    st.close()


def test_advance_creates_objects():
    """the new-file transactions of test_patch_creates_objects (100 new files, then a new folder
    with 20 files under it) advanced into one store snapshot in place: new objects on spare
    entities, every answer, goal count and Expand tree equal to a full build, oracle agreeing"""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    rng = np.random.default_rng(11)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    w, _ = world_from_workload(wl)
    folders = rng.integers(0, wl.meta["n_folders"], 100)
    n_uuids = wl.n_uuids
    new_ids = n_uuids + np.arange(100)
    ins = synth.drive_new_files(wl, new_ids, folders, rng)
    for step in range(2):
        if step == 1:
            fo_ns = wl.ns_names.index("Folder")
            new_folder = n_uuids
            files = n_uuids + 1 + np.arange(20)
            ins = synth.drive_new_files(wl, files, np.full(20, new_folder), rng)
            up = ins[:1].copy()
            up["ns"], up["obj"], up["s_obj"] = fo_ns, new_folder, int(folders[0])
            ins = np.concatenate([up, ins])
            new_ids = np.concatenate([[new_folder], files])
        n_uuids = int(new_ids.max()) + 1
        st.transact(ins, None)
        host = transact(host, ins, ins[:0])
        assert snap.advance(st), f"step {step}: declined"
        full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, n_uuids, store=st)
        q = synth.drive_queries(wl, 8192, seed=20 + step)
        k = 4096
        q["ns"][:k] = wl.ns_names.index("File") if step == 0 else np.where(np.arange(k) % 21 == 0, wl.ns_names.index("Folder"),
                                                                              wl.ns_names.index("File"))
        q["obj"][:k] = rng.choice(new_ids, k)
        q["rel"][:k] = rng.choice([wl.rel_names.index("view"), wl.rel_names.index("edit")], k)
        q["subj_kind"][:k], q["s_ns"][:k], q["s_rel"][:k] = 0, 0, 0
        q["s_obj"][:k] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], k)
        q["max_depth"][:k] = 0
        roots = _roots(wl, rng, 64)
        roots["ns"][:32], roots["obj"][:32] = wl.ns_names.index("File"), rng.choice(new_ids, 32)
        roots["rel"][:32] = wl.rel_names.index("viewers")
        allowed = _compare(wl, snap, full, q, roots)
        assert allowed[:k].any()
        orc = refsem.Oracle(w, host.view(refsem.TUPLE_DT).copy(), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
        np.testing.assert_array_equal(allowed, dec)
        full.close()
    st.close()


def test_advance_failure_after_first_write_breaks_the_snapshot(tmp_path, monkeypatch):
    """An in-place advance that fails after its first write (KETO_FAULT_ADVANCE injects a failure
    right after the first rows are written) leaves the snapshot half-advanced: the library marks it
    broken and refuses every later Check, Expand, advance, copy patch, save and dispatcher on it,
    while a fresh cut of the same store serves the new version (patch.hip)"""
    wl = synth.drive(depth=4, n_groups=500, n_users=1000, seed=4)
    t = wl.tuples
    st = km.TupleStore(t)
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 2048, seed=2)
    ins = t[5:6].copy()
    ins["subj_kind"], ins["s_obj"], ins["s_ns"], ins["s_rel"] = 0, wl.meta["ubase"] + 9, 0, 0
    ins["shard_id"] = np.random.default_rng(2).integers(0, 256, (1, 16), dtype=np.uint8)
    st.transact(ins, None)
    monkeypatch.setenv("KETO_FAULT_ADVANCE", "1")
    with pytest.raises(Exception, match="injected fault"):
        snap.advance(st)
    monkeypatch.delenv("KETO_FAULT_ADVANCE")
    eng = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    for call in (lambda: eng.check_batch(q), lambda: snap.advance(st), lambda: snap.save(str(tmp_path / "b.snap")),
                 lambda: km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=snap)):
        with pytest.raises(Exception, match="unusable"):
            call()
    fresh = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    full = km.Snapshot(wl.namespaces, transact(t, ins, ins[:0]), wl.ns_names, wl.rel_names, wl.n_uuids)
    a = km.CheckEngine(fresh, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    b = km.CheckEngine(full, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    for s in (snap, fresh, full):
        s.close()
    st.close()


def test_advance_declines_and_leaves_the_snapshot(tmp_path):
    """what the advance cannot do it declines before writing anything: an insert whose shard_id's
    high half ties a tuple of its row (only the full build orders it), a snapshot that is not this
    store's; a declined snapshot still answers its own version.  An advanced snapshot is neither
    saved nor the base of a copy patch (that builds in full)."""
    wl = synth.drive(depth=4, n_groups=500, n_users=1000, seed=4)
    t = wl.tuples
    st = km.TupleStore(t)
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 4096, seed=2)
    before = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    tie = t[:1].copy()  # the same row, another subject, a shard_id equal in its high half
    tie["subj_kind"], tie["s_obj"], tie["s_ns"], tie["s_rel"] = 0, wl.meta["ubase"] + 3, 0, 0
    tie["shard_id"][0, 8:] ^= 0x5A
    st.transact(tie, None)
    assert not snap.advance(st)
    assert snap.info()["version"] == 0
    after = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    np.testing.assert_array_equal(before[0], after[0])
    np.testing.assert_array_equal(before[1], after[1])
    other = km.TupleStore(t)
    assert not snap.advance(other)
    plain = km.Snapshot(wl.namespaces, t, wl.ns_names, wl.rel_names, wl.n_uuids)
    assert not plain.advance(st)
    # a fresh cut advances; then save refuses it and a copy patch of it builds in full
    snap2 = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    snap2.save(str(tmp_path / "fresh.snap"))  # (not advanced yet: saved)
    ins = t[5:6].copy()
    ins["subj_kind"], ins["s_obj"], ins["s_ns"], ins["s_rel"] = 0, wl.meta["ubase"] + 9, 0, 0
    ins["shard_id"] = np.random.default_rng(2).integers(0, 256, (1, 16), dtype=np.uint8)
    st.transact(ins, None)
    assert snap2.advance(st)
    with pytest.raises(Exception):
        snap2.save(str(tmp_path / "advanced.snap"))
    st.transact(None, ins)
    nxt = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st, base=snap2)
    assert not nxt.patched
    for s in (snap, snap2, nxt, plain):
        s.close()
    other.close()
    st.close()


def test_store_index_churn_and_mass_delete():
    """the store's content index (store.hip): 90 transactions of inserts and deletes on a small
    store fill the index with tombstones past its load bound (re-indexed on the way), and one
    delete key matching 3,001 duplicate rows overflows the first dead list (re-indexed, run again);
    the store's content stays the host restatement's -- the same count, and a snapshot of it equal
    to a full build of the host rows in every Check answer and Expand tree (rows in shard order:
    the duplicates' shard_ids included)"""
    wl = synth.drive(depth=3, n_groups=100, n_users=300, seed=2)
    rng = np.random.default_rng(9)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    for step in range(90):
        ins = host[rng.choice(len(host), 1000)].copy()
        acl = rng.random(len(ins)) < 0.8  # mostly new keys (other users), the rest duplicates of stored rows
        ins["subj_kind"][acl], ins["s_ns"][acl], ins["s_rel"][acl] = 0, 0, 0
        ins["s_obj"][acl] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], int(acl.sum()))
        ins["shard_id"] = rng.integers(0, 256, (len(ins), 16), dtype=np.uint8)
        dele = host[rng.choice(len(host), min(700, len(host) // 2), replace=False)].copy()
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        assert st.info()[0] == len(host), step
    dup = np.repeat(host[:1], 3001)
    dup["shard_id"] = rng.integers(0, 256, (len(dup), 16), dtype=np.uint8)
    st.transact(dup, None)
    host = transact(host, dup, dup[:0])
    extra = host[5:9].copy()
    extra["shard_id"] = rng.integers(0, 256, (len(extra), 16), dtype=np.uint8)
    st.transact(extra, host[:1])  # one key: 3,002 rows
    host = transact(host, extra, host[:1])
    assert st.info()[0] == len(host)
    inc = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    full = km.Snapshot(wl.namespaces, host, wl.ns_names, wl.rel_names, wl.n_uuids)
    q = synth.drive_queries(wl, 4096, seed=5)
    roots = np.zeros(len(host), dtype=km.SUBJSET_DT)
    roots["ns"], roots["obj"], roots["rel"] = host["ns"], host["obj"], host["rel"]
    roots = np.unique(roots)[:512]
    out = []
    for snap in (inc, full):
        a, e = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
        nodes, offs, xerr = km.ExpandEngine(snap, max_read_depth=wl.max_depth).build_trees(roots)
        out.append((a, e, nodes.tobytes(), offs, xerr))
    for x, y in zip(*out):
        np.testing.assert_array_equal(x, y)
    inc.close()
    full.close()
    st.close()


@pytest.mark.parametrize("room", [{"KETO_ADVANCE_SLACK": "6000"}, {"KETO_ADVANCE_RELOC": "3000"}])
def test_advance_declines_once_its_room_is_spent(room, monkeypatch):
    """a store snapshot's room -- slack past its rows, relocation entries -- is finite: transactions
    advance it until one would not fit, which declines and leaves it at its version (every answer
    still the previous version's); a fresh cut then carries on.  (Room shrunk by the env knobs.)"""
    for k, v in room.items():
        monkeypatch.setenv(k, v)
    wl = synth.drive(depth=4, n_groups=500, n_users=1000, seed=4)
    rng = np.random.default_rng(6)
    st = km.TupleStore(wl.tuples)
    host = wl.tuples.copy()
    snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    q = synth.drive_queries(wl, 4096, seed=8)
    advanced = 0
    for step in range(40):
        ins, dele = _delta(wl, rng, 600, 300)
        prev = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
        version = snap.info()["version"]
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        if not snap.advance(st):
            assert snap.info()["version"] == version
            now = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
            np.testing.assert_array_equal(prev[0], now[0])
            np.testing.assert_array_equal(prev[1], now[1])
            break
        advanced += 1
    else:
        pytest.fail("the room never ran out")
    assert advanced >= 1
    snap.close()
    monkeypatch.delenv(next(iter(room)))
    fresh = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st)
    ins, dele = _delta(wl, rng, 600, 300)
    st.transact(ins, dele)
    host = transact(host, ins, dele)
    assert fresh.advance(st)
    full = km.Snapshot(wl.namespaces, host, wl.ns_names, wl.rel_names, wl.n_uuids)
    a = km.CheckEngine(fresh, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    b = km.CheckEngine(full, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    fresh.close()
    full.close()
    st.close()
