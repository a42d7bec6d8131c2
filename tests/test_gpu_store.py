"""Incremental snapshots (keto_store_*): TransactRelationTuples deltas applied on the device
give exactly the snapshot a full rebuild from the host-side transaction result gives, and
the oracle agrees on it; versions count transactions; a dispatcher picks the new snapshot
up between batches."""
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
