"""GPU parity: the HIP engine (through the C ABI) against the reference's known answers
and against the oracle on the same seeded inputs.  Integer/boolean work: bit-exact."""
import os

import numpy as np
import pytest

import keto_mi355x as km
import refsem
from fixtures import fixture_names, load, world_for
from product_helpers import (product_snapshot, product_tree_to_nested, queries_to_oracle, queries_to_product,
                             world_from_workload)
from randworld import random_world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stream():
    s = km.Stream(0)
    yield s
    s.close()


def _oracle_decisions(orc, q, max_depth, max_width):
    orc.set_limits(max_depth, max_width)
    mem, err, st = orc.check(q)
    return ((err == 0) & (mem == refsem.IS_MEMBER)).astype(np.uint8), err, st


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("checks")])
def test_golden_checks(stream, name):
    fx = load(name)
    w, t, q = world_for(fx)
    snap = product_snapshot(w, t)
    for i, c in enumerate(fx["checks"]):
        eng = km.CheckEngine(snap, stream, max_read_depth=c.get("global", fx.get("global", 5)),
                             max_read_width=fx.get("max_width", 100))
        allowed, err = eng.check_batch(queries_to_product(q[i:i + 1]))
        assert int(err[0]) == c.get("err", 0), (name, c)
        assert bool(allowed[0]) == c["allowed"], (name, c)


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("expands")])
def test_golden_expands(stream, name):
    fx = load(name)
    w, t, _ = world_for(fx)
    snap = product_snapshot(w, t)
    eng = km.ExpandEngine(snap, stream, max_read_depth=fx.get("global", 5))
    cases = [e for e in fx["expands"] if "subject" in e]
    roots = np.zeros(len(cases), dtype=km.SUBJSET_DT)
    for i, e in enumerate(cases):
        ns, obj, rel = refsem.parse_subject_set(e["subject"])
        roots[i] = (w.ns_names.ids[ns], w.uuids.ids[obj], w.rel_names.ids[rel], e["depth"])
    nodes, offs, err = eng.build_trees(roots)
    assert (err == 0).all()
    for i, e in enumerate(cases):
        got = product_tree_to_nested(w, nodes[int(offs[i]):int(offs[i + 1])])
        if e.get("exact"):
            assert got == e["tree"], (name, e["src"])
        assert refsem.trees_equal_unordered(got, e["tree"]), (name, e["src"], got)


@pytest.mark.parametrize("rewrites", [True, False])
@pytest.mark.parametrize("seed", list(range(60)))
def test_random_worlds_vs_oracle(stream, seed, rewrites):
    w, t, q, expands = random_world(seed, rewrites=rewrites)
    orc = refsem.Oracle(w, t)
    snap = product_snapshot(w, t)
    dec, err, st = _oracle_decisions(orc, q, w.max_depth, w.max_width)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    stream.counters(reset=True)
    allowed, gerr = eng.check_batch(queries_to_product(q), count_work=True)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    c = stream.counters(reset=True)
    if (err == 0).all():  # work counters of completed queries: identical traversal
        assert (c["rows"], c["edges"], c["probes"]) == (st.rows, st.edges, st.probes)
    # expand trees: exact, including child order
    xe = km.ExpandEngine(snap, stream, max_read_depth=w.max_depth)
    roots = np.array([(w.ns_names.ids[a], w.uuids.ids[b], w.rel_names.ids[r], d) for a, b, r, d in expands],
                     dtype=km.SUBJSET_DT)
    nodes, offs, xerr = xe.build_trees(roots)
    assert (xerr == 0).all()
    orc.set_limits(w.max_depth, w.max_width)
    for i, (a, b, r, d) in enumerate(expands):
        on, _ = orc.expand(1, w.uuids.ids[b], w.ns_names.ids[a], w.rel_names.ids[r], d)
        assert product_tree_to_nested(w, nodes[int(offs[i]):int(offs[i + 1])]) == refsem.tree_to_nested(w, on)


@pytest.mark.parametrize("wl_name", ["nested_groups", "drive"])
def test_synthetic_small_vs_oracle(stream, wl_name):
    from keto_mi355x import synth
    if wl_name == "nested_groups":
        wl = synth.nested_groups(200_000, seed=5)
        q = synth.nested_groups_queries(wl, 20_000, seed=9, trunc_frac=0.05)
    else:
        wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=4)
        q = synth.drive_queries(wl, 20_000, seed=3)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    dec, err, st = orc.check_batch(queries_to_oracle(q), threads=8)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    stream.counters(reset=True)
    allowed, gerr = eng.check_batch(q, count_work=True)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    c = stream.counters(reset=True)
    assert (c["rows"], c["edges"], c["probes"]) == (st.rows, st.edges, st.probes)
    assert 0.05 < allowed.mean() < 0.95


def test_nested_groups_full_size_properties(stream):
    """BASELINE config 2 at full size (10M tuples): size-independent properties."""
    from keto_mi355x import synth
    wl = synth.nested_groups(10_000_000, seed=1)
    q = synth.nested_groups_queries(wl, 1 << 20, seed=7)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth)
    a1, e1 = eng.check_batch(q)
    assert (e1 == 0).all()
    # determinism and batch-split invariance (queries are independent units)
    a2, _ = eng.check_batch(q)
    np.testing.assert_array_equal(a1, a2)
    h = len(q) // 3
    parts = [eng.check_batch(q[i:j])[0] for i, j in ((0, h), (h, 2 * h), (2 * h, len(q)))]
    np.testing.assert_array_equal(np.concatenate(parts), a1)
    # random-walk positives at full request depth are members (union-only, no truncation)
    rng = np.random.Generator(np.random.PCG64(7))
    # regenerate which queries were positives: they are the ones whose subject is a real member
    full = q["max_depth"] == 0
    assert a1[full].mean() > 0.45
    # a sample of 4096 checked exactly against the oracle
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    idx = rng.choice(len(q), size=4096, replace=False)
    dec, err, _ = orc.check_batch(queries_to_oracle(q[idx]), threads=8)
    np.testing.assert_array_equal(a1[idx], dec)


def test_device_pointer_path(stream):
    w, t, q, _ = random_world(3)
    snap = product_snapshot(w, t)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    host_a, host_e = eng.check_batch(queries_to_product(q))
    pq = queries_to_product(q)
    dq = km.DeviceBuffer(0, pq.nbytes)
    da = km.DeviceBuffer(0, len(pq))
    de = km.DeviceBuffer(0, 4 * len(pq))
    dq.upload(stream, pq)
    eng.check_batch_device(dq, len(pq), da, de, sync=False)
    stream.sync()
    a = da.download(stream, np.zeros(len(pq), np.uint8))
    e = de.download(stream, np.zeros(len(pq), np.int32))
    np.testing.assert_array_equal(a, host_a)
    np.testing.assert_array_equal(e, host_e)
    assert stream.last_kernel_ms() > 0


def test_scratch_tiers(stream):
    """A query whose visited set (200 subgroups) and stack (deep chain) outgrow tier 1."""
    ns = {"g": []}
    tuples = [f"g:root#m@g:s{i}#m" for i in range(300)] + [f"g:s{i}#m@g:t{i}#m" for i in range(300)]
    tuples += [f"g:c{i}#m@g:c{i + 1}#m" for i in range(120)] + ["g:c120#m@deep_user", "g:t299#m@wide_user"]
    w = refsem.World(namespaces=ns, max_depth=200, max_width=1000)
    t = w.tuple_array(tuples)
    q = w.query_array([("g:root#m@wide_user", 0), ("g:root#m@nobody", 0), ("g:c0#m@deep_user", 0),
                       ("g:c0#m@nobody", 0), ("g:c0#m@deep_user", 50)])
    orc = refsem.Oracle(w, t)
    dec, err, _ = _oracle_decisions(orc, q, 200, 1000)
    snap = product_snapshot(w, t)
    eng = km.CheckEngine(snap, stream, max_read_depth=200, max_read_width=1000)
    a, e = eng.check_batch(queries_to_product(q))
    np.testing.assert_array_equal(e, err)
    np.testing.assert_array_equal(a, dec)
    assert list(dec) == [1, 0, 1, 0, 0]


def test_build_tree_single_root_matches_batch(stream):
    fx = load("expand_engine")
    w, t, _ = world_for(fx)
    snap = product_snapshot(w, t)
    eng = km.ExpandEngine(snap, stream, max_read_depth=fx.get("global", 5))
    for e in [e for e in fx["expands"] if "subject" in e]:
        ns, obj, rel = refsem.parse_subject_set(e["subject"])
        got = eng.build_tree(w.ns_names.ids[ns], w.uuids.ids[obj], w.rel_names.ids[rel], e["depth"])
        if e["tree"] is None:
            assert got is None
        else:
            assert refsem.trees_equal_unordered(product_tree_to_nested(w, got), e["tree"])


def test_fresh_stream_device_path_first_call():
    """Regression: a new stream's first batch on the device-pointer path, right after a
    snapshot build freed large temporaries (scratch zero-fill must finish before the
    interpreter reads its epochs / visited slots)."""
    from keto_mi355x import synth
    wl = synth.drive(depth=7, n_groups=20_000, n_users=200_000, seed=6)
    q = synth.drive_queries(wl, 1 << 16, seed=5)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    s = km.Stream(0)
    eng = km.CheckEngine(snap, s, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
    dq.upload(s, q)
    eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
    allowed = da.download(s, np.zeros(len(q), np.uint8))
    w, _ = world_from_workload(wl)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)  # engine layout, in place
    dec, err, _ = orc.check_batch(q.view(refsem.QUERY_DT), threads=8)
    np.testing.assert_array_equal(allowed, dec)
    s.close()


def test_small_batch_spreading_is_exact(stream):
    """Batches smaller than the resident grid run with fewer live lanes per wave (down to one):
    every batch size gives the same decisions, equal to the oracle's."""
    from keto_mi355x import synth
    wl = synth.drive(depth=6, n_groups=5000, n_users=20000, seed=11)
    q = synth.drive_queries(wl, 1 << 16, seed=4)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    whole, werr = eng.check_batch(q)
    cuts = [0, 1, 18, 1018, 21018, len(q)]
    parts = [eng.check_batch(q[i:j]) for i, j in zip(cuts[:-1], cuts[1:])]
    np.testing.assert_array_equal(np.concatenate([a for a, _ in parts]), whole)
    np.testing.assert_array_equal(np.concatenate([e for _, e in parts]), werr)
    big, _ = eng.check_batch(np.concatenate([q] * 8))  # full grid, 64 live lanes
    np.testing.assert_array_equal(big, np.tile(whole, 8))
    w, _ = world_from_workload(wl)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    dec, err, _ = orc.check_batch(q.view(refsem.QUERY_DT), threads=8)
    np.testing.assert_array_equal(whole, dec)
    np.testing.assert_array_equal(werr, err)
    assert 0.05 < whole.mean() < 0.95


def test_device_tuple_build_matches_host_build(stream):
    """keto_snapshot_build_device (tuples already in HBM, e.g. received over RCCL) builds the
    same snapshot as the host-pointer build: identical decisions and work counters."""
    from keto_mi355x import synth
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=8)
    q = synth.drive_queries(wl, 8192, seed=2)
    host = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    buf = km.DeviceBuffer(0, wl.tuples.nbytes)
    buf.upload(stream, wl.tuples)
    dev = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids,
                      device_tuples=(buf.ptr, len(wl.tuples)))
    buf.free()
    res = []
    for snap in (host, dev):
        eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
        stream.counters(reset=True)
        a, e = eng.check_batch(q, count_work=True)
        c = stream.counters(reset=True)
        res.append((a, e, (c["rows"], c["edges"], c["probes"])))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]
    assert host.info()["n_set_edges"] == dev.info()["n_set_edges"]


def test_expand_api_form_matches_docs_output(stream):
    """GPU Expand -> keto_trees_to_json: the docs sample's printed tree
    (01-expand-beach/expected_output.json), children compared without order."""
    import json
    import os

    from fixtures import GOLDEN
    from keto_mi355x import api
    from test_tree_api import _canon

    fx = load("docs_expand_beach")
    w, t, _ = world_for(fx)
    snap = product_snapshot(w, t)
    e = fx["expands"][0]
    ns, obj, rel = refsem.parse_subject_set(e["subject"])
    roots = np.array([(w.ns_names.ids[ns], w.uuids.ids[obj], w.rel_names.ids[rel], e["depth"])], dtype=km.SUBJSET_DT)
    nodes, offs, err = km.ExpandEngine(snap, stream, max_read_depth=w.max_depth).build_trees(roots)
    assert err[0] == 0
    out = api.trees_to_json(nodes, offs, api.NameTables(w.ns_names.names, w.rel_names.names, w.uuids.names))
    with open(os.path.join(GOLDEN, "api", "docs_expand_beach_expected_output.json")) as f:
        assert _canon(json.loads(out[0])) == _canon(json.load(f))


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("checks")])
def test_sqlite_loaded_snapshot_on_gpu(stream, tmp_path, name):
    """Keto SQLite store -> loader -> device snapshot -> Check kernels: the reference's own
    expected answers (tests/golden)."""
    import os

    from keto_mi355x.loader import KetoStore
    from keto_sqlite import subject_of, write_store

    fx = load(name)
    path = os.path.join(tmp_path, "keto.sqlite")
    write_store(path, fx["tuples"], seed=len(name))
    store = KetoStore(path, fx["namespaces"], strict=fx.get("strict", False))
    snap = store.snapshot()
    for c in fx["checks"]:
        t = refsem.parse_tuple(c["query"])
        q = store.query(t["ns"], t["obj"], t["rel"], subject_of(t), c.get("depth", 0))
        eng = km.CheckEngine(snap, stream, max_read_depth=c.get("global", fx.get("global", 5)),
                             max_read_width=fx.get("max_width", 100))
        allowed, err = eng.check_batch(q)
        assert err[0] == c.get("err", 0), (name, c)
        assert bool(allowed[0]) == c["allowed"], (name, c)


def test_sqlite_to_api_tree_on_gpu(stream, tmp_path):
    """the whole (f) path: Keto SQLite store -> device snapshot -> Expand kernel -> API JSON,
    against the docs sample's printed tree"""
    import json
    import os

    from fixtures import GOLDEN
    from keto_mi355x import api
    from keto_mi355x.loader import KetoStore
    from keto_sqlite import write_store
    from test_tree_api import _canon

    fx = load("docs_expand_beach")
    path = os.path.join(tmp_path, "keto.sqlite")
    write_store(path, fx["tuples"], seed=3)
    store = KetoStore(path, fx["namespaces"])
    q = store.query("files", "/photos/beach.jpg", "access", "x")[0]
    roots = np.array([(q["ns"], q["obj"], q["rel"], 3)], dtype=km.SUBJSET_DT)
    nodes, offs, err = km.ExpandEngine(store.snapshot(), stream, max_read_depth=5).build_trees(roots)
    assert err[0] == 0
    out = api.trees_to_json(nodes, offs, store.name_tables())
    with open(os.path.join(GOLDEN, "api", "docs_expand_beach_expected_output.json")) as f:
        assert _canon(json.loads(out[0])) == _canon(json.load(f))


def test_relation_error_detail_and_out_of_range_ids(stream):
    """`relation %q does not exist` (namespace/definitions.go:61) names the relation the walk
    rejected -- here one reached through a subject set, not the query's own -- and relation ids
    outside the snapshot's name table resolve like any undeclared relation (configured
    namespace: the error; legacy namespace: nil, not a member) instead of reading past a table."""
    ns = {"doc": [{"name": "viewer", "types": [{"namespace": "grp", "relation": "member"}]}],
          "grp": [{"name": "member", "types": [{"namespace": "user"}]}], "user": []}
    w = refsem.World(namespaces=ns)
    t = w.tuple_array(["doc:d#viewer@(grp:g#nope)", "grp:h#member@alice", "doc:e#viewer@(grp:h#member)"])
    q = w.query_array(["doc:d#viewer@alice", "doc:d#bogus@alice", "doc:e#viewer@alice", "user:u#x@alice"])
    snap = product_snapshot(w, t)
    eng = km.CheckEngine(snap, stream, max_read_depth=5)
    pq = queries_to_product(q)
    a, e = eng.check_batch(pq)
    orc = refsem.Oracle(w, t)
    mem, oerr, _ = orc.check(q)
    np.testing.assert_array_equal(e, oerr)
    assert list(e) == [1, 1, 0, 0] and list(a) == [0, 0, 1, 0]
    a2, e2 = eng.check_batch(pq, err_detail=True)
    np.testing.assert_array_equal(a2, a)
    assert w.rel_names.names[int(e2[0]) >> 8] == "nope"
    assert w.rel_names.names[int(e2[1]) >> 8] == "bogus"
    with pytest.raises(km.KetoError, match='relation "nope" does not exist'):
        eng.check_is_member(pq[0])
    assert eng.check_is_member(pq[2]) is True
    # ids past the name table: 9999 and 70000 (which would alias a real id if truncated to 16 bits)
    bad = pq.copy()
    bad["rel"][0] = 9999
    bad["rel"][1] = 70000 + int(pq["rel"][0])
    bad["rel"][3] = 123456
    a3, e3 = eng.check_batch(bad)
    assert list(e3) == [1, 1, 0, 0] and list(a3) == [0, 0, 1, 0]


@pytest.fixture
def regroup_forced():
    """tier 0 on the block-regrouped interpreter whatever the batch size (check.hip
    check_kernel_rg; by default only batches that fill its resident blocks 4x use it)"""
    import os
    old = os.environ.get("KETO_REGROUP")
    os.environ["KETO_REGROUP"] = "force"
    yield
    if old is None:
        del os.environ["KETO_REGROUP"]
    else:
        os.environ["KETO_REGROUP"] = old


@pytest.mark.parametrize("seed", list(range(0, 60, 3)))
def test_regrouped_interpreter_random_worlds(stream, regroup_forced, seed):
    w, t, q, _ = random_world(seed, rewrites=True)
    orc = refsem.Oracle(w, t)
    snap = product_snapshot(w, t)
    dec, err, st = _oracle_decisions(orc, q, w.max_depth, w.max_width)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    stream.counters(reset=True)
    allowed, gerr = eng.check_batch(queries_to_product(q), count_work=True)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    c = stream.counters(reset=True)
    if (err == 0).all():
        assert (c["rows"], c["edges"], c["probes"]) == (st.rows, st.edges, st.probes)


def test_regrouped_interpreter_drive(stream, regroup_forced):
    from keto_mi355x import synth
    wl = synth.drive(depth=6, n_groups=5000, n_users=20000, seed=11)
    q = synth.drive_queries(wl, 1 << 17, seed=4)
    q["max_depth"][:1000] = np.random.default_rng(0).integers(1, 5, 1000)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    stream.counters(reset=True)
    a, e = eng.check_batch(q, count_work=True)
    c = stream.counters(reset=True)
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, err, st = orc.check_batch(q.view(refsem.QUERY_DT), threads=8)
    np.testing.assert_array_equal(a, dec)
    np.testing.assert_array_equal(e, err)
    assert (c["rows"], c["edges"], c["probes"]) == (st.rows, st.edges, st.probes)
    assert c["per_tier"]["queries"][0] > 0


@pytest.mark.parametrize("output", ["pageable", "pinned"])
@pytest.mark.parametrize("mode", ["wave", "mixed", "lane"])
def test_expand_drive_trees_wave_and_fallback(stream, mode, output):
    """Expand on a Drive world: the wave-per-root kernel (every root), a batch where trees larger
    than a lowered staging capacity fall back to the lane kernel (both paths in one batch, placed
    in root order), and the lane kernel alone -- exact trees, child order included, vs the oracle;
    into pageable output (staged copy) and pinned output (keto_host_alloc: one DMA); 2,400 roots"""
    from keto_mi355x import synth
    wl = synth.drive(depth=5, n_groups=400, members_per_group=6, n_users=3000, seed=13)
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    rng = np.random.default_rng(3)
    n = 2400
    roots = np.zeros(n, dtype=km.SUBJSET_DT)
    h = n // 2
    roots["ns"][:h], roots["rel"][:h] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    roots["obj"][:h] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], h)
    roots["ns"][h:], roots["rel"][h:] = wl.ns_names.index("Folder"), wl.rel_names.index("viewers")
    roots["obj"][h:] = rng.integers(0, wl.meta["folders_per_root"], n - h)
    roots["max_depth"] = rng.integers(0, 8, n)
    env = {"wave": {}, "mixed": {"KETO_XW_PRIV": "12"}, "lane": {"KETO_EXPAND_WAVE": "0"}}[mode]
    old = {k: os.environ.get(k) for k in ("KETO_XW_PRIV", "KETO_EXPAND_WAVE")}
    os.environ.update(env)
    try:
        pin = km.PinnedArray(1 << 19, km.TREE_DT) if output == "pinned" else None
        nodes, offs, err = km.ExpandEngine(snap, stream, max_read_depth=6).build_trees(roots, out=pin)
        if pin is not None:
            assert int(offs[-1]) <= len(pin.array) and nodes.ctypes.data == pin.array.ctypes.data
            nodes = nodes.copy()
        # keto_expand_batch_spans: the same trees in completion order (pinned: written in place
        # by the walks, over PCIe)
        pin2 = km.PinnedArray(1 << 19, km.TREE_DT) if output == "pinned" else None
        sn, first, count, serr = km.ExpandEngine(snap, stream, max_read_depth=6).build_trees_spans(roots, out=pin2)
        np.testing.assert_array_equal(serr, err)
        assert int(count.sum()) == len(sn) == int(offs[-1])
        for i in range(n):
            np.testing.assert_array_equal(sn[int(first[i]):int(first[i]) + int(count[i])], nodes[int(offs[i]):int(offs[i + 1])])
        runs = sorted((int(first[i]), int(count[i])) for i in range(n) if count[i])
        assert all(a + c <= b for (a, c), (b, _) in zip(runs, runs[1:]))  # disjoint runs
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert (err == 0).all()
    big = 0
    for i, r in enumerate(roots):
        d = int(r["max_depth"])
        on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), d if 0 < d <= 6 else 6)
        mine = nodes[int(offs[i]):int(offs[i + 1])]
        assert len(mine) == len(on), i
        big += len(on) > 12
        for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                         ("s_rel", "srel"), ("n_children", "n_children")):
            np.testing.assert_array_equal(mine[f_p], on[f_o])
    assert big > 80  # the mixed batch really sends trees to the fallback


def test_expand_pinned_output_capacity(stream):
    """keto_expand_batch into pinned output one node too small: KETO_E_CAPACITY with the size
    needed in offsets[n] and nothing written (the total is checked before the copy); then the
    exact capacity: the trees equal those of a pageable-output call"""
    import ctypes
    from keto_mi355x import _abi, synth
    wl = synth.drive(depth=4, n_groups=200, members_per_group=5, n_users=1000, seed=5)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    eng = km.ExpandEngine(snap, stream, max_read_depth=5)
    n = 64
    rng = np.random.default_rng(1)
    roots = np.zeros(n, dtype=km.SUBJSET_DT)
    roots["ns"], roots["rel"] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    roots["obj"] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], n)
    ref, ref_offs, ref_err = eng.build_trees(roots)
    total = int(ref_offs[-1])
    assert total > n
    for cap in (total - 1, total):
        pin = km.PinnedArray(cap, km.TREE_DT)
        pin.array.view(np.uint8)[:] = 0xAB
        offs = np.zeros(n + 1, np.uint64)
        err = np.zeros(n, np.int32)
        rc = _abi.lib().keto_expand_batch(snap.handle, stream.handle, roots.ctypes.data, n, ctypes.byref(eng.limits),
                                          pin.array.ctypes.data, cap, offs.ctypes.data, err.ctypes.data)
        np.testing.assert_array_equal(offs, ref_offs)
        if cap < total:
            assert rc == _abi.KETO_E_CAPACITY
            assert (pin.array.view(np.uint8) == 0xAB).all()
        else:
            assert rc == 0
            np.testing.assert_array_equal(err, ref_err)
            assert pin.array.tobytes() == ref.tobytes()
        pin.free()


C1_OBJECTS = ["/cats", "/cats/1.mp4", "/cats/2.mp4"]
C1_RELATIONS = ["owner", "view"]
C1_SUBJECTS = ["cat lady", "*", "nobody"]



def test_expand_spans_capacity(stream):
    """keto_expand_batch_spans one node too small (pinned and pageable output): KETO_E_CAPACITY with
    the nodes needed in *out_total; then the exact capacity: every root's run holds its tree as
    keto_expand_batch gives it"""
    import ctypes
    from keto_mi355x import _abi, synth
    wl = synth.drive(depth=4, n_groups=200, members_per_group=5, n_users=1000, seed=6)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    eng = km.ExpandEngine(snap, stream, max_read_depth=5)
    n = 96
    rng = np.random.default_rng(2)
    roots = np.zeros(n, dtype=km.SUBJSET_DT)
    roots["ns"], roots["rel"] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    roots["obj"] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], n)
    roots["obj"][:8] = 0  # (a few nil or tiny trees)
    ref, ref_offs, ref_err = eng.build_trees(roots)
    total = int(ref_offs[-1])
    assert total > n
    for pinned in (True, False):
        for cap in (total - 1, total):
            pin = km.PinnedArray(cap, km.TREE_DT) if pinned else None
            buf = pin.array if pinned else np.zeros(cap, km.TREE_DT)
            first, count = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
            err, tot = np.zeros(n, np.int32), ctypes.c_uint64(0)
            rc = _abi.lib().keto_expand_batch_spans(snap.handle, stream.handle, roots.ctypes.data, n, ctypes.byref(eng.limits),
                                                    buf.ctypes.data, cap, first.ctypes.data, count.ctypes.data,
                                                    err.ctypes.data, ctypes.byref(tot))
            assert tot.value == total
            if cap < total:
                assert rc == _abi.KETO_E_CAPACITY
            else:
                assert rc == 0
                np.testing.assert_array_equal(err, ref_err)
                for i in range(n):
                    np.testing.assert_array_equal(buf[int(first[i]):int(first[i]) + int(count[i])],
                                                  ref[int(ref_offs[i]):int(ref_offs[i + 1])])
            if pin is not None:
                pin.free()


def c1_queries(n: int = 10_000, seed: int = 42) -> list:
    """BASELINE configs[0] as SURVEY.md 8.1 (d) configures it: n seed-42 uniform draws over the
    18 combinations {/cats, /cats/1.mp4, /cats/2.mp4} x {owner, view} x {cat lady, *, nobody}"""
    combos = [(o, r, s) for o in C1_OBJECTS for r in C1_RELATIONS for s in C1_SUBJECTS]
    pick = np.random.default_rng(seed).integers(0, len(combos), n)
    return [f"videos:{combos[i][0]}#{combos[i][1]}@{combos[i][2]}" for i in pick]


def test_c1_cat_videos_as_configured(stream):
    """configs[0]: the cat-videos example's 7 tuples (contrib/cat-videos-example/relation-tuples/
    *.json, namespace `videos` without relation config, keto.yml), 10,000 seed-42 Checks over all
    18 combinations in one batch: every decision equal to the oracle's, and every combination's
    answer equal to the hand-derived fixture answers where it has one"""
    fx = load("cat_videos")
    w = refsem.World(namespaces=fx["namespaces"], max_depth=5, max_width=100)
    t = w.tuple_array(fx["tuples"])
    strs = c1_queries()
    q = w.query_array([(s, 0) for s in strs])
    assert len(set(strs)) == 18  # every combination is asked
    snap = product_snapshot(w, t)
    allowed, err = km.CheckEngine(snap, stream, max_read_depth=5, max_read_width=100).check_batch(queries_to_product(q))
    orc = refsem.Oracle(w, t)
    dec, oerr, _ = _oracle_decisions(orc, q, 5, 100)
    np.testing.assert_array_equal(err, oerr)
    np.testing.assert_array_equal(allowed, dec)
    known = {c["query"]: c["allowed"] for c in fx["checks"] if c.get("depth", 0) == 0}
    by_combo = {s: bool(a) for s, a in zip(strs, allowed)}
    for s, a in known.items():
        if s in by_combo:
            assert by_combo[s] == a, s
    assert 0 < allowed.mean() < 1
