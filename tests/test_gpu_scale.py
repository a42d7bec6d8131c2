"""BASELINE configs 3, 4 and 5 at their configured sizes on the GPU, through the C ABI.

  C3  Drive-style folder forest, 105M tuples (synth.drive(): fanout 5, depth 10, OPL
      union + intersection + exclusion), max_read_depth 16
  C4  the same graph x10: 1.05B tuples, 889M nodes (synth.drive_scaled(10))
  C5  C4's graph partitioned by object (one rank here): closure exchange -> device
      snapshot -> the unmodified kernels, for Check and for Expand

Each runs a 2^20-query batch whose first 1% asks request depths 1-4 (the truncation
sub-batch: engine.go:82-84 clamps only depths <= 0 or > global, so these really cut the
walk short).  Whole-batch properties (determinism, batch-split invariance) cover all of it;
an exact sample of every truncation query plus 64Ki others is compared with the oracle
(oracle/refsem.c over the whole graph: decision, error code).  Reference for the expected
shape of the answers: the deep-chain benchmarks, internal/check/bench_test.go:104-131.
"""
import sys
import time

import numpy as np
import pytest

import keto_mi355x as km
import refsem
from keto_mi355x import synth
from product_helpers import world_from_workload

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N = 1 << 20
SAMPLE = 1 << 16


def _log(msg):
    print(f"[scale {time.strftime('%H:%M:%S')}] {msg}", file=sys.__stderr__, flush=True)


def _batch(wl, seed):
    q = synth.drive_queries(wl, N, seed=seed)
    rng = np.random.default_rng(seed)
    k = N // 100
    q["max_depth"][:k] = rng.integers(1, 5, k)  # the truncation sub-batch
    return q


def _sample(seed):
    rng = np.random.default_rng(seed + 1)
    rest = rng.choice(np.arange(N // 100, N), size=SAMPLE, replace=False)
    return np.concatenate([np.arange(N // 100), np.sort(rest)])


def _oracle(wl):
    w, _ = world_from_workload(wl, with_tuples=False)
    t0 = time.perf_counter()
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    _log(f"oracle index over {len(wl.tuples)} tuples: {time.perf_counter() - t0:.1f} s")
    return orc


def _check_config(wl, orc, seed):
    """full batch on the replicated snapshot: properties + exact oracle sample"""
    t0 = time.perf_counter()
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    _log(f"snapshot {snap.info()['n_tuples']} tuples: {time.perf_counter() - t0:.1f} s")
    st = km.Stream(0)
    eng = km.CheckEngine(snap, st, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    q = _batch(wl, seed)
    a1, e1 = eng.check_batch(q)
    a2, e2 = eng.check_batch(q)
    np.testing.assert_array_equal(a1, a2)  # determinism
    np.testing.assert_array_equal(e1, e2)
    cuts = [0, 1, N // 100, N // 3, N]  # batch-split invariance (queries are independent units)
    parts = [eng.check_batch(q[i:j]) for i, j in zip(cuts[:-1], cuts[1:])]
    np.testing.assert_array_equal(np.concatenate([a for a, _ in parts]), a1)
    np.testing.assert_array_equal(np.concatenate([e for _, e in parts]), e1)
    assert (e1 == 0).all()
    assert 0.2 < a1.mean() < 0.8
    idx = _sample(seed)
    t0 = time.perf_counter()
    dec, err, _ = orc.check_batch(q[idx].view(refsem.QUERY_DT), threads=16)
    _log(f"oracle sample of {len(idx)}: {time.perf_counter() - t0:.1f} s")
    np.testing.assert_array_equal(e1[idx], err)
    np.testing.assert_array_equal(a1[idx], dec)
    # the truncation sub-batch really truncates: shallower requests allow less
    trunc = a1[: N // 100].mean()
    assert trunc < a1[N // 100:].mean()
    # Expand on the replicated snapshot at full size: 512 roots, every tree exact against the
    # oracle's (internal/expand/engine.go:54-124), child order included
    roots = _roots(wl, 512, seed + 100)
    nodes, offs, xerr = km.ExpandEngine(snap, st, max_read_depth=wl.max_depth).build_trees(roots)
    _check_trees(orc, wl, roots, nodes, offs, xerr)
    st.close()
    snap.close()
    return a1


def _check_trees(orc, wl, roots, nodes, offs, xerr):
    assert (xerr == 0).all()
    n_nodes = 0
    for i, r in enumerate(roots):
        on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), wl.max_depth)
        mine = nodes[int(offs[i]):int(offs[i + 1])]
        assert len(mine) == len(on)
        n_nodes += len(on)
        for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                         ("s_rel", "srel"), ("n_children", "n_children")):
            np.testing.assert_array_equal(mine[f_p], on[f_o])
    assert n_nodes > len(roots)


def test_c3_drive_100m_tuples():
    t0 = time.perf_counter()
    wl = synth.drive()
    assert len(wl.tuples) > 100_000_000
    _log(f"C3 generated {len(wl.tuples)} tuples: {time.perf_counter() - t0:.1f} s")
    orc = _oracle(wl)
    _check_config(wl, orc, seed=21)
    orc.close()


@pytest.fixture(scope="module")
def c4():
    t0 = time.perf_counter()
    wl = synth.drive_scaled(10)
    _log(f"C4 generated {len(wl.tuples)} tuples: {time.perf_counter() - t0:.1f} s")
    orc = _oracle(wl)
    yield wl, orc
    orc.close()


def test_c4_drive_1b_tuples(c4):
    wl, orc = c4
    assert len(wl.tuples) > 1_000_000_000
    _check_config(wl, orc, seed=23)


def _roots(wl, n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, dtype=km.SUBJSET_DT)
    h = n // 2
    r["ns"][:h], r["rel"][:h] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    r["obj"][:h] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], h)
    r["ns"][h:], r["rel"][h:] = wl.ns_names.index("Folder"), wl.rel_names.index("viewers")
    per = wl.meta["nodes_per_root"]
    forest = rng.integers(0, wl.meta["roots"], n - h)
    r["obj"][h:] = forest * per + rng.integers(0, wl.meta["folders_per_root"], n - h)
    return r


def test_c5_partitioned_one_rank(c4, monkeypatch):
    """C5's data path on C4's graph: the partitioned engine (closure exchange, per-batch
    device snapshot, unmodified kernels) on one rank, Check + 256 Expand roots.  (A job of one
    rank runs on a resident snapshot by default; KETO_PART_CLOSURE keeps the closure path, the
    one every rank of a multi-rank job runs.)"""
    from keto_mi355x import partition
    monkeypatch.setenv("KETO_PART_CLOSURE", "1")
    wl, orc = c4
    t0 = time.perf_counter()
    eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, wl.tuples,
                                      max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    _log(f"C5 object store: {time.perf_counter() - t0:.1f} s")
    q = _batch(wl, 25)
    a, e = eng.check_batch(q)
    _log(f"C5 batch: {eng.last}")
    a2, e2 = eng.check_batch(q)  # the second batch reuses the workspace: same answers
    np.testing.assert_array_equal(a, a2)
    _log(f"C5 batch 2: {eng.last}")
    assert 0 < eng.last["tuples"] < len(wl.tuples)
    idx = _sample(25)
    dec, err, _ = orc.check_batch(q[idx].view(refsem.QUERY_DT), threads=16)
    np.testing.assert_array_equal(e[idx], err)
    np.testing.assert_array_equal(a[idx], dec)
    roots = _roots(wl, 256, 26)
    nodes, offs, xerr = eng.expand_batch(roots)
    _check_trees(orc, wl, roots, nodes, offs, xerr)
    eng.close()
