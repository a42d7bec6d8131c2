"""Frontier engine (csrc/frontier.hip) against the oracle.

A check batch on a rewrite snapshot runs breadth-first: one goal per sub-check, evaluated
without visited pruning (oracle/refsem.c "Frontier semantics", rs_check_u), and the queries
whose result could depend on pruning are routed to the DFS interpreter.  The decisions must be
the oracle's canonical ones (rs_check) for every query; the routed count and, where nothing is
routed, the number of goals spawned must equal the oracle's restatement of the engine's rules
(rs_check_u) -- so the spawn rules themselves are pinned, not only the answers."""
import os

import numpy as np
import pytest

import keto_mi355x as km
import refsem
from product_helpers import product_snapshot, queries_to_oracle, queries_to_product, world_from_workload
from randworld import random_world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stream():
    s = km.Stream(0)
    yield s
    s.close()


@pytest.fixture
def budget():
    """budget(b) -> a stream whose frontier routes queries past b goals (KETO_FR_BUDGET is read
    once, when a stream is created)"""
    old = os.environ.get("KETO_FR_BUDGET")
    made = []

    def set_budget(b):
        os.environ["KETO_FR_BUDGET"] = str(b)
        made.append(km.Stream(0))
        return made[-1]

    yield set_budget
    for s in made:
        s.close()
    if old is None:
        os.environ.pop("KETO_FR_BUDGET", None)
    else:
        os.environ["KETO_FR_BUDGET"] = old


def _frontier_batch(stream, eng, q):
    stream.frontier_stats(reset=True)
    allowed, err = eng.check_batch(q)
    return allowed, err, stream.frontier_stats(reset=True)


# (552, 591, 1269: worlds with more than 128 decisive expand-subject children in one chunk of the
# block engine, which once routed the queries past that count -- tools/parity_sweep.py found them)
@pytest.mark.parametrize("rewrites", [True, False])
@pytest.mark.parametrize("b", [1024, 6])
@pytest.mark.parametrize("seed", list(range(60)) + [552, 591, 1269])
def test_random_worlds_frontier_vs_oracle(budget, seed, b, rewrites):
    stream = budget(b)
    w, t, q, _ = random_world(seed, rewrites=rewrites)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    dec, err, _ = orc.check_batch(q, threads=4)
    udec, uerr, routed, goals, _ = orc.check_u_batch(q, threads=4, budget=b)
    # the restatement's claim: unrouted queries decide as the canonical DFS does
    ok = routed == 0
    np.testing.assert_array_equal(udec[ok], dec[ok])
    np.testing.assert_array_equal(uerr[ok], err[ok])
    snap = product_snapshot(w, t)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    allowed, gerr, fs = _frontier_batch(stream, eng, queries_to_product(q))
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    assert fs["batches"] == 1 and fs["queries"] == len(q)
    assert fs["routed"] == int(routed.sum())
    if not routed.any():
        assert fs["goals"] == int(goals.sum())


def test_drive_small_frontier_vs_oracle(stream):
    from keto_mi355x import synth
    wl = synth.drive(depth=6, n_groups=3000, n_users=8000, seed=4)
    q = synth.drive_queries(wl, 20_000, seed=3)
    q["max_depth"][:500] = np.random.default_rng(1).integers(1, 6, 500)  # truncation sub-batch
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    orc.set_limits(wl.max_depth, wl.max_width)
    qo = queries_to_oracle(q)
    dec, err, _ = orc.check_batch(qo, threads=8)
    _, _, routed, goals, gens = orc.check_u_batch(qo, threads=8, budget=1024)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    allowed, gerr, fs = _frontier_batch(stream, eng, q)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    assert fs["routed"] == int(routed.sum())
    assert fs["max_generations"] == int(gens.max())
    if not routed.any():
        assert fs["goals"] == int(goals.sum())
    assert fs["routed"] < 0.01 * len(q)


def test_nested_groups_small_frontier_vs_oracle(stream):
    """a rewrite-free snapshot (BASELINE config 2's shape) on the frontier engine, the default for
    every snapshot: decisions, routed count and goals pinned to the restatement"""
    from keto_mi355x import synth
    wl = synth.nested_groups(200_000, seed=5)
    q = synth.nested_groups_queries(wl, 20_000, seed=9, trunc_frac=0.05)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    orc.set_limits(wl.max_depth, wl.max_width)
    qo = queries_to_oracle(q)
    dec, err, _ = orc.check_batch(qo, threads=8)
    _, _, routed, goals, gens = orc.check_u_batch(qo, threads=8, budget=1024)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    allowed, gerr, fs = _frontier_batch(stream, eng, q)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    assert fs["batches"] == 1 and fs["routed"] == int(routed.sum())
    assert fs["max_generations"] == int(gens.max())
    if not routed.any():
        assert fs["goals"] == int(goals.sum())
    assert 0.05 < allowed.mean() < 0.95


def test_every_query_routed_matches_oracle(budget):
    """budget 1: every query whose root goal has a sub-check goes to the DFS interpreter through the
    routed list (rs_check_u's count with the same budget: a root the shaping makes a rewrite goal
    that decides alone -- an IN-shortcut hit -- is not routed)"""
    from keto_mi355x import synth
    stream = budget(1)
    wl = synth.drive(depth=5, n_groups=500, n_users=2000, seed=8)
    q = synth.drive_queries(wl, 4096, seed=5)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, err, _ = orc.check_batch(queries_to_oracle(q), threads=8)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    allowed, gerr, fs = _frontier_batch(stream, eng, q)
    np.testing.assert_array_equal(gerr, err)
    np.testing.assert_array_equal(allowed, dec)
    _, _, routed, _, _ = orc.check_u_batch(queries_to_oracle(q), threads=8, budget=1)
    assert fs["routed"] == int(routed.sum()) > len(q) // 2


@pytest.mark.parametrize("seed", [3, 17, 41])
def test_async_batches_match_sync(seed):
    """KETO_F_ASYNC: H2D, the speculated generations, the reductions, the DFS on the device-side
    routed count and D2H are all enqueued with no host read-back; two streams' batches in flight
    at once give the synchronous answers.  A fresh stream has no depth history (24 generations
    speculated); the deep random worlds route what lies deeper and the interpreter answers it."""
    w, t, q, _ = random_world(seed, rewrites=True)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    dec, err, _ = orc.check_batch(q, threads=4)
    snap = product_snapshot(w, t)
    qp = queries_to_product(q)
    streams = [km.Stream(0), km.Stream(0)]
    engs = [km.CheckEngine(snap, s, max_read_depth=w.max_depth, max_read_width=w.max_width) for s in streams]
    qs = [km.PinnedArray(len(qp), km.QUERY_DT) for _ in range(2)]
    outs = [(km.PinnedArray(len(qp), np.uint8), km.PinnedArray(len(qp), np.int32)) for _ in range(2)]
    for i in range(2):
        qs[i].array[:] = qp
        engs[i].check_batch_async(qs[i].array, outs[i][0].array, outs[i][1].array)
    for i in range(2):
        streams[i].sync()
        np.testing.assert_array_equal(outs[i][1].array, err)
        np.testing.assert_array_equal(outs[i][0].array, dec)
        fs = streams[i].frontier_stats()
        assert fs["async_batches"] == 1 and fs["batches"] == 0
    for s in streams:
        s.close()


@pytest.mark.parametrize("seed", list(range(0, 60, 4)))
def test_generation_engine_matches_block_engine(stream, seed):
    """the block engine (frontier_block.hip, a workgroup per chunk of queries runs all its
    generations: batches up to KETO_FR_BLOCK_MAX queries) and the generation engine
    (frontier.hip, larger batches), each forced with KETO_FR_ENGINE: the same decisions, routed
    queries and goal counts -- both evaluate frontier_goal.inc's phases"""
    w, t, q, _ = random_world(seed, rewrites=True)
    snap = product_snapshot(w, t)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    qp = queries_to_product(q)
    old = os.environ.get("KETO_FR_ENGINE")
    try:
        os.environ["KETO_FR_ENGINE"] = "gen"
        a_g, e_g, fs_g = _frontier_batch(stream, eng, qp)
        os.environ["KETO_FR_ENGINE"] = "block"
        a_b, e_b, fs_b = _frontier_batch(stream, eng, qp)
    finally:
        if old is None:
            os.environ.pop("KETO_FR_ENGINE")
        else:
            os.environ["KETO_FR_ENGINE"] = old
    np.testing.assert_array_equal(a_b, a_g)
    np.testing.assert_array_equal(e_b, e_g)
    assert fs_b["routed"] == fs_g["routed"]
    assert fs_b["max_generations"] == fs_g["max_generations"]
    if not fs_b["routed"]:
        assert fs_b["goals"] == fs_g["goals"]


def test_async_batches_in_flight_on_one_stream():
    """KETO_F_ASYNC host batches queued back to back on one stream: the library overlaps their
    copies with the kernels through two staging slots (H2D and D2H on copy streams, ordered by
    events); five batches in flight -- each slot reused -- all give the oracle's answers"""
    w, t, q, _ = random_world(29, rewrites=True)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    snap = product_snapshot(w, t)
    stream = km.Stream(0)
    eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
    rng = np.random.default_rng(5)
    batches = []
    for k in range(5):
        sub = q[rng.permutation(len(q))[: 40 + 15 * k]]
        qa = km.PinnedArray(len(sub), km.QUERY_DT)
        qa.array[:] = queries_to_product(sub)
        out = (km.PinnedArray(len(sub), np.uint8), km.PinnedArray(len(sub), np.int32))
        eng.check_batch_async(qa.array, out[0].array, out[1].array)
        batches.append((sub, qa, out))
    stream.sync()
    for sub, _, (a, e) in batches:
        dec, err, _ = orc.check_batch(sub, threads=2)
        np.testing.assert_array_equal(e.array, err)
        np.testing.assert_array_equal(a.array, dec)
    stream.close()
