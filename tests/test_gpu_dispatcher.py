"""Request coalescing (keto_dispatcher_*): many concurrent callers, batched launches, answers
equal to the oracle's (oracle/refsem.c), a snapshot swap under sustained load, and Expand
coalescing (expand/handler.go:115-152) against the oracle's trees."""
import threading
import time

import numpy as np
import pytest

import keto_mi355x as km
import refsem
from keto_mi355x import synth
from product_helpers import world_from_workload

pytestmark = pytest.mark.gpu


def _oracle(wl, tuples=None):
    w, _ = world_from_workload(wl, with_tuples=False)
    t = wl.tuples if tuples is None else tuples
    orc = refsem.Oracle(w, np.ascontiguousarray(t).view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    return orc


def _oracle_answers(orc, q):
    dec, err, _ = orc.check_batch(q.view(refsem.QUERY_DT), threads=8)
    return dec, err


def test_concurrent_callers_match_oracle():
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=4)
    q = synth.drive_queries(wl, 24_000, seed=3)
    q["max_depth"][:500] = np.random.default_rng(1).integers(1, 5, 500)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    want, werr = _oracle_answers(_oracle(wl), q)
    events = []
    d = km.Dispatcher(snap, wl.max_depth, wl.max_width, max_batch=4096, on_batch=events.append)
    got = np.full(len(q), 7, np.uint8)
    gerr = np.full(len(q), -1, np.int32)
    errors = []

    def client(t, T):
        try:
            rng = np.random.default_rng(t)
            i = t * 64
            while i < len(q):
                k = int(rng.integers(1, 65))  # requests of 1..64 queries
                a, e = d.check(q[i:i + k])
                got[i:i + len(a)], gerr[i:i + len(a)] = a, e
                i += T * 64
        except Exception as ex:  # surfaced by the assertion below
            errors.append(ex)

    T = 24
    th = [threading.Thread(target=client, args=(t, T)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors
    st = d.stats()
    assert st["batches"] < st["requests"]  # requests really were coalesced
    assert st["max_batch_seen"] <= 4096
    # the per-batch hook (the shim's metrics): one event per batch, the same totals as the stats
    assert len(events) == st["batches"] and sum(e["queries"] for e in events) == st["queries"]
    assert all(e["kind"] == 0 and e["rc"] == 0 and e["wall_ms"] > 0 for e in events)
    assert sum(e["device_ms"] for e in events) > 0
    covered = got != 7
    assert covered.sum() > len(q) // 2
    np.testing.assert_array_equal(got[covered], want[covered])
    np.testing.assert_array_equal(gerr[covered], werr[covered])
    # a request larger than the staging runs alone through the host path
    a, e = d.check(q[:10_000])
    np.testing.assert_array_equal(a, want[:10_000])
    np.testing.assert_array_equal(e, werr[:10_000])
    d.close()


def test_snapshot_swap_under_load():
    """set_snapshot while 16 clients keep the dispatcher busy: the swap returns (no
    starvation), every answer is the oracle's on the old or the new tuples, and every
    request issued after the swap returned gets the new snapshot's (oracle) answer.
    Starvation-freedom is counted in batches, not seconds, so a loaded box does not decide
    the verdict: while set_snapshot waits, the dispatcher completes at most a few rounds of
    its inflight slots (the old snapshot's batches drain, new ones run beside them)."""
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=9)
    q = synth.drive_queries(wl, 8192, seed=1)
    keep = np.random.default_rng(2).random(len(wl.tuples)) < 0.6  # the new snapshot: 60% of the tuples
    t_new = wl.tuples[keep]
    old = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    new = km.Snapshot(wl.namespaces, t_new, wl.ns_names, wl.rel_names, wl.n_uuids)
    a_old, _ = _oracle_answers(_oracle(wl), q)
    a_new, _ = _oracle_answers(_oracle(wl, t_new), q)
    assert (a_old != a_new).sum() > 100
    d = km.Dispatcher(old, wl.max_depth, wl.max_width, max_batch=2048, inflight=4)
    stop = threading.Event()
    swapped_at = [None]
    log, errors = [], []

    def client(t):
        rng = np.random.default_rng(100 + t)
        try:
            while not stop.is_set():
                i = int(rng.integers(0, len(q) - 64))
                t0 = time.monotonic()
                a, _ = d.check(q[i:i + 64])
                log.append((t0, i, a.copy()))
        except Exception as ex:
            errors.append(ex)

    th = [threading.Thread(target=client, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    time.sleep(0.5)
    t0 = time.monotonic()
    b0 = d.stats()["batches"]
    d.set_snapshot(new)
    swapped_at[0] = time.monotonic()
    swap_batches = d.stats()["batches"] - b0
    swap_s = swapped_at[0] - t0
    old.close()  # no longer in use once set_snapshot returned
    time.sleep(0.5)
    stop.set()
    for x in th:
        x.join()
    d.close()
    assert not errors
    assert swap_batches <= 16 * 4, f"the swap waited through {swap_batches} batches ({swap_s:.2f} s)"
    assert swap_s < 120.0  # (a hang guard only)
    after = 0
    for ts, i, a in log:
        want_new, want_old = a_new[i:i + 64], a_old[i:i + 64]
        if ts > swapped_at[0]:
            np.testing.assert_array_equal(a, want_new)
            after += 1
        else:
            assert (a == want_new).all() or (a == want_old).all()
    assert after > 10


def test_expand_coalescing_matches_oracle():
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=7)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    orc = _oracle(wl)
    rng = np.random.default_rng(3)
    roots = np.zeros(600, dtype=km.SUBJSET_DT)
    roots["ns"][:300], roots["rel"][:300] = wl.ns_names.index("Group"), wl.rel_names.index("members")
    roots["obj"][:300] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 300)
    roots["ns"][300:], roots["rel"][300:] = wl.ns_names.index("Folder"), wl.rel_names.index("viewers")
    roots["obj"][300:] = rng.integers(0, wl.meta["folders_per_root"], 300)
    roots["max_depth"] = rng.integers(0, 6, 600)
    d = km.Dispatcher(snap, wl.max_depth, wl.max_width, max_batch=256)
    results, errors = {}, []

    def client(t):
        try:
            for k in range(t, 600 // 10, 12):
                results[k] = d.expand(roots[10 * k:10 * k + 10], cap=4 if k % 3 == 0 else 0)
        except Exception as ex:
            errors.append(ex)

    th = [threading.Thread(target=client, args=(t,)) for t in range(12)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    st = d.stats()
    d.close()
    assert not errors
    assert st["batches"] < st["requests"]
    orc.set_limits(wl.max_depth, wl.max_width)
    for k, (nodes, offs, err) in results.items():
        assert (err == 0).all()
        for j in range(10):
            r = roots[10 * k + j]
            on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), int(r["max_depth"]))
            mine = nodes[int(offs[j]):int(offs[j + 1])]
            assert len(mine) == len(on)
            for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                             ("s_rel", "srel"), ("n_children", "n_children")):
                np.testing.assert_array_equal(mine[f_p], on[f_o])


def test_native_closed_loop_load():
    """bench.py's serving probe: native client threads through keto_dispatcher_check."""
    wl = synth.drive(depth=4, n_groups=500, n_users=2000, seed=6)
    q = synth.drive_queries(wl, 4096, seed=2)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    d = km.Dispatcher(snap, wl.max_depth, wl.max_width, max_batch=1024)
    r = synth.closed_loop(d, q, clients=16, req=32, seconds=0.5)
    st = d.stats()
    d.close()
    assert r["requests"] > 0 and r["checks"] == 32 * r["requests"]
    assert st["queries"] >= r["checks"]  # every request went through the dispatcher's batches
    assert 0 < r["p50_ms"] <= r["p99_ms"] <= r["max_ms"]


def test_two_snapshot_rotation_with_in_place_advance():
    """the serving pattern keto_store_snapshot_advance asks for: two store snapshots, one served,
    one idle.  Per transaction the idle one is advanced in place, swapped in (set_snapshot waits
    for the old one's batches), and the old one -- idle now -- advanced in turn.  Under 16 busy
    clients every answer is the oracle's at the version served when the request was issued (or the
    next one, if a swap landed during it)"""
    from store_ref import transact

    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=9)
    q = synth.drive_queries(wl, 8192, seed=1)
    rng = np.random.default_rng(4)
    st = km.TupleStore(wl.tuples)
    snaps = [km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, store=st) for _ in range(2)]
    host = wl.tuples.copy()
    answers = [_oracle_answers(_oracle(wl, host), q)[0]]
    d = km.Dispatcher(snaps[0], wl.max_depth, wl.max_width, max_batch=2048, inflight=4)
    stop = threading.Event()
    swaps, log, errors = [], [], []

    def client(t):
        r = np.random.default_rng(100 + t)
        try:
            while not stop.is_set():
                i = int(r.integers(0, len(q) - 64))
                t0 = time.monotonic()
                a, _ = d.check(q[i:i + 64])
                log.append((t0, i, a.copy()))
        except Exception as ex:
            errors.append(ex)

    th = [threading.Thread(target=client, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    served = 0
    for step in range(3):
        time.sleep(0.3)
        t = host
        ins = t[rng.choice(len(t), 800, replace=False)].copy()
        ins["subj_kind"], ins["s_ns"], ins["s_rel"] = 0, 0, 0
        ins["s_obj"] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], len(ins))
        ins["shard_id"] = rng.integers(0, 256, (len(ins), 16), dtype=np.uint8)
        dele = t[rng.choice(len(t), 1500, replace=False)].copy()
        st.transact(ins, dele)
        host = transact(host, ins, dele)
        answers.append(_oracle_answers(_oracle(wl, host), q)[0])
        idle = 1 - served
        assert snaps[idle].advance(st)
        d.set_snapshot(snaps[idle])
        swaps.append(time.monotonic())
        served = idle
        assert snaps[1 - served].advance(st)  # the old one: idle once set_snapshot returned
    time.sleep(0.3)
    stop.set()
    for x in th:
        x.join()
    d.close()
    assert not errors
    assert (answers[0] != answers[-1]).sum() > 100
    late = 0
    for ts, i, a in log:
        v = sum(1 for s in swaps if s < ts)
        ok = [answers[v][i:i + 64]] + ([answers[v + 1][i:i + 64]] if v + 1 < len(answers) else [])
        assert any((a == w).all() for w in ok), (v, i)
        late += v == len(swaps)
    assert late > 10
    for s in snaps:
        s.close()
    st.close()
