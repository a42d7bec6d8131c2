"""Request coalescing (keto_dispatcher_*): many concurrent callers, batched launches, the
same decisions as one keto_check_batch over the same queries, and a live snapshot swap."""
import threading

import numpy as np
import pytest

import keto_mi355x as km
from keto_mi355x import synth

pytestmark = pytest.mark.gpu


def test_concurrent_callers_get_batch_identical_answers():
    wl = synth.drive(depth=5, n_groups=2000, n_users=5000, seed=4)
    q = synth.drive_queries(wl, 24_000, seed=3)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    want, werr = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(q)
    d = km.Dispatcher(snap, wl.max_depth, wl.max_width, max_batch=4096)
    got = np.zeros(len(q), np.uint8)
    gerr = np.zeros(len(q), np.int32)
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
    # a request larger than the staging runs alone through the host path
    a, e = d.check(q[:10_000])
    np.testing.assert_array_equal(a, want[:10_000])
    # every caller's slice came back intact: compare the ranges the clients covered
    covered = np.zeros(len(q), bool)
    for t in range(T):
        for i in range(t * 64, len(q), T * 64):
            covered[i:i + 1] = True
    np.testing.assert_array_equal(got[covered], want[covered])
    np.testing.assert_array_equal(gerr[covered], werr[covered])
    d.close()


def test_snapshot_swap_between_batches():
    wl = synth.drive(depth=4, n_groups=500, n_users=2000, seed=9)
    q = synth.drive_queries(wl, 4096, seed=1)
    full = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    empty = km.Snapshot(wl.namespaces, wl.tuples[:0], wl.ns_names, wl.rel_names, wl.n_uuids)
    d = km.Dispatcher(full, wl.max_depth, wl.max_width)
    a1, _ = d.check(q)
    assert a1.sum() > 0
    d.set_snapshot(empty)
    full.close()  # no longer in use once set_snapshot returned
    a2, _ = d.check(q)
    assert a2.sum() == 0
    d.close()


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
