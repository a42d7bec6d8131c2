"""keto_query16 (ABI 7, include/keto_mi355x.h): the 16-byte Check record SURVEY 8.1 A1 sizes --
host packing on the CPU (every field that fits round-trips; anything outside the form is refused
with KETO_E_LIMIT, never truncated), and on the GPU keto_check_batch16 deciding exactly as
keto_check_batch on the same requests (synchronous and KETO_F_ASYNC over pinned buffers)."""
import numpy as np
import pytest

import keto_mi355x as km
from keto_mi355x import synth


def _unpack(p):
    return dict(obj=p["obj"], s_obj=p["s_obj"], ns=p["ns_rel"] & 0xFFF, rel=(p["ns_rel"] >> 12) & 0x3FF,
                s_rel=p["ns_rel"] >> 22, s_ns=p["s_ns_depth"] & 0xFFF, subj_kind=(p["s_ns_depth"] >> 12) & 1,
                max_depth=(p["s_ns_depth"] >> 16).astype(np.uint16).view(np.int16).astype(np.int32))


def _random_queries(n, rng):
    q = np.zeros(n, dtype=km.QUERY_DT)
    q["ns"], q["rel"] = rng.integers(0, 4096, n), rng.integers(0, 1024, n)
    q["obj"], q["s_obj"] = rng.integers(0, 2**32, n, dtype=np.uint64), rng.integers(0, 2**32, n, dtype=np.uint64)
    q["subj_kind"] = rng.integers(0, 2, n)
    q["s_ns"], q["s_rel"] = rng.integers(0, 4096, n), rng.integers(0, 1024, n)
    q["max_depth"] = rng.integers(-32768, 32768, n)
    return q


def test_pack_round_trips_every_field_that_fits():
    q = _random_queries(20_000, np.random.default_rng(1))
    u = _unpack(km.pack_queries16(q))
    for f in ("obj", "s_obj", "ns", "rel", "subj_kind", "max_depth"):
        np.testing.assert_array_equal(u[f], q[f].astype(u[f].dtype), err_msg=f)
    s = q["subj_kind"] == 1  # a subject id's namespace and relation are never read: packed as 0
    np.testing.assert_array_equal(u["s_ns"][s], q["s_ns"][s])
    np.testing.assert_array_equal(u["s_rel"][s], q["s_rel"][s])
    assert (u["s_ns"][~s] == 0).all() and (u["s_rel"][~s] == 0).all()


@pytest.mark.parametrize("field,value", [("ns", 4096), ("rel", 1024), ("max_depth", 32768), ("max_depth", -32769),
                                         ("subj_kind", 2), ("s_ns", 4096), ("s_rel", 1024)])
def test_pack_refuses_what_does_not_fit(field, value):
    q = _random_queries(8, np.random.default_rng(2))
    q["subj_kind"] = 1
    q[field][5] = value
    with pytest.raises(km.KetoError) as e:
        km.pack_queries16(q)
    assert e.value.code == km._abi.KETO_E_LIMIT and "16-byte" in str(e.value)


@pytest.mark.gpu
def test_check_batch16_equals_check_batch():
    wl = synth.drive(depth=6, n_groups=3000, n_users=20_000, seed=21)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    q = synth.drive_queries(wl, 50_000, seed=5)
    q["max_depth"][:2000] = np.random.default_rng(3).integers(-3, 9, 2000)
    eng = km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    a32, e32 = eng.check_batch(q, err_detail=True)
    q16 = km.pack_queries16(q)
    a16, e16 = eng.check_batch16(q16, err_detail=True)
    np.testing.assert_array_equal(a16, a32)
    np.testing.assert_array_equal(e16, e32)
    assert 0 < a32.sum() < len(q)
    pq = km.PinnedArray(len(q), km.QUERY16_DT)
    pq.array[:] = q16
    pa, pe = km.PinnedArray(len(q), np.uint8), km.PinnedArray(len(q), np.int32)
    eng.check_batch_async(pq.array, pa.array, pe.array)
    eng.stream.sync()
    np.testing.assert_array_equal(pa.array, a32)
    np.testing.assert_array_equal(pe.array & 0xFF, e32 & 0xFF)
    snap.close()


@pytest.mark.gpu
@pytest.mark.parametrize("copy_streams", ["1", "2"])
def test_async_batches_interleaved_with_synchronous_ones(monkeypatch, copy_streams):
    """KETO_F_ASYNC host batches on one copy stream (default: each batch's D2H enqueued behind the
    next batch's H2D, or by keto_stream_sync) and on two (KETO_COPY_STREAMS=2): five async batches
    of different sizes in a row, a synchronous batch on the same stream between them, then one
    sync -- every batch's outputs equal its synchronous answers (no D2H lost, none written into
    another batch's buffers)"""
    monkeypatch.setenv("KETO_COPY_STREAMS", copy_streams)
    wl = synth.drive(depth=5, n_groups=800, n_users=5000, seed=23)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    eng = km.CheckEngine(snap, km.Stream(0), max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    sizes = [30_000, 4_096, 77_000, 1, 12_345]
    qs = [synth.drive_queries(wl, n, seed=40 + k) for k, n in enumerate(sizes)]
    ref = [eng.check_batch(q) for q in qs]
    pins = []
    for k, q in enumerate(qs):
        pq = km.PinnedArray(len(q), km.QUERY16_DT)
        pq.array[:] = km.pack_queries16(q)
        pa, pe = km.PinnedArray(len(q), np.uint8), km.PinnedArray(len(q), np.int32)
        pa.array[:] = 0xEE
        pins.append((pq, pa, pe))
        eng.check_batch_async(pq.array, pa.array, pe.array)
        if k == 2:  # a synchronous batch on the same stream, between async ones
            a, e = eng.check_batch(qs[0])
            np.testing.assert_array_equal(a, ref[0][0])
    eng.stream.sync()
    for (pq, pa, pe), (a, e) in zip(pins, ref):
        np.testing.assert_array_equal(pa.array, a)
        np.testing.assert_array_equal(pe.array, e)
    snap.close()
