"""Config-5 partitioned path on the GPU through the C ABI (keto_partition_*): device closure
exchange -> device snapshot build -> the unmodified Check / Expand kernels, against the oracle
over the whole graph (bit-exact), on one rank and on two gloo ranks sharing the box's GPU.
The device closure has exactly the size of the numpy restatement's (tests/closure_ref.py)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import keto_mi355x as km
import refsem
from closure_ref import closure
from keto_mi355x import partition, synth
from product_helpers import queries_to_oracle, world_from_workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _wl(roots=1):
    return synth.drive(depth=6, fanout=4, acl_per_node=6, n_groups=3000, members_per_group=10, n_users=20_000,
                       seed=12, roots=roots)


def _roots(wl, rng, n):
    r = np.zeros(n, dtype=km.SUBJSET_DT)
    h = n // 2
    r["ns"][:h], r["rel"][:h] = 1, wl.rel_names.index("members")
    r["obj"][:h] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], h)
    r["ns"][h:], r["rel"][h:] = 2, wl.rel_names.index("viewers")
    r["obj"][h:] = rng.integers(0, wl.meta["folders_per_root"], n - h)
    return r


def _oracle(wl):
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    return orc


@pytest.fixture
def closure_path(monkeypatch):
    """a one-rank job through the per-batch closure path (KETO_PART_CLOSURE: by default one rank
    runs on its resident snapshot), to test the closure machinery on one GPU"""
    monkeypatch.setenv("KETO_PART_CLOSURE", "1")


def test_single_rank_resident_snapshot_matches_oracle():
    """a job of one rank (no collective) holds the whole graph: its partition becomes one resident
    snapshot at creation and every batch runs on it -- no closure, no per-batch build; the same
    decisions, pipelined batches and Expand trees as the oracle over the whole graph"""
    wl = _wl()
    q = synth.drive_queries(wl, 20_000, seed=31)
    q["max_depth"][:2000] = np.random.default_rng(0).integers(1, 8, 2000)
    eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, wl.tuples,
                                      max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    allowed, err = eng.check_batch(q, count_work=True)
    assert eng.last["tuples"] == 0 and eng.last["levels"] == 0 and eng.level_stats() == []
    assert eng.last["queries"] == len(q) and eng.last["rows"] > 0
    orc = _oracle(wl)
    dec, oerr, _ = orc.check_batch(queries_to_oracle(q), threads=8)
    np.testing.assert_array_equal(err, oerr)
    np.testing.assert_array_equal(allowed, dec)
    q2 = synth.drive_queries(wl, 5000, seed=32)
    d2, oe2, _ = orc.check_batch(queries_to_oracle(q2), threads=8)
    many = eng.check_batches([q2, q, q2, q, q2])
    for (a, e), d, oe in zip(many, (d2, dec, d2, dec, d2), (oe2, oerr, oe2, oerr, oe2)):
        np.testing.assert_array_equal(a, d)
        np.testing.assert_array_equal(e, oe)
    roots = _roots(wl, np.random.default_rng(1), 256)
    nodes, offs, xerr = eng.expand_batch(roots)
    assert (xerr == 0).all()
    for i, r in enumerate(roots):
        on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), wl.max_depth)
        mine = nodes[int(offs[i]):int(offs[i + 1])]
        assert len(mine) == len(on)
        for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                         ("s_rel", "srel"), ("n_children", "n_children")):
            np.testing.assert_array_equal(mine[f_p], on[f_o])
    eng.close()


def test_single_rank_partitioned_matches_oracle(closure_path):
    # closure buffers sized by the batches alone (no 64 MB floor): a later, larger batch then
    # outgrows the buffer its slot kept, and the one-rank closure falls back to the synchronous
    # levels (read once per process, before its first partition batch)
    os.environ["KETO_PART_MIN_CLOSURE"] = "1000"
    wl = _wl()
    q = synth.drive_queries(wl, 20_000, seed=31)
    q["max_depth"][:2000] = np.random.default_rng(0).integers(1, 8, 2000)
    eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, wl.tuples,
                                      max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    allowed, err = eng.check_batch(q)
    ref = closure(wl.tuples, q["ns"], q["obj"], wl.max_depth + 1, subjects=q["s_obj"][q["subj_kind"] == 0])
    assert eng.last["tuples"] == len(ref)
    assert 0 < eng.last["tuples"] < len(wl.tuples)
    orc = _oracle(wl)
    dec, oerr, _ = orc.check_batch(queries_to_oracle(q), threads=8)
    np.testing.assert_array_equal(err, oerr)
    np.testing.assert_array_equal(allowed, dec)
    # a second batch on the same engine (workspace reuse): its closure is enqueued level after
    # level with no host round trip (closure_self); the same batch again on the synchronous levels
    q2 = synth.drive_queries(wl, 5000, seed=32)
    a2, e2 = eng.check_batch(q2)
    ref2 = closure(wl.tuples, q2["ns"], q2["obj"], wl.max_depth + 1, subjects=q2["s_obj"][q2["subj_kind"] == 0])
    assert eng.last["tuples"] == len(ref2)
    levels2 = eng.last["levels"]
    d2, oe2, _ = orc.check_batch(queries_to_oracle(q2), threads=8)
    np.testing.assert_array_equal(a2, d2)
    os.environ["KETO_PART_SYNC_LEVELS"] = "1"
    try:
        a3, e3 = eng.check_batch(q2)
    finally:
        del os.environ["KETO_PART_SYNC_LEVELS"]
    assert eng.last["tuples"] == len(ref2) and eng.last["levels"] == levels2
    lv = eng.level_stats()  # the synchronous levels: per level, timed
    assert len(lv) == levels2 and sum(x["tuples"] for x in lv) == len(ref2) and all(x["ms"] > 0 for x in lv)
    assert sum(x["objects"] for x in lv) == eng.last["objects"]
    np.testing.assert_array_equal(a3, d2)
    # pipelined batches (keto_partition_check_many): each batch's closure on the helper thread
    # while the batch before it is built and checked; the same answers in the same order
    for sequential in (False, True):  # the closure of k+1 beside batch k, and one after another
        if sequential:
            os.environ["KETO_PART_SEQUENTIAL"] = "1"
        try:
            many = eng.check_batches([q2, q, q2, q])
        finally:
            os.environ.pop("KETO_PART_SEQUENTIAL", None)
        for (a, e), d, oe in zip(many, (d2, dec, d2, dec), (oe2, oerr, oe2, oerr)):
            np.testing.assert_array_equal(a, d)
            np.testing.assert_array_equal(e, oe)
        assert eng.last["tuples"] == len(ref)
    roots = _roots(wl, np.random.default_rng(1), 256)
    nodes, offs, xerr = eng.expand_batch(roots)
    assert eng.last["tuples"] == len(closure(wl.tuples, roots["ns"], roots["obj"], wl.max_depth + 1))
    assert (xerr == 0).all()
    for i, r in enumerate(roots):
        on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), wl.max_depth)
        mine = nodes[int(offs[i]):int(offs[i + 1])]
        assert len(mine) == len(on)
        for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                         ("s_rel", "srel"), ("n_children", "n_children")):
            np.testing.assert_array_equal(mine[f_p], on[f_o])
    eng.close()


def test_single_rank_closure_outgrows_its_buffer(closure_path):
    """a batch whose closure is over twice the largest its slot saw: the one-rank closure
    (closure_self, no host round trip per level) overflows the buffer it was sized by, and the
    batch's closure is redone on the synchronous levels, which grow it"""
    os.environ["KETO_PART_MIN_CLOSURE"] = "1000"  # (no 64 MB floor; read once per process)
    wl = _wl()
    eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, wl.tuples,
                                      max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    orc = _oracle(wl)
    for n, seed in ((64, 41), (128, 42), (20_000, 43), (64, 44)):
        q = synth.drive_queries(wl, n, seed=seed)
        allowed, err = eng.check_batch(q)
        ref = closure(wl.tuples, q["ns"], q["obj"], wl.max_depth + 1, subjects=q["s_obj"][q["subj_kind"] == 0])
        assert eng.last["tuples"] == len(ref)
        dec, oerr, _ = orc.check_batch(queries_to_oracle(q), threads=8)
        np.testing.assert_array_equal(allowed, dec)
        np.testing.assert_array_equal(err, oerr)
    eng.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, device_buffers=False, mode="dist"):
    for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    placed = "_placed" in mode  # every root's folder tree on one rank (keto_placement)
    repl = mode.endswith("_repl")  # ... and the groups on every rank (KETO_PLACE_ALL)
    mode = mode.replace("_placed", "").replace("_repl", "")
    if mode == "closure":
        os.environ["KETO_PART_CLOSURE"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch_collective import TorchCollective
        wl = _wl(3 if placed else 1)
        place = synth.drive_placement(wl, replicate_groups=repl) if placed else None
        eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids,
                                          synth.drive_partition(wl, world, rank, placement=place),
                                          max_read_depth=wl.max_depth, max_read_width=wl.max_width,
                                          collective=TorchCollective(device_buffers=device_buffers), placement=place)
        q = synth.drive_queries(wl, 8192, seed=40 + rank)
        allowed, err = eng.check_batch(q)
        st = dict(eng.last)
        lv = eng.level_stats()  # per level: the bytes of both exchanges (the batch's subject list aside)
        lv_bytes = sum(x["request_bytes"] + x["tuple_bytes_sent"] for x in lv)
        if mode == "closure":
            lv_ok = len(lv) == st["levels"] and 0 < lv_bytes <= st["bytes_sent"] and sum(x["objects"] for x in lv) == st["objects"]
        else:  # the distributed frontier: one generation record each (ABI 7), goal records out and
            # values back; level_stats holds only the routed queries' closure levels
            gens = eng.generation_stats()
            g_bytes = sum(g["record_bytes_out"] + g["value_bytes_back"] for g in gens)
            lv_ok = len(gens) == st["generations"] and g_bytes == st["exchange_bytes"] > 0 and \
                sum(g["goals"] for g in gens) == st["goals"] and (st["build_s"] == 0 or st["routed"] > 0) and \
                len(lv) == st["levels"]  # (any rank's routed queries: every rank joins the closure)
        orc = _oracle(wl)
        dec, oerr, _ = orc.check_batch(queries_to_oracle(q), threads=4)
        roots = _roots(wl, np.random.default_rng(rank), 64)
        nodes, offs, xerr = eng.expand_batch(roots)
        tree_mis = 0
        for i, r in enumerate(roots):
            on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), wl.max_depth)
            mine = nodes[int(offs[i]):int(offs[i + 1])]
            tree_mis += len(mine) != len(on) or not (mine["s_obj"] == on["sid"]).all()
        # pipelined: the closures of batches 2 and 3 exchanged from the helper thread while the
        # batch before them is checked (every rank passes the same number of batches)
        q2 = synth.drive_queries(wl, 4096, seed=60 + rank)
        d2, oe2, _ = orc.check_batch(queries_to_oracle(q2), threads=4)
        many = eng.check_batches([q, q2, q])  # (the exchange from the helper thread)
        pipe_mis = 0
        for (a, e), d, oe in zip(many, (dec, d2, dec), (oerr, oe2, oerr)):
            pipe_mis += int((a != d).sum() + (e != oe).sum())
        out[rank] = (int((allowed != dec).sum()), int((err != oerr).sum()), int(dec.sum()),
                     st["bytes_sent"] if mode == "closure" else st["exchange_bytes"], tree_mis, int((xerr != 0).sum()),
                     pipe_mis, lv_ok)
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["dist", "closure", "dist_placed", "closure_placed", "dist_placed_repl",
                                  "closure_placed_repl"])
@pytest.mark.parametrize("device_buffers", [False, True])
def test_two_rank_partitioned_matches_oracle(device_buffers, mode):
    """two ranks sharing the GPU: the exchange over host copies (keto_collective.alltoallv), and
    over the library's device buffers on its stream (alltoallv_device; gloo stages on the
    adapter's side, RCCL would move the bytes GPU to GPU).  mode "dist": resident partitions and
    the distributed frontier (frontier_dist.hip), its routed queries and Expand through the
    closure over those partitions' rows; "closure": every batch through the per-batch closure
    over a separate store (KETO_PART_CLOSURE)."""
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out, device_buffers, mode), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        dmis, emis, n_allowed, sent, tree_mis, xerr, pipe_mis, lv_ok = res[r]
        assert dmis == 0 and emis == 0 and tree_mis == 0 and xerr == 0 and pipe_mis == 0 and lv_ok
        assert n_allowed > 0 and sent > 0
