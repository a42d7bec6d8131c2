"""Config-5 partitioned path (keto_mi355x/partition.py) on the CPU: the object partition, the
closure exchange over two gloo ranks, and the claim that makes it exact.  The claim is that
the oracle over a batch's closure decides every query of the batch (and builds every Expand
tree) exactly as the oracle over the whole graph does."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import keto_mi355x as km  # noqa: E402
from keto_mi355x import partition, synth  # noqa: E402


def _small_drive(seed=4):
    return synth.drive(depth=4, fanout=3, acl_per_node=6, n_groups=300, members_per_group=8, n_users=2000,
                       seed=seed)


def _rows_sorted(t):
    return np.sort(np.ascontiguousarray(t).view(np.uint8).reshape(len(t), -1).view("V48").reshape(-1))


def test_owner_numpy_and_torch_agree():
    rng = np.random.default_rng(1)
    ns = rng.integers(0, 64, 5000).astype(np.uint32)
    obj = rng.integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)
    for n in (1, 2, 3, 8):
        a = partition.object_owner(ns, obj, n)
        k = partition._keys(torch.from_numpy(ns.view(np.int32)), torch.from_numpy(obj.view(np.int32)))
        b = partition._owner(k, n).numpy()
        np.testing.assert_array_equal(a, b)
        assert a.max() < n
    # a fixed value, so the C inline function in the header and this mirror cannot drift apart
    assert int(partition.object_owner(np.array([3], np.uint32), np.array([12345], np.uint32), 8)[0]) == \
        (((((3 << 32) | 12345) * 0x9E3779B97F4A7C15) % (1 << 64)) >> 32) % 8


def test_partitions_cover_the_graph_exactly():
    w = _small_drive()
    parts = [synth.drive_partition(w, 3, r) for r in range(3)]
    assert sum(len(p) for p in parts) == len(w.tuples)
    for r, p in enumerate(parts):
        assert (partition.object_owner(p["ns"], p["obj"], 3) == r).all()
    np.testing.assert_array_equal(_rows_sorted(np.concatenate(parts)), _rows_sorted(w.tuples))


def test_object_store_rows_of():
    w = _small_drive()
    st = partition.ObjectStore(w.tuples, "cpu")
    objs = np.unique(w.tuples[["ns", "obj"]])[:50]
    req = partition._keys(torch.from_numpy(objs["ns"].astype(np.uint32).view(np.int32)),
                          torch.from_numpy(objs["obj"].astype(np.uint32).view(np.int32)))
    req = torch.cat([req, torch.tensor([(7 << 32) | 99], dtype=torch.int64)])  # absent object
    rows, cnt = st.rows_of(req)
    assert int(cnt[-1]) == 0
    want = w.tuples[np.isin(w.tuples[["ns", "obj"]], objs)]
    assert int(cnt.sum()) == len(want)
    np.testing.assert_array_equal(_rows_sorted(rows.numpy().view(synth.TUPLE_DT).reshape(-1)), _rows_sorted(want))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import refsem
        from product_helpers import queries_to_oracle, world_from_workload

        wl = _small_drive()
        eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids,
                                          synth.drive_partition(wl, world, rank), store_device="cpu")
        q = synth.drive_queries(wl, 3000, seed=20 + rank)
        rng = np.random.default_rng(rank)
        q["max_depth"][:500] = rng.integers(1, 6, 500)  # request depths below the global one
        roots = np.zeros(200, dtype=km.SUBJSET_DT)
        roots["ns"][:100], roots["rel"][:100] = 1, wl.rel_names.index("members")
        roots["obj"][:100] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 100)
        roots["ns"][100:], roots["rel"][100:] = 2, wl.rel_names.index("viewers")
        roots["obj"][100:] = rng.integers(0, wl.meta["folders_per_root"], 100)
        w, t_full = world_from_workload(wl)
        full = refsem.Oracle(w, t_full)
        res = {}
        for depth in (2, 3, 16):
            eng.max_read_depth = depth
            full.set_limits(depth, wl.max_width)
            rows, st = eng.closure_tuples(q["ns"], q["obj"])
            sub = refsem.Oracle(w, rows.numpy().copy().view(refsem.TUPLE_DT).reshape(-1), shard_bytes=True)
            sub.set_limits(depth, wl.max_width)
            d0, e0, _ = full.check_batch(queries_to_oracle(q), threads=2)
            d1, e1, _ = sub.check_batch(queries_to_oracle(q), threads=2)
            xrows, _ = eng.closure_tuples(roots["ns"], roots["obj"])
            xsub = refsem.Oracle(w, xrows.numpy().copy().view(refsem.TUPLE_DT).reshape(-1), shard_bytes=True)
            xsub.set_limits(depth, wl.max_width)
            tree_diff = 0
            for r in roots:
                a, _ = full.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), depth)
                b, _ = xsub.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), depth)
                tree_diff += a.tobytes() != b.tobytes()  # pre-order node arrays, child order included
            res[depth] = (int((d0 != d1).sum()), int((e0 != e1).sum()), int(d0.sum()), st["tuples"], st["levels"],
                          tree_diff)
        out[rank] = (res, len(wl.tuples), eng.comm.bytes_sent)
    finally:
        dist.destroy_process_group()


def test_two_rank_closure_decides_like_the_whole_graph():
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        per_depth, n_total, sent = res[rank]
        assert sent > 0  # the other rank's objects really came over the exchange
        for depth, (dmis, emis, n_allowed, n_closure, levels, tree_diff) in per_depth.items():
            assert dmis == 0 and emis == 0 and tree_diff == 0, (rank, depth)
            assert 0 < n_allowed < 3000
            assert 0 < n_closure < n_total
            assert levels <= depth + 1
