"""Config-5 partitioned path on the CPU: the object partition, the claim that makes the
closure exchange exact -- the oracle over a batch's closure (tests/closure_ref.py, the numpy
restatement of csrc/partition.hip) decides every query of the batch, and builds every Expand
tree, exactly as the oracle over the whole graph; with the Check filter that ships only the
batch's own subject ids -- and the keto_collective adapter over two gloo ranks."""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import keto_mi355x as km  # noqa: E402
import refsem  # noqa: E402
from closure_ref import closure  # noqa: E402
from keto_mi355x import partition, synth  # noqa: E402
from product_helpers import queries_to_oracle, world_from_workload  # noqa: E402


def _small_drive(seed=4):
    return synth.drive(depth=4, fanout=3, acl_per_node=6, n_groups=300, members_per_group=8, n_users=2000,
                       seed=seed)


def _rows_sorted(t):
    return np.sort(np.ascontiguousarray(t).view(np.uint8).reshape(len(t), -1).view("V48").reshape(-1))


def test_owner_matches_the_header_function():
    # a fixed value, so the C inline function in the header and this mirror cannot drift apart
    assert int(partition.object_owner(np.array([3], np.uint32), np.array([12345], np.uint32), 8)[0]) == \
        (((((3 << 32) | 12345) * 0x9E3779B97F4A7C15) % (1 << 64)) >> 32) % 8
    rng = np.random.default_rng(1)
    ns = rng.integers(0, 64, 5000).astype(np.uint32)
    obj = rng.integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)
    for n in (1, 2, 3, 8):
        a = partition.object_owner(ns, obj, n)
        b = np.array([(((((int(x) << 32) | int(y)) * 0x9E3779B97F4A7C15) % (1 << 64)) >> 32) % n
                      for x, y in zip(ns[:200], obj[:200])])
        np.testing.assert_array_equal(a[:200], b)
        assert a.max() < n


def test_partitions_cover_the_graph_exactly():
    w = _small_drive()
    parts = [synth.drive_partition(w, 3, r) for r in range(3)]
    assert sum(len(p) for p in parts) == len(w.tuples)
    for r, p in enumerate(parts):
        assert (partition.object_owner(p["ns"], p["obj"], 3) == r).all()
    np.testing.assert_array_equal(_rows_sorted(np.concatenate(parts)), _rows_sorted(w.tuples))


def test_placed_partitions_keep_each_tree_on_one_rank():
    """keto_placement (keto_object_owner_placed): a placed namespace's owner is (obj / block) %
    world, every other namespace keeps the hash; synth.drive_placement puts each root's Folder and
    File objects on one rank, and the placed partitions still cover the graph exactly once"""
    w = synth.drive(depth=3, fanout=3, acl_per_node=3, n_groups=80, members_per_group=4, n_users=300, seed=4, roots=5)
    pl = synth.drive_placement(w)
    ns = np.array([0, 1, 2, 3, 17, 2], np.uint32)
    obj = np.array([5, 9, 130, 41, 7, 2**32 - 1], np.uint32)
    own = partition.object_owner(ns, obj, 3, pl)
    hashed = partition.object_owner(ns, obj, 3)
    for i in range(len(ns)):
        b = int(pl[ns[i]]) if ns[i] < 16 else 0
        assert own[i] == ((int(obj[i]) // b) % 3 if b else hashed[i])
    parts = [synth.drive_partition(w, 3, r, placement=pl) for r in range(3)]
    np.testing.assert_array_equal(_rows_sorted(np.concatenate(parts)), _rows_sorted(w.tuples))
    per = w.meta["nodes_per_root"]
    for r, p in enumerate(parts):
        assert (partition.object_owner(p["ns"], p["obj"], 3, pl) == r).all()
        tree = np.isin(p["ns"], [w.ns_names.index("Folder"), w.ns_names.index("File")])
        assert ((p["obj"][tree] // per) % 3 == r).all()  # whole trees


def test_replicated_groups_on_every_rank():
    """KETO_PLACE_ALL: a replicated namespace's objects are OWNER_ALL (keto_object_owner_placed
    returns KETO_OWNER_ALL), every rank's partition holds all of its tuples, the others are split
    as before"""
    w = synth.drive(depth=3, fanout=3, acl_per_node=3, n_groups=80, members_per_group=4, n_users=300, seed=4, roots=5)
    pl = synth.drive_placement(w, replicate_groups=True)
    g = w.ns_names.index("Group")
    assert pl[g] == partition.PLACE_ALL
    parts = [synth.drive_partition(w, 3, r, placement=pl) for r in range(3)]
    groups = w.tuples[w.tuples["ns"] == g]
    for r, p in enumerate(parts):
        o = partition.object_owner(p["ns"], p["obj"], 3, pl)
        assert ((o == r) | (o == partition.OWNER_ALL)).all()
        np.testing.assert_array_equal(_rows_sorted(p[p["ns"] == g]), _rows_sorted(groups))
    rest = np.concatenate([p[p["ns"] != g] for p in parts])
    np.testing.assert_array_equal(_rows_sorted(rest), _rows_sorted(w.tuples[w.tuples["ns"] != g]))


@pytest.mark.parametrize("depth", [2, 3, 16])
def test_closure_decides_like_the_whole_graph(depth):
    """the exactness claim, Check (with the subject filter) and Expand; fewer levels than
    max_read_depth + 1 do produce mismatches, so the comparison is not vacuous"""
    wl = _small_drive()
    q = synth.drive_queries(wl, 3000, seed=20)
    q["max_depth"][:500] = np.random.default_rng(0).integers(1, 6, 500)
    w, _ = world_from_workload(wl, with_tuples=False)
    full = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    full.set_limits(depth, wl.max_width)
    d0, e0, _ = full.check_batch(queries_to_oracle(q), threads=4)
    subj = q["s_obj"][q["subj_kind"] == 0]
    rows = closure(wl.tuples, q["ns"], q["obj"], depth + 1, subjects=subj)
    assert len(rows) < len(wl.tuples)
    sub = refsem.Oracle(w, rows.view(refsem.TUPLE_DT), shard_bytes=True)
    sub.set_limits(depth, wl.max_width)
    d1, e1, _ = sub.check_batch(queries_to_oracle(q), threads=4)
    np.testing.assert_array_equal(d0, d1)
    np.testing.assert_array_equal(e0, e1)
    if depth == 16:  # one level short: the found-lookahead beyond the last row is missing
        short = refsem.Oracle(w, closure(wl.tuples, q["ns"], q["obj"], 3, subjects=subj).view(refsem.TUPLE_DT),
                              shard_bytes=True)
        short.set_limits(depth, wl.max_width)
        assert (short.check_batch(queries_to_oracle(q), threads=4)[0] != d0).any()
    rng = np.random.default_rng(5)
    roots = np.zeros(100, dtype=km.SUBJSET_DT)
    roots["ns"][:50], roots["rel"][:50] = 1, wl.rel_names.index("members")
    roots["obj"][:50] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 50)
    roots["ns"][50:], roots["rel"][50:] = 2, wl.rel_names.index("viewers")
    roots["obj"][50:] = rng.integers(0, wl.meta["folders_per_root"], 50)
    xrows = closure(wl.tuples, roots["ns"], roots["obj"], depth + 1)
    xsub = refsem.Oracle(w, xrows.view(refsem.TUPLE_DT), shard_bytes=True)
    xsub.set_limits(depth, wl.max_width)
    for r in roots:
        a, _ = full.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), depth)
        b, _ = xsub.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), depth)
        assert a.tobytes() == b.tobytes()  # pre-order node arrays, child order included


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
        from torch_collective import TorchCollective
        coll = TorchCollective()
        # the adapter itself
        got = coll.alltoall_u64(np.array([10 * rank + r for r in range(world)], np.uint64))
        send_bytes = [r + 1 + rank for r in range(world)]
        send = np.concatenate([np.full(b, 16 * rank + r, np.uint8) for r, b in enumerate(send_bytes)])
        recv_bytes = [r + 1 + rank for r in range(world)]  # rank r sent rank+1+r bytes to me
        recv_bytes = [rank + 1 + r for r in range(world)]
        recv = np.zeros(sum(recv_bytes), np.uint8)
        coll.alltoallv(send, send_bytes, recv, recv_bytes)
        mx = coll.allreduce_max_u64(100 + rank)
        # and through the C callbacks the library calls
        c, fns = partition._c_collective(coll)
        a = (ctypes.c_uint64 * world)(*[7 * rank + r for r in range(world)])
        b = (ctypes.c_uint64 * world)()
        rc1 = c.alltoall_u64(None, a, b)
        v = (ctypes.c_uint64 * 1)(5 + rank)
        rc2 = c.allreduce_max_u64(None, v)
        out[rank] = (got.tolist(), recv.tolist(), recv_bytes, mx, rc1, list(b), rc2, v[0])
    finally:
        dist.destroy_process_group()


def test_collective_adapter_two_gloo_ranks():
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        got, recv, recv_bytes, mx, rc1, b, rc2, v = res[rank]
        assert got == [10 * r + rank for r in range(world)]
        want = []
        for r in range(world):
            want += [16 * r + rank] * recv_bytes[r]
        assert recv == want
        assert mx == 100 + world - 1
        assert rc1 == 0 and b == [7 * r + rank for r in range(world)]
        assert rc2 == 0 and v == 5 + world - 1


def test_generator_rows_give_the_same_closure():
    """synth.drive_object_tuples (the generator's rows of given objects, used for config 5 at x40
    where the graph is never held whole) against the materialized graph: same closure, same rows"""
    from closure_ref import closure
    from keto_mi355x import synth
    wl = synth.drive(depth=5, fanout=4, n_groups=2000, n_users=5000, seed=6)
    q = synth.drive_queries(wl, 3000, seed=2)
    sub = q["s_obj"][q["subj_kind"] == 0]
    a = closure(wl.tuples, q["ns"], q["obj"], wl.max_depth + 1, subjects=sub)
    b = closure(lambda k: synth.drive_object_tuples(wl, k), q["ns"], q["obj"], wl.max_depth + 1, subjects=sub)
    assert len(a) == len(b) > 0
    ka = np.sort(a.view(np.uint8).reshape(len(a), -1), axis=0)
    kb = np.sort(b.view(np.uint8).reshape(len(b), -1), axis=0)
    # same multiset of records (the generator emits objects in key order, the array in tuple order)
    sa = np.unique(a.view(np.dtype((np.void, a.dtype.itemsize))))
    sb = np.unique(b.view(np.dtype((np.void, b.dtype.itemsize))))
    assert len(sa) == len(a) and np.array_equal(sa, sb)
    assert ka.shape == kb.shape
