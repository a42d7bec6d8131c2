"""bench.py's N>1 replicated path (configs 2-4) run by two gloo ranks sharing
the box's GPU: rank 0 generates the tuples, `bench.broadcast_tuples` sends them to every rank,
each rank builds its replica on the device from the received buffer (keto_snapshot_build_device)
and checks its own seeded shard of the query stream.  Every rank's decisions must equal the
oracle's over the tuples that rank received, the replicas must be identical, and the job rate
is all ranks' checks over the slowest rank's time."""
import hashlib
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import keto_mi355x as km
        import refsem
        from keto_mi355x import synth
        from product_helpers import queries_to_oracle, world_from_workload

        wl = synth.drive(depth=7, fanout=4, acl_per_node=6, n_groups=5000, members_per_group=10, n_users=50_000,
                         seed=21, materialize=(rank == 0))
        nt = wl.meta["n_tuples"]
        buf = bench.broadcast_tuples(wl.tuples, nt * km.TUPLE_DT.itemsize, 0, rank)
        received = buf.cpu().numpy().view(km.TUPLE_DT).copy()
        snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict, device=0,
                           device_tuples=(buf.data_ptr(), nt))
        del buf
        eng = km.CheckEngine(snap, km.Stream(0), max_read_depth=wl.max_depth, max_read_width=wl.max_width)
        q = synth.drive_queries(wl, 8192, seed=bench.shard_seed(11, rank))
        allowed, err = eng.check_batch(q)
        w, _ = world_from_workload(wl, with_tuples=False)
        orc = refsem.Oracle(w, received.view(refsem.TUPLE_DT), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, oerr, _ = orc.check_batch(queries_to_oracle(q), threads=4)
        orc.close()
        value, t, units = bench.job_rate(1.0 + rank, len(q), "cpu")
        out[rank] = (int((allowed != dec).sum()), int((err != oerr).sum()), int(dec.sum()), value, t, units,
                     hashlib.sha256(received.tobytes()).hexdigest(), q.tobytes())
    finally:
        dist.destroy_process_group()


def test_two_rank_replicas_match_oracle():
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        dmis, emis, n_allowed, value, t, units, _, _ = res[r]
        assert dmis == 0 and emis == 0
        assert n_allowed > 0
        assert t == pytest.approx(2.0) and units == 2 * 8192 and value == pytest.approx(units / 2.0)
    assert res[0][6] == res[1][6]  # identical replicas
    assert res[0][7] != res[1][7]  # each rank checks its own shard of the query stream
