"""N>1 path of bench.py on CPU: two gloo ranks (127.0.0.1) run the same cross-rank
aggregation the GPU job uses -- whole-job units = sum over ranks, time = max over ranks --
and shard the query stream by rank (distinct seeded batches, identical replicas)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "djy-keto_amd"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from keto_mi355x import synth

    wl = synth.nested_groups(20_000, seed=1)  # same replica on every rank
    q = synth.nested_groups_queries(wl, 512, seed=bench.shard_seed(7, rank))
    elapsed = 0.5 + rank  # rank 1 is the slow one
    value, t, units = bench.job_rate(elapsed, len(q) * 3, "cpu")
    out[rank] = (value, t, units, int(wl.tuples["obj"].sum()), q.tobytes())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_job_rate_and_sharding():
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        value, t, units, _, _ = res[r]
        assert t == pytest.approx(1.5)            # max over ranks
        assert units == 2 * 512 * 3               # sum over ranks
        assert value == pytest.approx(units / 1.5)
    assert res[0][3] == res[1][3]                 # identical replicas
    assert res[0][4] != res[1][4]                 # each rank its own shard of the query stream


def test_single_rank_job_rate_without_group():
    import bench
    assert not dist.is_initialized()
    assert bench.job_rate(2.0, 10) == (5.0, 2.0, 10)
    assert np.isfinite(bench.job_rate(1e-3, 1)[0])


def test_bench_gpus_2_launches_two_ranks_cpu_dry_run():
    """`bench.py --gpus 2` without torchrun starts two rank processes itself (fresh children,
    127.0.0.1 rendezvous); --dry-run swaps the GPU work for an oracle batch per rank, so the
    launcher, the max-over-ranks timing and the per-rank ms are exercised on the CPU"""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "0",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and len(out["per_rank_ms_per_step"]) == 2
    assert out["checks"] == 2 * 256 * 2  # both ranks' units
    assert out["ms_per_step"] == pytest.approx(max(out["per_rank_ms_per_step"]), rel=1e-6)


def test_bench_gpus_n_fails_loudly_without_gpus():
    """no GPU here: `bench.py --gpus 2` must exit non-zero, never print a 1-GPU line"""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "{" not in r.stdout
    assert "GPU(s) visible" in r.stderr


def test_bench_world_must_match_gpus():
    import subprocess

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
