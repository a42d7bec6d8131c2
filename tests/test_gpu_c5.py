"""BASELINE config 5 at its configured size on the GPU: the Drive forest x40 (4.22B tuples)
partitioned by object over 8 ranks (the node's 8 GPUs; here 8 gloo ranks sharing the box's one
GPU), each rank generating only its own partition (synth.drive_partition), through the C ABI
(keto_partition_*): every rank's partition built once into a resident snapshot; per Check batch
the distributed frontier (csrc/frontier_dist.hip: goal records to the nodes' owners and values
back, one all-to-all each per generation) -- no closure gather, no per-batch build; per Expand
batch the rows the walks can read fetched from their owners level by level and walked on the
device (csrc/expand_dist.hip) -- no build either.

No single snapshot can hold this graph (its 3.6B nodes exceed the u32 node space, and its
tuples alone outgrow one GPU), so there is no replicated run to compare against.  Parity is
pinned instead by the oracle over a closure computed on the host, independently of the device:
tests/closure_ref.py walks the generator's own rows (synth.drive_object_tuples) level by level
from each rank's sample of queries -- every tuple those queries can read, so the oracle's answers
are the whole graph's (oracle/refsem.c, internal/check/engine.go:65-266).

Per rank: a 2^20-query batch whose first 1% asks request depths 1-4 (the truncation sub-batch,
engine.go:82-84), run twice (determinism); an exact oracle sample of every truncation query
plus 64Ki others; 512 Expand roots (4,096 over the job: BASELINE config 5's "batched Expand
trees") against oracle trees, child order included (internal/expand/engine.go:54-124).

Every rank's phase record (generations, goals, queries routed to the closure path, bytes of goal
records and values it sent, device time of its kernels, time inside the collective) and its
exchange generation by generation (keto_partition_generations_get) go to gpurun_out/c5x40_phases.json
(profiles/ keeps a copy per round).
"""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1100)]

WORLD = 8
SCALE = int(os.environ.get("KETO_C5_SCALE", "40"))
# KETO_C5_PLACED=1: every root's folder tree on one rank (keto_placement, synth.drive_placement),
# groups and users hashed -- the same graph and queries, another owner rule
PLACED = os.environ.get("KETO_C5_PLACED") in ("1", "repl")
REPL = os.environ.get("KETO_C5_PLACED") == "repl"  # ... and the groups replicated on every rank
PHASES = f"c5x{SCALE}{'_placed' if PLACED else ''}{'_repl' if REPL else ''}_phases.json"
N = 1 << 20
SAMPLE = 1 << 16
ROOTS = 512  # Expand roots per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _log(rank, msg):
    print(f"[c5 rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.__stderr__, flush=True)


def _batch(synth, wl, seed):
    q = synth.drive_queries(wl, N, seed=seed)
    rng = np.random.default_rng(seed)
    k = N // 100
    q["max_depth"][:k] = rng.integers(1, 5, k)
    return q


def _sample(seed):
    rng = np.random.default_rng(seed + 1)
    rest = rng.choice(np.arange(N // 100, N), size=SAMPLE, replace=False)
    return np.concatenate([np.arange(N // 100), np.sort(rest)])


def _roots(km, wl, n, seed):
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


def _free_gib():
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    fr, tot = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(fr), ctypes.byref(tot))
    return f"{fr.value / 2**30:.1f} of {tot.value / 2**30:.0f} GiB free"


_PHASE_KEYS = ("generations", "goals", "routed", "exchange_bytes", "device_s", "exchange_s", "run_s", "closure_s",
               "build_s", "tuples", "levels", "bytes_sent")


def _worker(rank, world, port, out):
    for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import datetime

    # eight ranks share this one device: the partitions are created one after another (staged:
    # the slot layout is checked and the relation flags agreed at the first batch), the allocation
    # caches stay small, and the engine's arena holds fewer goals per query than a GPU of its own
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KETO_POOL_CAP_MB="1", KETO_SCRATCH_CAP_MB="1",
                      KETO_PART_TRIM="1", KETO_PART_STAGED="1", KETO_FR_GOALS_PER_QUERY=os.environ.get("KETO_C5_GOALS_PER_QUERY", "160"),
                      KETO_PART_CHUNK=os.environ.get("KETO_C5_CHUNK", "262144"))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(minutes=30))
    try:
        import keto_mi355x as km
        import refsem
        from closure_ref import closure
        from keto_mi355x import partition, synth
        from product_helpers import world_from_workload
        from torch_collective import TorchCollective

        wl = synth.drive_scaled(SCALE, materialize=False)
        eng, n_part = None, 0
        # one rank at a time generates its partition and builds its resident snapshot: the peak of
        # a build (the raw upload + the sorts) then meets only the other ranks' finished partitions
        for r in range(world):
            if r == rank:
                t0 = time.perf_counter()
                place = synth.drive_placement(wl, replicate_groups=REPL) if PLACED else None
                part = synth.drive_partition(wl, world, rank, placement=place)
                n_part = len(part)
                t1 = time.perf_counter()
                eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, part,
                                                  max_read_depth=wl.max_depth, max_read_width=wl.max_width,
                                                  collective=TorchCollective(device_buffers=True), placement=place)
                del part
                _log(rank, f"partition {n_part} tuples: generated {t1 - t0:.1f} s, resident snapshot "
                           f"{time.perf_counter() - t1:.1f} s, {_free_gib()}")
            dist.barrier()
        total = int(wl.meta["n_tuples"])
        q = _batch(synth, wl, 70 + rank)
        t0 = time.perf_counter()
        a1, e1 = eng.check_batch(q)
        st1 = dict(eng.last)
        _log(rank, f"batch 1: {time.perf_counter() - t0:.1f} s, {st1['generations']} generations, {st1['goals']} goals, "
                   f"{st1['routed']} routed, {st1['exchange_bytes'] / 1e6:.0f} MB out, {_free_gib()}")
        t0 = time.perf_counter()
        a2, e2 = eng.check_batch(q)
        wall2 = time.perf_counter() - t0
        st2, lv2 = dict(eng.last), eng.generation_stats()
        idx = _sample(70 + rank)
        qs = q[idx]
        rows = lambda k: synth.drive_object_tuples(wl, k)  # noqa: E731 -- the generator's rows, not the device's
        t0 = time.perf_counter()
        ct = closure(rows, qs["ns"], qs["obj"], wl.max_depth + 1, subjects=qs["s_obj"][qs["subj_kind"] == 0])
        w, _ = world_from_workload(wl, with_tuples=False)
        orc = refsem.Oracle(w, ct.view(refsem.TUPLE_DT), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        dec, err, _ = orc.check_batch(qs.view(refsem.QUERY_DT), threads=2)
        _log(rank, f"oracle sample {len(idx)} over a host closure of {len(ct)} tuples: {time.perf_counter() - t0:.1f} s")
        orc.close()
        roots = _roots(km, wl, ROOTS, 90 + rank)
        t0 = time.perf_counter()
        nodes, offs, xerr = eng.expand_batch(roots)
        xwall = time.perf_counter() - t0
        xst, xlv = dict(eng.last), eng.level_stats()
        ct2 = closure(rows, roots["ns"], roots["obj"], wl.max_depth + 1)
        orc2 = refsem.Oracle(w, ct2.view(refsem.TUPLE_DT), shard_bytes=True)
        orc2.set_limits(wl.max_depth, wl.max_width)
        tree_mis, n_nodes = 0, 0
        for i, r in enumerate(roots):
            on, _ = orc2.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), wl.max_depth)
            mine = nodes[int(offs[i]):int(offs[i + 1])]
            n_nodes += len(on)
            same = len(mine) == len(on)
            for f_p, f_o in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"),
                             ("s_rel", "srel"), ("n_children", "n_children")):
                same = same and np.array_equal(mine[f_p], on[f_o])
            tree_mis += 0 if same else 1
        orc2.close()
        trunc = N // 100
        out[rank] = {
            "n_part": n_part, "total": total, "routed": st1["routed"], "exchange_bytes": st1["exchange_bytes"],
            "build_s": st1["build_s"] + st2["build_s"],
            "det_mis": int((a1 != a2).sum() + (e1 != e2).sum()), "errors": int((e1 != 0).sum()),
            "allowed": float(a1.mean()), "trunc_allowed": float(a1[:trunc].mean()),
            "rest_allowed": float(a1[trunc:].mean()),
            "sample": len(idx), "dec_mis": int((a1[idx] != dec).sum()), "err_mis": int((e1[idx] != err).sum()),
            "host_closure": len(ct), "tree_mis": tree_mis, "xerr": int((xerr != 0).sum()), "tree_nodes": n_nodes,
            "x_build_s": xst["build_s"],
            "phases": {"check_batch": {"queries": N, "wall_s": wall2, **{k: st2[k] for k in _PHASE_KEYS},
                                       "generations_detail": lv2},
                       "check_batch_first": {k: st1[k] for k in _PHASE_KEYS},
                       "expand_batch": {"roots": ROOTS, "wall_s": xwall, "tree_nodes": int(offs[-1]),
                                        **{k: xst[k] for k in ("closure_s", "build_s", "run_s", "tuples", "objects",
                                                               "levels", "bytes_sent", "exchange_s")},
                                        "levels_detail": xlv}},
        }
        eng.close()
    except BaseException:
        import traceback
        _log(rank, "failed:\n" + traceback.format_exc())  # (spawn reports one rank's error: maybe a peer's)
        raise
    finally:
        dist.destroy_process_group()


def synth_meta(scale):
    """the Drive layout of C3 x scale (no tuples generated)"""
    for p in (ROOT, os.path.join(ROOT, "djy-keto_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from keto_mi355x import synth
    return synth.drive_scaled(scale, materialize=False).meta


def test_c5_x40_eight_ranks_matches_oracle():
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(WORLD, _free_port(), out), nprocs=WORLD, join=True)
        res = dict(out)
    assert sorted(res) == list(range(WORLD))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", PHASES), "w") as f:
        json.dump({"what": f"tests/test_gpu_c5.py: C3 x{SCALE} over 8 gloo ranks sharing one MI355X, resident partitions "
                           f"({('each root folder tree on one rank (keto_placement), groups ' + ('replicated on every rank' if REPL else 'hashed')) if PLACED else 'keto_object_owner'}); "
                           "per rank the second (warm) 2^20-query check batch through the distributed frontier "
                           "(keto_partition_stats_get: generations, goals, routed, bytes of goal records + values sent to "
                           "other ranks, device time of the generations' kernels, time inside the collective; "
                           "keto_partition_generations_get: per generation goals, record_bytes_out, records_in, "
                           "value_bytes_back, device ms) and one 512-root Expand batch (keto_partition_levels_get: rows "
                           "fetched per level, walked on the device)",
                   "ranks": {str(k): v["phases"] for k, v in sorted(res.items())}}, f, indent=1)
    total = res[0]["total"]
    if SCALE == 40:
        assert total > 4_000_000_000  # configs[4]: C3 x40
    replicated = (WORLD - 1) * int(synth_meta(SCALE)["n_member_tuples"]) if REPL else 0
    assert sum(r["n_part"] for r in res.values()) == total + replicated  # the partitions cover the graph once
    for rank, r in res.items():
        print(rank, {k: v for k, v in r.items() if k != "phases"})
        assert r["det_mis"] == 0, r
        assert r["errors"] == 0, r
        assert r["dec_mis"] == 0 and r["err_mis"] == 0, r
        assert r["tree_mis"] == 0 and r["xerr"] == 0, r
        assert r["tree_nodes"] > ROOTS
        assert 0.2 < r["allowed"] < 0.8
        assert r["trunc_allowed"] < r["rest_allowed"]  # the truncation sub-batch really truncates
        assert r["exchange_bytes"] > 0
        assert r["x_build_s"] == 0  # Expand: no snapshot build
        assert r["routed"] > 0 or r["build_s"] == 0  # no build unless the closure path answered routed queries
