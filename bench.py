#!/usr/bin/env python3
"""Headline benchmark: batched permission Check (BASELINE.json metric: checks/sec + p99
batch latency) on MI355X.

Default workload = BASELINE configs[1] (C2: nested-group graph, 10M tuples, union-only,
max_read_depth 8, 2^20 queries per batch, 50% random-walk positives, 1% truncation
sub-batch); `--workload c3` = configs[2] (Drive-style folder tree, ~105M tuples, depth 10,
OPL union + intersection + exclusion through the rewrite interpreter).  One "step" = one
batch of 2^20 Checks through the whole device pipeline (resolve pre-pass -> interpreter
tiers -> decisions) with the queries already resident in HBM.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): every rank builds the same
replica (queries shard naturally); each rank checks its own
2^20-query batch per step, no collective on the data path; timing = max over ranks.
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "djy-keto_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(wl, queries, max_depth, max_width, budget_s=12.0):
    """The oracle (C restatement of the reference, oracle/refsem.c) on the host cores,
    on a bounded sample of the same batch -- reported beside the GPU, never the target."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refsem

    w = refsem.World(namespaces=wl.namespaces, strict=wl.strict, max_depth=max_depth, max_width=max_width)
    w.ns_names, w.rel_names, w.uuids = refsem.Interner(), refsem.Interner(), refsem.Interner()
    for n in wl.ns_names:
        w.ns_names(n)
    for r in wl.rel_names:
        w.rel_names(r)
    w._walk_names()
    t = np.zeros(len(wl.tuples), dtype=refsem.TUPLE_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("kind", "subj_kind"), ("sid", "s_obj"),
                 ("sns", "s_ns"), ("srel", "s_rel")):
        t[a] = wl.tuples[b]
    sb = wl.tuples["shard_id"]
    t["shard_hi"] = sb[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
    t["shard_lo"] = sb[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)
    orc = refsem.Oracle(w, t)
    del t
    q = np.zeros(len(queries), dtype=refsem.QUERY_DT)
    for a, b in (("ns", "ns"), ("obj", "obj"), ("rel", "rel"), ("kind", "subj_kind"), ("sid", "s_obj"),
                 ("sns", "s_ns"), ("srel", "s_rel"), ("depth", "max_depth")):
        q[a] = queries[b]
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))  # the GPU box grants 16 host cores per GPU
    n = 1 << 12
    while True:
        t0 = time.perf_counter()
        dec, err, st = orc.check_batch(q[:n], threads=cores)
        dt = time.perf_counter() - t0
        if dt * 2.5 > budget_s or n >= len(q):
            break
        n = min(len(q), int(n * max(2.0, min(8.0, budget_s / 2.5 / max(dt, 1e-3)))))
    orc.close()
    return {"value": n / dt, "unit": "checks/s", "cores": cores, "kind": "port",
            "sample": f"first {n} of the {len(q)}-query batch, oracle/refsem.c (C restatement of "
                      f"internal/check + persistence/sql read path), {cores} threads, {dt:.2f} s"}, dec


def job_rate(elapsed_local: float, units_local: int, device: str = "cpu"):
    """Whole-job rate over all ranks: units summed over ranks / the slowest rank's time
    (max over ranks).  Without an initialised process group: this rank alone."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return units_local / elapsed_local, elapsed_local, units_local
    t = torch.tensor([elapsed_local], dtype=torch.float64, device=device)
    u = torch.tensor([units_local], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    elapsed, units = float(t.item()), int(u.item())
    return units / elapsed, elapsed, units


def shard_seed(base: int, rank: int) -> int:
    """each rank checks its own seeded batch: the query stream shards by rank"""
    return base + rank


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2")
    ap.add_argument("--tuples", type=int, default=10_000_000, help="C2 graph size")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--latency-batch", type=int, default=1 << 16)
    ap.add_argument("--latency-iters", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl")
    import keto_mi355x as km
    from keto_mi355x import synth

    device = local
    t0 = time.perf_counter()
    if args.workload == "c2":
        wl = synth.nested_groups(args.tuples, seed=1)  # identical replica on every rank
    else:
        wl = synth.drive(seed=3)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict,
                       device=device)
    info = snap.info()
    log(f"[rank {rank}] snapshot: {info['n_tuples']} tuples, {info['n_nodes']} nodes, "
        f"{info['device_bytes'] / 2**20:.0f} MiB on device, build {info['build_seconds']:.2f}s "
        f"(total setup {time.perf_counter() - t0:.1f}s)")
    stream = km.Stream(device)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    # this rank's shard of the query stream: its own seeded 2^20 batch
    if args.workload == "c2":
        q = synth.nested_groups_queries(wl, args.batch, seed=shard_seed(7, rank))
    else:
        q = synth.drive_queries(wl, args.batch, seed=shard_seed(11, rank))
    union_only = not any("rewrite" in r for rels in wl.namespaces.values() for r in rels)
    dq = km.DeviceBuffer(device, q.nbytes)
    da = km.DeviceBuffer(device, len(q))
    de = km.DeviceBuffer(device, 4 * len(q))
    dq.upload(stream, q)

    # algorithmic bytes per launch: one counted batch outside the timed region
    stream.counters(reset=True)
    eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
    c = stream.counters(reset=True)
    pt = c["per_tier"]
    bytes_t0 = 8 * pt["rows"][0] + 4 * pt["edges"][0] + 8 * pt["probes"][0] + 17 * pt["queries"][0]
    allowed = da.download(stream, np.zeros(len(q), np.uint8))
    errs = de.download(stream, np.zeros(len(q), np.int32))
    assert (errs == 0).all(), "unexpected query errors"

    for _ in range(args.warmup):
        eng.check_batch_device(dq, len(q), da, de, sync=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    stream.sync()
    kms = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.check_batch_device(dq, len(q), da, de, sync=True)
        kms.append(stream.last_kernel_ms())
    stream.sync()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed_local = time.perf_counter() - t_start
    value, elapsed, total = job_rate(elapsed_local, args.batch * args.steps,
                                     f"cuda:{local}" if dist_on else "cpu")
    kernel_ms = float(np.mean(kms))

    # p99 batch latency over >= 100 batches of 64Ki queries (one rank's stream)
    # PCIe-inclusive rate (host buffers: H2D queries, kernels, D2H decisions) -- never `value`
    t1 = time.perf_counter()
    for _ in range(3):
        eng.check_batch(q)
    pcie_rate = 3 * len(q) / (time.perf_counter() - t1)

    lat = []
    nl = min(args.latency_batch, len(q))
    for i in range(args.latency_iters):
        off = (i * nl) % max(1, len(q) - nl + 1)
        ql = q[off:off + nl]
        dql = km.DeviceBuffer(device, ql.nbytes) if i == 0 else dql
        dql.upload(stream, ql)
        stream.sync()
        t1 = time.perf_counter()
        eng.check_batch_device(dql, nl, da, de, sync=True)
        lat.append(time.perf_counter() - t1)
    p99_ms = float(np.percentile(np.array(lat) * 1e3, 99)) if lat else None

    achieved = bytes_t0 / (kernel_ms * 1e-3) / 1e9
    kname = "check_union_kernel" if union_only else "check_kernel"
    traffic = None  # HBM bytes per tier-0 launch from the committed PMC passes (tools/pmc_traffic.sh)
    tf = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{args.workload}.json")))
    if tf:
        t = json.load(open(tf[-1]))
        if kname in t.get("kernel", "") and int(t.get("grid", 0)) > 0:
            traffic = t["traffic_bytes_per_launch"]
    out = {
        "metric": "checks/sec (node) + p99 batch latency, 1B-tuple depth-10 graph, 1/2/4/8 GPU",
        "value": value,
        "unit": "checks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded PCG64 %s, BASELINE config %d)" % (
            ("nested-group graph", 2) if args.workload == "c2" else ("Drive-style folder tree", 3)),
        "config": {"workload": (f"C2 nested groups: {info['n_tuples']} tuples, 5 levels, union-only, max_read_depth 8, "
                                f"{args.batch} checks/batch/GPU, 50% random-walk positives, 1% depth 1-4")
                   if args.workload == "c2" else
                   (f"C3 Drive-style: {info['n_tuples']} tuples, fanout 5, depth 10, view = (viewers | editors | "
                    f"owners | parents.traverse(view)) & !banned, max_read_depth 16, {args.batch} checks/batch/GPU"),
                   "tuples": int(info["n_tuples"]), "batch_per_gpu": args.batch,
                   "parallelism": f"replica x{world} (query batch sharded, no data-path collective)"},
        "p99_batch_latency_ms": p99_ms,
        "latency_batch": nl,
        "allowed_fraction": float(allowed.mean()),
        "pcie_inclusive_checks_per_s": pcie_rate,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname + " (tier 0)", "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": int(bytes_t0),
                     "bytes_model": "8*rows + 4*edges + 8*probes + 17*queries (BASELINE.md)",
                     "work": {"rows": pt["rows"][0], "edges": pt["edges"][0], "probes": pt["probes"][0],
                              "queries_tier0": pt["queries"][0], "queries_tier1": pt["queries"][1],
                              "queries_tier2": pt["queries"][2]}},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, dec = cpu_baseline(wl, q, wl.max_depth, wl.max_width, args.cpu_budget)
        out["cpu_baseline"] = cb
        ns = len(dec)
        out["cpu_parity_sample"] = {"n": ns, "mismatches": int((dec != allowed[:ns]).sum())}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
