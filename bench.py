#!/usr/bin/env python3
"""Headline benchmark: batched permission Check (BASELINE.json metric: checks/sec + p99
batch latency, 1B-tuple depth-10 graph) on MI355X.

Workloads:
  c4 (default) = configs[3]: Drive-style folder forest x10 -- ~1.05B tuples, fanout 5,
      depth 10, OPL union + intersection + exclusion through the rewrite interpreter,
      max_read_depth 16.  The configuration the metric is quoted on; it fits one GPU.
  c3 = configs[2]: the same forest x1 (~105M tuples).
  c2 = configs[1]: nested-group graph, 10M tuples, union-only, max_read_depth 8.
  c5 = configs[4]: the forest x40 (~4.2B tuples) partitioned by object over the ranks;
      per batch a closure exchange over RCCL, a device build of the closure, then Check.
One "step" = one batch of 2^20 Checks per GPU through the whole device pipeline (resolve
pre-pass -> interpreter tiers -> decisions) with the queries already resident in HBM.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): the graph is replicated on every GPU
and the query stream shards by rank (no collective on the data path).  For c3/c4 rank 0
generates the tuples and broadcasts them over RCCL/xGMI; every rank builds its replica on its
own device (keto_snapshot_build_device).  Timing = max over ranks; value = all ranks' checks
/ that time.
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "djy-keto_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "checks/sec (node) + p99 batch latency, 1B-tuple depth-10 graph, 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))  # the GPU box grants 16 host cores per GPU


def lib_sha256():
    import keto_mi355x._abi as abi
    with open(abi.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def committed_traffic(workload: str, kname: str):
    """HBM bytes per tier-0 launch from the newest committed PMC passes (tools/gpu_round.sh OUT traffic ->
    profiles/r*_traffic_<workload>.json) -- only if they profiled THIS library build (sha256 of
    libketo_mi355x.so); a kernel change makes the figure stale and it is dropped (null)."""
    tf = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{workload}.json")))
    if not tf:
        return None, "no PMC profile committed"
    t = json.load(open(tf[-1]))
    if kname not in t.get("kernel", "") or int(t.get("grid", 0)) <= 0:
        return None, f"{os.path.basename(tf[-1])} profiled another kernel"
    if t.get("lib_sha256") != lib_sha256():
        return None, f"{os.path.basename(tf[-1])} profiled another build of libketo_mi355x.so"
    return t["traffic_bytes_per_launch"], os.path.basename(tf[-1])


def schedule_report(orc, q, gpu_allowed, n: int, cores: int):
    """the oracle's schedule-sensitivity flags (refsem.h rs_check_ex) on the
    first n queries of the batch, and the GPU's agreement with the canonical answer on them"""
    import refsem

    n = min(n, len(q))
    dec, err, flags, _ = orc.check_batch_ex(q[:n], threads=cores)
    sens = (flags & refsem.F_SENSITIVE) != 0
    diff = (flags & refsem.F_SEQ_DIFFERS) != 0
    return {"n": int(n), "flagged": int(sens.sum()), "flagged_frac": float(sens.mean()),
            "sequential_schedule_differs": int(diff.sum()),
            "gpu_mismatches_on_flagged": int((dec[sens] != gpu_allowed[:n][sens]).sum()),
            "gpu_mismatches": int((dec != gpu_allowed[:n]).sum()),
            "flagged_by_maximal_exploration": int(((flags & refsem.F_MAXEXP) != 0).sum()),
            "criterion": "a visited scope reached a key twice and saw width truncation / an error / AND-NOT, or "
                         "reached it at different rest depths plus depth truncation -- in either simulated "
                         "schedule or in the tree of every check the reference's eager construction can start "
                         "(oracle/refsem.c); sound against oracle/refconc.py's goroutine-level interleavings "
                         "(tests/test_schedule.py)"}


SQL_MAX_ROWS = 2_000_000  # per worker: the rows become Python tuples before they reach SQLite


_SQL_CTX = None  # (oracle, workload, max_depth, max_width): inherited by the forked workers, never pickled


def _sql_worker(q):
    """one host core of the SQL-mode baseline: load the rows its queries can read into an
    in-memory SQLite store (untimed), then run the restated engine (oracle/refsql.py).  On a
    graph where the sample's closure exceeds SQL_MAX_ROWS the share is halved until it fits."""
    orc, wl, max_depth, max_width = _SQL_CTX
    import refsql
    while True:
        rows = refsql.closure_rows(orc, q["ns"], q["obj"], max_depth + 1, max_rows=SQL_MAX_ROWS)
        if rows is not None or len(q) <= 1:
            break
        q = q[: len(q) // 2]
    if rows is None:
        return np.zeros(0, np.uint8), 0.0, 0, 0
    eng = refsql.SqlEngine(rows, wl.namespaces, wl.ns_names, wl.rel_names, max_depth=max_depth, max_width=max_width,
                           strict=wl.strict)
    dec = np.zeros(len(q), np.uint8)
    t0 = time.perf_counter()
    for i, r in enumerate(q):
        subj = (0, int(r["sid"])) if r["kind"] == 0 else (1, wl.ns_names[r["sns"]], int(r["sid"]), wl.rel_names[r["srel"]])
        m, e = eng.check(wl.ns_names[r["ns"]], int(r["obj"]), wl.rel_names[r["rel"]], subj, int(r["depth"]))
        dec[i] = e == 0 and m == refsql.IS_MEMBER
    return dec, time.perf_counter() - t0, eng.statements, len(rows)


def sql_baseline(orc, wl, q, max_depth, max_width, cores, per_core=512):
    """"restated reference (SQL mode)": the engine recursion issuing the reference's four read
    statements per hop (traverser.go:68-92,146-154; relationtuples.go:216-227,253-260) against
    in-memory SQLite -- the cost model of Keto with its in-memory SQLite persister -- on the
    host cores, one process per core, each over the rows its share of the sample can read
    (per_core queries each: a few seconds in all, store loading included)"""
    import multiprocessing as mp
    global _SQL_CTX
    n = min(len(q), per_core * cores)
    parts = [np.ascontiguousarray(q[i:n:cores]) for i in range(cores)]
    _SQL_CTX = (orc, wl, max_depth, max_width)  # the workers fork with it: only the query shares travel
    try:
        with mp.get_context("fork").Pool(cores) as pool:
            res = pool.map(_sql_worker, parts)
    finally:
        _SQL_CTX = None
    dt = max(r[1] for r in res)
    done = sum(len(r[0]) for r in res)
    if done < n:  # some shares were cut to fit SQL_MAX_ROWS: the first len(share) of each
        n = done
        dec = np.concatenate([r[0] for r in res])
        parity_idx = np.concatenate([np.arange(i, i + cores * len(r[0]), cores)[:len(r[0])] for i, r in enumerate(res)])
    else:
        dec = np.zeros(n, np.uint8)
        for i in range(cores):
            dec[i:n:cores] = res[i][0]
        parity_idx = np.arange(n)
    stmts = sum(r[2] for r in res)
    sql_baseline.parity_idx = parity_idx
    return {"value": n / dt, "unit": "checks/s", "cores": cores, "kind": "port",
            "label": "restated reference (SQL mode)",
            "sample": f"{n} queries of the {len(q)}-query batch (a strided sample; each process's share cut to "
                      f"closures of <= {SQL_MAX_ROWS} rows), oracle/refsql.py: the engine recursion issuing the "
                      f"reference's 4 SQL statements per hop against in-memory SQLite (python sqlite3 "
                      f"{__import__('sqlite3').sqlite_version}), {cores} processes, slowest {dt:.2f} s; "
                      f"{stmts / n:.1f} statements/check; store = the {sum(r[3] for r in res)} rows the sample can "
                      f"read (loaded untimed)"}, dec


def cpu_baseline(wl, queries, max_depth, max_width, budget_s=12.0, gpu_allowed=None, pipe=None, pipe_per_batch=4096):
    """The oracle (C restatement of the reference, oracle/refsem.c) on the host cores, on a
    bounded sample of the same batch over the same graph -- reported beside the GPU, never
    the target.  The oracle indexes the engine's tuple records in place (no copy).  pipe: the
    timed pipelined batches [(queries, gpu decisions)]: a strided sample of each is checked by the
    same oracle (cpu_baseline.pipe)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refsem

    w = refsem.World(namespaces=wl.namespaces, strict=wl.strict, max_depth=max_depth, max_width=max_width)
    w.ns_names, w.rel_names, w.uuids = refsem.Interner(), refsem.Interner(), refsem.Interner()
    for n in wl.ns_names:
        w.ns_names(n)
    for r in wl.rel_names:
        w.rel_names(r)
    w._walk_names()
    cores = cpu_threads()
    t0 = time.perf_counter()
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    build_s = time.perf_counter() - t0
    q = np.ascontiguousarray(queries).view(refsem.QUERY_DT)
    n = 1 << 12
    while True:
        t0 = time.perf_counter()
        dec, err, st = orc.check_batch(q[:n], threads=cores)
        dt = time.perf_counter() - t0
        if dt * 2.5 > budget_s or n >= len(q):
            break
        n = min(len(q), int(n * max(2.0, min(8.0, budget_s / 2.5 / max(dt, 1e-3)))))
    log(f"cpu baseline: {n} checks in {dt:.2f}s on {cores} threads (index {build_s:.1f}s)")
    sched = None
    if gpu_allowed is not None:
        t0 = time.perf_counter()
        sched = schedule_report(orc, q, gpu_allowed, max(1 << 12, min(n, 1 << 16)), cores)
        log(f"schedule report ({sched['n']} queries): {time.perf_counter() - t0:.1f}s")
    cpu_baseline.pipe = None
    if pipe:
        t0 = time.perf_counter()
        mis = n_chk = 0
        for qk, ak in pipe:
            idx = np.arange(0, len(qk), max(1, len(qk) // pipe_per_batch))
            d_, _, _ = orc.check_batch(np.ascontiguousarray(qk[idx]).view(refsem.QUERY_DT), threads=cores)
            mis += int((d_ != ak[idx]).sum())
            n_chk += len(idx)
        cpu_baseline.pipe = {"n": n_chk, "batches": len(pipe), "mismatches": mis,
                             "what": f"a strided sample (every {max(1, len(pipe[0][0]) // pipe_per_batch)}th query) of "
                                     "each timed pipelined batch, decided by oracle/refsem.c over the whole graph",
                             "seconds": time.perf_counter() - t0}
        log(f"pipelined batches vs the oracle: {n_chk} queries, {mis} mismatches ({time.perf_counter() - t0:.1f}s)")
    sql = None
    try:
        t0 = time.perf_counter()
        sql, sdec = sql_baseline(orc, wl, q, max_depth, max_width, cores)
        idx = sql_baseline.parity_idx
        ok = idx < len(dec)
        sql["parity_vs_port"] = {"n": int(ok.sum()), "mismatches": int((sdec[ok] != dec[idx[ok]]).sum())}
        log(f"sql-mode baseline: {sql['value']:.0f} checks/s ({time.perf_counter() - t0:.1f}s)")
    except Exception as e:  # reported, never fatal to the bench line
        sql = {"error": repr(e)}
    orc.close()
    cpu_baseline.sql = sql
    return sched, {"value": n / dt, "unit": "checks/s", "cores": cores, "kind": "port",
            "sample": f"first {n} of the {len(q)}-query batch over the full {len(wl.tuples)}-tuple graph, "
                      f"oracle/refsem.c (C restatement of internal/check + persistence/sql read path), "
                      f"{cores} threads, {dt:.2f} s (index build {build_s:.1f} s, untimed)"}, dec


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


def broadcast_tuples(host_tuples, n_bytes: int, device: int, rank: int):
    """rank 0's tuple records -> a uint8 tensor on every rank's GPU (RCCL broadcast over xGMI,
    in 1 GiB pieces)."""
    import torch
    import torch.distributed as dist

    buf = torch.empty(n_bytes, dtype=torch.uint8, device=f"cuda:{device}")
    if rank == 0:
        buf.copy_(torch.from_numpy(host_tuples.view(np.uint8).reshape(-1)))
    piece = 1 << 30
    for off in range(0, n_bytes, piece):
        dist.broadcast(buf[off:off + piece], src=0)
    torch.cuda.synchronize(device)
    return buf


def build_workload(name, rank, world, device, args):
    import keto_mi355x as km
    from keto_mi355x import synth

    t0 = time.perf_counter()
    if name == "c2":
        wl = synth.nested_groups(args.tuples, seed=1)  # cheap: every rank generates its replica
        snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict,
                           device=device)
        return wl, snap, time.perf_counter() - t0
    scale = 10 if name == "c4" else 1
    wl = synth.drive_scaled(scale, materialize=(rank == 0))
    if world == 1:
        snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict,
                           device=device)
    else:
        import torch

        nt = wl.meta["n_tuples"]
        buf = broadcast_tuples(wl.tuples, nt * km.TUPLE_DT.itemsize, device, rank)
        snap = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict,
                           device=device, device_tuples=(buf.data_ptr(), nt))
        del buf
        torch.cuda.empty_cache()
    return wl, snap, time.perf_counter() - t0


def expand_probe(km, snap, wl, stream, n: int = 4096, reps: int = 5):
    """Batched Expand (configs[4]'s "4096 Expand queries per batch"): n subject-set roots (half
    Group#members, half Folder#viewers) per batch, host buffers in and out, both kernel passes
    (count, emit) included.  Bytes model 8*rows + 4*edges + 12*out_nodes."""
    rng = np.random.default_rng(5)
    r = np.zeros(n, dtype=km.SUBJSET_DT)
    h = n // 2
    r["ns"][:h], r["rel"][:h] = 1, wl.rel_names.index("members")
    r["obj"][:h] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], h)
    r["ns"][h:], r["rel"][h:] = 2, wl.rel_names.index("viewers")
    r["obj"][h:] = rng.integers(0, wl.meta["folders_per_root"], n - h)
    xe = km.ExpandEngine(snap, stream, max_read_depth=wl.max_depth)
    nodes, offs, err = xe.build_trees(r)  # warm-up (sizes the output buffer)
    # the API into pageable numpy memory, then into pinned memory (keto_host_alloc: the trees'
    # one D2H runs as a straight DMA) -- what a Go shim gets with C.malloc vs keto_host_alloc
    t0 = time.perf_counter()
    for _ in range(reps):
        xe.build_trees(r)
    dt_pageable = (time.perf_counter() - t0) / reps
    pin = km.PinnedArray(int(offs[n]) * 5 // 4 + 64, km.TREE_DT)
    xe.build_trees(r, out=pin)
    stream.counters(reset=True)
    stream.expand_time(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        nodes, offs, err = xe.build_trees(r, out=pin)
    dt = (time.perf_counter() - t0) / reps
    nodes = nodes.copy()
    c = stream.counters(reset=True)
    ms, nb = stream.expand_time(reset=True)
    kms = ms / max(1, nb)
    # keto_expand_batch_spans into the same pinned buffer: each tree written as its walk ends, the
    # copy-out overlapping the other walks; the same trees (checked root by root)
    xe.build_trees_spans(r, out=pin)
    t0 = time.perf_counter()
    for _ in range(reps):
        sn, first, count, serr = xe.build_trees_spans(r, out=pin)
    dt_spans = (time.perf_counter() - t0) / reps
    stream.counters(reset=True)
    stream.expand_time(reset=True)
    spans_mis = int((serr != err).sum()) + sum(
        0 if np.array_equal(sn[int(first[i]):int(first[i]) + int(count[i])], nodes[int(offs[i]):int(offs[i + 1])]) else 1
        for i in range(n))
    pin.free()
    # algorithmic bytes: 8*rows + 4*edges + 12*out_nodes per batch
    xbytes = (8 * c["rows"] + 4 * c["edges"] + 12 * c["out_nodes"]) / reps
    return {"roots_per_batch": n, "ms_per_batch": dt * 1e3, "ms_per_batch_pageable_out": dt_pageable * 1e3,
            "ms_per_batch_spans": dt_spans * 1e3, "spans_tree_mismatches": spans_mis,
            "trees_per_s": n / dt, "nodes_per_batch": int(offs[n]),
            "errors": int((err != 0).sum()), "max_read_depth": wl.max_depth,
            "traversal_kernel_ms": kms,
            "roofline": {"bound": "hbm", "achieved": xbytes / (kms * 1e-3) / 1e9 if kms else None, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": xbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS if kms else None,
                         "algorithmic_bytes_per_batch": xbytes,
                         "bytes_model": "8*rows + 4*edges + 12*out_nodes (SURVEY.md 8.1 (d))",
                         "kernel": "expand_wave (wave per root, one traversal) + fallback count pass if any"},
            "note": "ms_per_batch: host roots in, trees out into pinned host memory (API form, root order) incl. "
                    "PCIe; ms_per_batch_spans: keto_expand_batch_spans into the same pinned memory (completion "
                    "order, each tree written over PCIe as its walk ends; trees compared root by root with "
                    "ms_per_batch's); ms_per_batch_pageable_out: the same into pageable memory; traversal_kernel_ms: HIP events "
                    "around the traversal on the engine stream; roots: Group#members and Folder#viewers"}


def synth_new_files(wl, ids, parents, rng):
    from keto_mi355x import synth
    return synth.drive_new_files(wl, ids, parents, rng)


def store_probe(km, wl, q, n_ins: int = 600, n_del: int = 400):
    """Incremental snapshots at the workload's size: the graph in a
    device tuple store (keto_store_*), a TransactRelationTuples of n_ins + n_del rows (new ACL rows
    on existing objects, deletes of stored rows), then the new version cut two ways -- by patching
    a copy of the previous snapshot (keto_store_snapshot_patch: O(graph) copies, the base stays
    valid) and by advancing the previous snapshot in place (keto_store_snapshot_advance: work in
    proportion to the touched rows) -- timed beside the full device build of the same version and
    checked against it on the bench's query batch; then a second transaction creating 100 new
    files, advanced in place too."""
    import torch

    rng = np.random.default_rng(21)
    t = wl.tuples
    t0 = time.perf_counter()
    st = km.TupleStore(t)
    load_s = time.perf_counter() - t0
    base = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict, store=st)
    ins = t[rng.choice(len(t), n_ins, replace=False)].copy()
    acl = (ins["ns"] >= 2) & (ins["rel"] != wl.rel_names.index("parents"))
    ins["subj_kind"][acl], ins["s_ns"][acl], ins["s_rel"][acl] = 0, 0, 0
    ins["s_obj"][acl] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], int(acl.sum()))
    ins["shard_id"] = rng.integers(0, 256, (n_ins, 16), dtype=np.uint8)
    dele = t[rng.choice(len(t), n_del, replace=False)].copy()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.transact(ins, dele)
    transact_ms = (time.perf_counter() - t0) * 1e3

    def checks(snap, qq):
        return km.CheckEngine(snap, max_read_depth=wl.max_depth, max_read_width=wl.max_width).check_batch(qq)

    # the copy patch (base untouched), then the in-place advance of base to the same version
    t0 = time.perf_counter()
    patched = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict, store=st,
                          base=base)
    patch_ms = (time.perf_counter() - t0) * 1e3
    was_patched = patched.patched
    res_patch = checks(patched, q)
    pi = patched.info()
    patched.close()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    advanced = base.advance(st)
    advance_ms = (time.perf_counter() - t0) * 1e3
    res_adv = checks(base, q)
    ai = base.info()
    # a second transaction creates objects (verdict r3: Keto's most common write is a new file):
    # 100 new files, a parent tuple + 9 ACL rows each, ids past the graph's -- advanced in place
    # onto the snapshot's spare entities
    n_new = 100
    new_ids = wl.n_uuids + np.arange(n_new)
    ins2 = synth_new_files(wl, new_ids, rng.integers(0, wl.meta["n_folders"], n_new), rng)
    n_uuids2 = wl.n_uuids + n_new
    st.transact(ins2, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    advanced2 = base.advance(st)
    advance2_ms = (time.perf_counter() - t0) * 1e3
    q2 = q.copy()
    k = min(len(q2), 1 << 16)  # view / edit of the new files by random users
    q2["ns"][:k], q2["obj"][:k] = wl.ns_names.index("File"), rng.choice(new_ids, k)
    q2["rel"][:k] = rng.choice([wl.rel_names.index("view"), wl.rel_names.index("edit")], k)
    q2["subj_kind"][:k], q2["s_ns"][:k], q2["s_rel"][:k], q2["max_depth"][:k] = 0, 0, 0, 0
    q2["s_obj"][:k] = wl.meta["ubase"] + rng.integers(0, wl.meta["n_users"], k)
    res2 = [checks(base, q2)]
    new_objs = {"transaction_rows": int(len(ins2)), "new_files": n_new, "advanced": advanced2, "advance_ms": advance2_ms,
                "new_file_checks_allowed": float(res2[0][0][:k].mean())}
    base.close()  # (device memory: the full builds of the same versions come next)
    t0 = time.perf_counter()
    full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, n_uuids2, strict=wl.strict, store=st)
    full_ms = (time.perf_counter() - t0) * 1e3
    res2.append(checks(full, q2))
    new_objs["checks_vs_full_build"] = {"n": int(len(q2)), "mismatches": int((res2[0][0] != res2[1][0]).sum()
                                                                           + (res2[0][1] != res2[1][1]).sum())}
    # version 1 against a full build of it: the store without the second transaction's rows
    st.transact(None, ins2)
    full.close()
    full = km.Snapshot(wl.namespaces, None, wl.ns_names, wl.rel_names, n_uuids2, strict=wl.strict, store=st)
    res_full = checks(full, q)
    fi = full.info()

    def mism(a):
        return int((a[0] != res_full[0]).sum() + (a[1] != res_full[1]).sum())

    out = {"transaction_rows": n_ins + n_del, "advanced": advanced, "advance_ms": advance_ms,
           "patched": was_patched, "patch_ms": patch_ms, "full_build_ms": full_ms,
           "new_objects": new_objs,
           "transact_ms": transact_ms, "store_load_s": load_s, "version": int(ai["version"]),
           "n_tuples_equal": pi["n_tuples"] == fi["n_tuples"] == ai["n_tuples"],
           "checks_vs_full_build": {"n": int(len(q)), "mismatches_advanced": mism(res_adv), "mismatches_patched": mism(res_patch)},
           "what": "keto_store_transact of the rows; then the version cut by keto_store_snapshot_patch of the previous "
                   "snapshot (a copy, base untouched) and by keto_store_snapshot_advance of the previous snapshot in "
                   "place (host API call to a usable snapshot each); full_build_ms: keto_store_snapshot of the same "
                   "version; new_objects: a second transaction creating 100 files, advanced in place"}
    full.close()
    st.close()
    torch.cuda.empty_cache()
    return out


def serving_probe(km, snap, q, wl, clients: int, req: int, seconds: float):
    """Closed-loop serving load through the coalescing dispatcher (keto_dispatcher_*): `clients`
    native threads (synth.closed_loop, C++) each send `req`-query requests back to back, the way
    the Go shim's goroutines call it through cgo.  Reported beside the batch numbers; the
    per-request latency includes the queueing a request sees behind the batch in flight."""
    from keto_mi355x import synth

    d = km.Dispatcher(snap, wl.max_depth, wl.max_width, max_batch=1 << 16)
    r = synth.closed_loop(d, q, clients, req, seconds)
    st = d.stats()
    d.close()
    return {"clients": clients, "request_checks": req, "seconds": r["seconds"],
            "checks_per_s": r["checks"] / r["seconds"], "requests_per_s": r["requests"] / r["seconds"],
            "mean_batch": st["queries"] / max(1, st["batches"]),
            "p50_request_ms": r["p50_ms"], "p99_request_ms": r["p99_ms"], "max_request_ms": r["max_ms"],
            "host_client": "native closed loop: C++ threads calling keto_dispatcher_check"}


def c5_cpu_baseline(wl, q, budget_s: float):
    """configs[4]'s CPU side: the oracle (oracle/refsem.c) over the closure of a sample of the
    batch, computed on the host from the generator's own rows (tests/closure_ref.py with
    synth.drive_object_tuples) -- the graph itself is never held on the host.  Returns the
    baseline record and (sample indices, decisions) for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refsem
    from closure_ref import closure
    from keto_mi355x import synth
    from product_helpers import world_from_workload

    cores = cpu_threads()
    n = 1 << 11
    while True:
        qs = q[:n]
        ct = closure(lambda k: synth.drive_object_tuples(wl, k), qs["ns"], qs["obj"], wl.max_depth + 1,
                     subjects=qs["s_obj"][qs["subj_kind"] == 0])
        w, _ = world_from_workload(wl, with_tuples=False)
        orc = refsem.Oracle(w, ct.view(refsem.TUPLE_DT), shard_bytes=True)
        orc.set_limits(wl.max_depth, wl.max_width)
        t0 = time.perf_counter()
        dec, _, _ = orc.check_batch(qs.view(refsem.QUERY_DT), threads=cores)
        dt = time.perf_counter() - t0
        orc.close()
        if dt * 2.5 > budget_s or n >= len(q):
            break
        n = min(len(q), int(n * max(2.0, min(8.0, budget_s / 2.5 / max(dt, 1e-3)))))
    return {"value": n / dt, "unit": "checks/s", "cores": cores, "kind": "port",
            "sample": f"first {n} queries of rank 0's batch, oracle/refsem.c over their closure ({len(ct)} tuples, "
                      f"generated from the Drive generator's rows on the host: the x{wl.meta['roots']} graph is never "
                      f"held whole), {cores} threads, {dt:.2f} s (closure + index untimed)"}, dec


def run_c5(args, rank, world, device, dist_on):
    """configs[4]: a graph partitioned by object over the ranks (keto_partition_*).  Every rank's
    partition is built once into a resident snapshot; one step = one batch of this rank's Checks:
    several ranks run the distributed frontier (csrc/frontier_dist.hip: goal records to the nodes'
    owners and values back, one all-to-all each per generation), one rank the engine on its
    resident snapshot (the whole graph).  KETO_PART_CLOSURE=1: the per-batch closure path instead
    (closure exchange -> closure snapshot build -> the Check kernels).  Ranks sharing one GPU
    (KETO_BENCH_BACKEND=gloo, a rehearsal) build their partitions one after another
    (KETO_PART_STAGED)."""
    import torch

    import keto_mi355x as km
    from keto_mi355x import partition, synth

    t0 = time.perf_counter()
    wl = synth.drive_scaled(args.scale, materialize=False)
    coll = None
    if dist_on:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from torch_collective import TorchCollective  # keto_collective over the job's process group
        coll = TorchCollective(device_buffers=True)  # (RCCL: the exchange moves GPU to GPU)
    shared = os.environ.get("KETO_BENCH_BACKEND", "nccl") == "gloo"
    if dist_on and shared:
        os.environ["KETO_PART_STAGED"] = "1"  # (created in turn: the slot layout is checked at the first batch)
    eng, n_part = None, 0
    for r in range(world if (dist_on and shared) else 1):
        if not (dist_on and shared) or r == rank:
            place = (synth.drive_placement(wl, replicate_groups=args.placement == "tree_repl")
                     if args.placement != "hash" else None)
            part = synth.drive_partition(wl, world, rank, placement=place)
            n_part = len(part)
            eng = partition.PartitionedEngine(wl.namespaces, wl.ns_names, wl.rel_names, wl.n_uuids, part,
                                              device=device, max_read_depth=wl.max_depth,
                                              max_read_width=wl.max_width, collective=coll, placement=place)
            del part
        if dist_on and shared:
            import torch.distributed as dist
            dist.barrier()
    setup_s = time.perf_counter() - t0
    log(f"[rank {rank}] partition {rank}/{world}: {n_part} of {wl.meta['n_tuples']} tuples, setup {setup_s:.1f}s")
    q = synth.drive_queries(wl, args.batch, seed=shard_seed(11, rank))
    # algorithmic bytes: one counted batch (the check kernels' reference-traversal counters) plus
    # the closure it moved
    allowed, err = eng.check_batch(q, count_work=True)
    assert (err == 0).all(), "unexpected query errors"
    cw = eng.last_work
    closure_tuples = eng.last["tuples"]
    for _ in range(max(0, args.warmup - 1)):
        eng.check_batch(q)
    if dist_on:
        import torch.distributed as dist
        dist.barrier()
    # one batch per call, phase by phase (closure -> build -> check; the distributed frontier: its
    # device time and the time inside the collective): where a batch's time goes
    phases = {"closure_s": 0.0, "build_s": 0.0, "run_s": 0.0, "device_s": 0.0, "exchange_s": 0.0}
    n_seq = min(args.steps, 4)
    torch.cuda.synchronize()
    t_seq = time.perf_counter()
    for _ in range(n_seq):
        eng.check_batch(q)
        for k in phases:
            phases[k] += eng.last[k]
    dist_last = dict(eng.last)
    dist_levels = eng.generation_stats()
    seq_ms = (time.perf_counter() - t_seq) / n_seq * 1e3
    # the timed region: K fresh seeded batches through one keto_partition_check_many call, in
    # pinned host memory as the C4 line's (keto_host_alloc: straight DMA for the one-rank path)
    pin_q = [km.PinnedArray(args.batch, km.QUERY_DT) for _ in range(args.steps)]
    pin_o = [(km.PinnedArray(args.batch, np.uint8), km.PinnedArray(args.batch, np.int32)) for _ in range(args.steps)]
    for s_, pq in enumerate(pin_q):
        pq.array[:] = q if s_ == 0 else synth.drive_queries(wl, args.batch, seed=shard_seed(11 + 1000 * s_, rank))
    batches = [pq.array for pq in pin_q]
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    outs = eng.check_batches(batches, outs=[(a.array, e.array) for a, e in pin_o])
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed_local = time.perf_counter() - t_start
    pipe_vs_first = int((outs[0][0] != allowed).sum())
    # every distinct timed batch again, counted (the DFS interpreter on the same closure / snapshot)
    pipe_vs_dfs = 0
    for b, (a, _) in zip(batches, outs):
        a2, _ = eng.check_batch(b, count_work=True)
        pipe_vs_dfs += int((a2 != a).sum())
    levels_detail = eng.level_stats()
    value, elapsed, total = job_rate(elapsed_local, args.batch * args.steps, f"cuda:{device}" if dist_on else "cpu")
    ranks_ms = per_rank_ms(elapsed_local / args.steps * 1e3, f"cuda:{device}" if dist_on else "cpu")
    ms_step = elapsed_local / args.steps * 1e3
    # roofline of the step (this rank): the check's algorithmic bytes (BASELINE.md model, counted
    # by the DFS interpreter on the batch's closure snapshot) + on the closure path the closure the
    # step moves (each tuple gathered -- read + written -- and read by the build: 3 x 48 B), over
    # the whole step's time
    check_bytes = 8 * cw["rows"][0] + 4 * cw["edges"][0] + 8 * cw["probes"][0] + 17 * cw["queries"][0]
    step_bytes = check_bytes + 3 * 48 * closure_tuples
    achieved = step_bytes / (ms_step * 1e-3) / 1e9
    distributed = world > 1 and os.environ.get("KETO_PART_CLOSURE") is None
    resident = world == 1 and os.environ.get("KETO_PART_CLOSURE") is None
    if distributed:  # the counted batch ran on the closure path: the step itself moves goal records, no tuples
        step_bytes = check_bytes
        achieved = step_bytes / (ms_step * 1e-3) / 1e9
    how = ("one rank: the partition is the whole graph, built once into a resident snapshot -- no closure, no "
           "per-batch build" if resident else
           "resident partitions, distributed frontier: goal records to their nodes' owners and values back, one "
           "all-to-all each per generation -- no closure, no per-batch build" if distributed else
           f"closure of max_read_depth+1 = {eng.levels()} levels per batch")
    out = {
        "metric": METRIC, "value": value, "unit": "checks/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "per_rank_ms_per_step": ranks_ms,
        "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (seeded Drive-style folder forest, BASELINE config 5; generated per partition)",
        "config": {"workload": f"C5 Drive-style x{args.scale}: {wl.meta['n_tuples']} tuples partitioned by "
                               f"object over {world} rank(s), {args.batch} checks/batch/GPU, {how}",
                   "tuples": int(wl.meta["n_tuples"]), "batch_per_gpu": args.batch, "placement": args.placement,
                   "parallelism": f"object partition x{world} (" + ("RCCL all-to-all of goal records per generation" if distributed
                                                                      else "RCCL all-to-all closure exchange per level") + ")"},
        "allowed_fraction": float(allowed.mean()),
        "phases_ms_per_step": {k: v / n_seq * 1e3 for k, v in phases.items()},
        "pipeline": {"what": ("value: the K timed fresh batches (pinned host memory) in one keto_partition_check_many "
                              "call -- " + ("one rank: each batch's H2D + check path + D2H enqueued on the engine stream "
                                            "(KETO_F_ASYNC, two copy streams), one synchronisation at the end"
                                            if resident else
                                            "batch k+1's closure (its query upload included) on a helper thread beside "
                                            "batch k's remap, build and check") +
                              "; phases_ms_per_step and sequential_ms_per_step: one batch (the counted one) again and "
                              "again, one call at a time (warm caches: not comparable with value)"),
                     "sequential_ms_per_step": seq_ms, "distinct_batches": len(batches),
                     "first_batch_vs_counted_mismatches": pipe_vs_first,
                     "mismatches": pipe_vs_dfs,
                     "mismatches_what": "every distinct timed batch vs a counted rerun of it (DFS interpreter)"},
        "closure": {"tuples": eng.last["tuples"], "objects": eng.last["objects"], "levels": eng.last["levels"],
                    "bytes_sent": eng.last["bytes_sent"],
                    "partition_tuples": n_part, "levels_detail": levels_detail},
        "distributed": ({k: dist_last[k] for k in ("generations", "goals", "routed", "exchange_bytes", "device_s",
                                                    "exchange_s", "run_s")} | {"generations_detail": dist_levels}
                        if distributed else None),
        "shared_gpu": bool(dist_on and shared),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": ("the whole step: H2D + check path + D2H on the resident snapshot" if resident else
                                "the whole step of this rank: its generations' kernels, the exchanges and waits"
                                if distributed else "the whole step: closure exchange + closure build + check (one rank)"),
                     "algorithmic_bytes_per_step": int(step_bytes), "check_bytes": int(check_bytes),
                     "closure_tuples": int(closure_tuples),
                     "bytes_model": ("8*rows + 4*edges + 8*probes + 17*queries (check; the goal records and values "
                                     "the step exchanges are in distributed.exchange_bytes)" if distributed or resident else
                                     "8*rows + 4*edges + 8*probes + 17*queries (check) + 3*48*closure tuples")},
        "cpu_baseline": None,
    }
    if rank == 0 and not args.no_cpu_baseline:
        cb, dec = c5_cpu_baseline(wl, q, args.cpu_budget)
        out["cpu_baseline"] = cb
        out["cpu_parity_sample"] = {"n": len(dec), "mismatches": int((dec != allowed[:len(dec)]).sum())}
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising HIP (torch.cuda.device_count()
    does not on this image), so the launcher can still start fresh children afterwards"""
    import torch
    return int(torch.cuda.device_count())


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` (N > 1) without torchrun: N fresh child processes, one per GPU, each
    one rank of an RCCL job (RANK / LOCAL_RANK / WORLD_SIZE, MASTER_ADDR 127.0.0.1).  Nothing in
    this process touches the GPU; it waits for the children and exits with the worst status.
    Fewer visible GPUs than N is an error, never a silent 1-GPU run."""
    import signal
    import socket
    import subprocess

    n = args.gpus
    # KETO_BENCH_BACKEND=gloo: a rehearsal whose ranks share the visible GPUs (its line says so)
    shared = os.environ.get("KETO_BENCH_BACKEND", "nccl") == "gloo"
    have = n if (args.dry_run or shared) else visible_gpus()
    if have < n:
        log(f"bench.py --gpus {n}: only {have} GPU(s) visible -- refusing to report a {n}-GPU line")
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0):  # one rank failed: the others would wait forever
                    for q in procs:
                        if q.poll() is None:
                            q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    worst = max((abs(rc) for rc in rcs), default=0)
    if worst:
        log(f"bench.py --gpus {n}: rank exit codes {rcs}")
    return worst


def per_rank_ms(ms_local: float, device: str):
    """every rank's ms/step (all ranks' values, rank order); without a process group: [this rank's]"""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [ms_local]
    t = torch.zeros(dist.get_world_size(), dtype=torch.float64, device=device)
    t[dist.get_rank()] = ms_local
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()]


def dry_run_rank(args, rank, world):
    """--dry-run (CPU, tests): the launcher and the rank protocol without a GPU -- every rank
    joins a gloo group, checks its own seeded shard of a small nested-group batch with the
    oracle `steps` times, and rank 0 prints the line the GPU job prints (n_gpus, per-rank ms)"""
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refsem
    from keto_mi355x import synth
    from product_helpers import queries_to_oracle, world_from_workload

    if world > 1:
        dist.init_process_group("gloo")
    wl = synth.nested_groups(20_000, seed=1)
    q = synth.nested_groups_queries(wl, 256, seed=shard_seed(7, rank))
    w, t = world_from_workload(wl)
    orc = refsem.Oracle(w, t)
    orc.set_limits(wl.max_depth, wl.max_width)
    qo = queries_to_oracle(q)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dec, _, _ = orc.check_batch(qo, threads=1)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    value, elapsed, total = job_rate(el, len(q) * args.steps, "cpu")
    ranks_ms = per_rank_ms(el / args.steps * 1e3, "cpu")
    out = {"metric": METRIC, "value": value, "unit": "checks/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "per_rank_ms_per_step": ranks_ms,
           "dry_run": True, "checks": total, "allowed_checksum": int(dec.sum())}
    if rank == 0:
        print(json.dumps(out), flush=True)
    orc.close()
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c4")
    ap.add_argument("--scale", type=int, default=40, help="C5 graph = C3 x scale (40: ~4.2B tuples)")
    ap.add_argument("--placement", choices=["hash", "tree", "tree_repl"], default="hash",
                    help="C5 owner rule: keto_object_owner's hash, every root folder tree on one rank (keto_placement), "
                         "or that with the groups replicated on every rank")
    ap.add_argument("--tuples", type=int, default=10_000_000, help="C2 graph size")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--engine-streams", type=int, default=int(os.environ.get("KETO_BENCH_STREAMS", "1")),
                    help="value pipeline: batches alternate over this many engine streams")
    ap.add_argument("--latency-batch", type=int, default=1 << 16)
    ap.add_argument("--query-record", type=int, choices=[16, 32], default=16,
                    help="value pipeline: request record bytes over PCIe (16: keto_check_batch16)")
    ap.add_argument("--latency-iters", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--serve-clients", type=int, default=128, help="0 skips the dispatcher probe")
    ap.add_argument("--serve-request", type=int, default=64)
    ap.add_argument("--serve-seconds", type=float, default=3.0)
    ap.add_argument("--no-store-probe", action="store_true", help="skip the incremental-snapshot probe")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)  # CPU: launcher + rank protocol only
    argv = sys.argv[1:] if argv is None else list(argv)
    args = ap.parse_args(argv)
    if os.environ.get("KETO_BENCH_MAPS"):  # diagnostics: the process's mappings at exit (map a crash's PCs)
        import atexit

        def dump_maps(path=os.environ["KETO_BENCH_MAPS"]):
            with open("/proc/self/maps") as f, open(path, "w") as o:
                o.write(f.read())
        atexit.register(dump_maps)

    # --gpus N decides the job size: without torchrun's environment this process launches the N
    # ranks itself (before anything initialises HIP); under torchrun the world must be N
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: refusing a line whose n_gpus would be wrong")
        return 2
    if args.dry_run:
        return dry_run_rank(args, rank, world)
    import torch
    import torch.distributed as dist

    dist_on = world > 1
    # one process per GPU; KETO_BENCH_BACKEND=gloo rehearses the multi-rank path with several
    # ranks sharing one GPU (RCCL needs distinct devices)
    shared = os.environ.get("KETO_BENCH_BACKEND", "nccl") == "gloo"
    ndev = visible_gpus()
    if ndev < 1 or (not shared and local >= ndev):
        log(f"rank {rank}: LOCAL_RANK {local} needs GPU {local}, {ndev} visible")
        return 2
    device = local % ndev
    if dist_on:
        import datetime

        torch.cuda.set_device(device)
        dist.init_process_group(backend=os.environ.get("KETO_BENCH_BACKEND", "nccl"),
                                timeout=datetime.timedelta(minutes=30))
    if args.workload == "c5":
        return run_c5(args, rank, world, device, dist_on)
    import keto_mi355x as km
    from keto_mi355x import synth

    t_setup = time.perf_counter()
    wl, snap, setup_s = build_workload(args.workload, rank, world, device, args)
    info = snap.info()
    log(f"[rank {rank}] snapshot: {info['n_tuples']} tuples, {info['n_nodes']} nodes, "
        f"{info['device_bytes'] / 2**30:.1f} GiB on device, device build {info['build_seconds']:.2f}s "
        f"(setup incl. generation {setup_s:.1f}s)")
    stream = km.Stream(device)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    # this rank's shard of the query stream: its own seeded 2^20 batch
    if args.workload == "c2":
        q = synth.nested_groups_queries(wl, args.batch, seed=shard_seed(7, rank))
    else:
        q = synth.drive_queries(wl, args.batch, seed=shard_seed(11, rank))
    dq = km.DeviceBuffer(device, q.nbytes)
    da = km.DeviceBuffer(device, len(q))
    de = km.DeviceBuffer(device, 4 * len(q))
    dq.upload(stream, q)

    # algorithmic bytes per launch: one counted batch outside the timed region
    stream.counters(reset=True)
    log(f"[rank {rank}] counted batch ({time.perf_counter() - t_setup:.1f}s since start)")
    eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
    c = stream.counters(reset=True)
    pt = c["per_tier"]
    bytes_t0 = 8 * pt["rows"][0] + 4 * pt["edges"][0] + 8 * pt["probes"][0] + 17 * pt["queries"][0]
    dfs_allowed = da.download(stream, np.zeros(len(q), np.uint8))  # (the counted batch runs the DFS interpreter)
    errs = de.download(stream, np.zeros(len(q), np.int32))
    assert (errs == 0).all(), "unexpected query errors"

    dev = f"cuda:{device}" if dist_on else "cpu"
    # (1) device-resident: queries already in HBM, one synchronous batch per step -- the kernels'
    # own time (HIP events on the engine's stream around every batch's check path) for the roofline
    for _ in range(args.warmup):
        eng.check_batch_device(dq, len(q), da, de, sync=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    stream.sync()
    stream.kernel_time(reset=True)
    stream.frontier_stats(reset=True)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.check_batch_device(dq, len(q), da, de, sync=True)
    stream.sync()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    resident_local = time.perf_counter() - t_start
    resident_rate, resident_el, _ = job_rate(resident_local, args.batch * args.steps, dev)
    # average device time of a batch's check path over the timed region: HIP event pairs recorded
    # on the engine's own stream around every batch (rewrite snapshots: the frontier engine's
    # generations plus the DFS interpreter on the routed queries; C2: the union kernel's tier 0)
    k_sum, k_n = stream.kernel_time(reset=True)
    assert k_n == args.steps, f"timed {k_n} kernel launches, expected {args.steps}"
    kernel_ms = k_sum / k_n
    fr = stream.frontier_stats(reset=True)
    # the timed batches' decisions: they must equal the counted batch's DFS decisions on the same
    # queries
    allowed = da.download(stream, np.zeros(len(q), np.uint8))
    errs = de.download(stream, np.zeros(len(q), np.int32))
    assert (errs == 0).all(), "unexpected query errors"
    dfs_mismatches = int((allowed != dfs_allowed).sum())
    log(f"[rank {rank}] device-resident: {resident_local / args.steps * 1e3:.2f} ms/step, kernel {kernel_ms:.2f} ms "
        f"({time.perf_counter() - t_setup:.1f}s since start)")

    # (2) `value` -- the metric's pipeline (BASELINE.md:46-51): per step a fresh seeded batch in
    # (pinned) host memory, H2D of the queries + the check kernels + D2H of the decisions, all
    # enqueued with KETO_F_ASYNC on one engine stream: the library puts the copies on its two copy
    # streams through two staging slots, so batch k+1's H2D and batch k-1's D2H overlap batch k's
    # kernels and the kernels of two batches never share the GPU.  Timed from the first enqueue to
    # the stream drained.
    nb = min(args.steps, 32)  # distinct batches (cycled beyond 32 steps)
    if args.workload == "c2":
        qgen = lambda k: synth.nested_groups_queries(wl, args.batch, seed=shard_seed(7, rank) + 1000 * (k + 1))  # noqa: E731
    else:
        qgen = lambda k: synth.drive_queries(wl, args.batch, seed=shard_seed(11, rank) + 1000 * (k + 1))  # noqa: E731
    # the requests cross PCIe as 16-byte records (keto_check_batch16, ABI 7) when every one fits
    # that form, else as 32-byte keto_query records; qh keeps the 32-byte form for the parity reruns
    qh = [qgen(k) for k in range(nb)]
    rec16 = args.query_record == 16
    if rec16:
        try:
            km.pack_queries16(qh[0][:1])
        except km.KetoError:
            rec16 = False
    qb = [km.PinnedArray(args.batch, km.QUERY16_DT if rec16 else km.QUERY_DT) for _ in range(nb)]
    ab = [km.PinnedArray(args.batch, np.uint8) for _ in range(nb)]
    eb = [km.PinnedArray(args.batch, np.int32) for _ in range(nb)]
    for k in range(nb):
        if rec16:
            km.pack_queries16(qh[k], out=qb[k].array)
        else:
            qb[k].array[:] = qh[k]
    # engine streams: consecutive batches alternate between them, so one batch's sparse late
    # generations (a few blocks each) share the GPU with the next batch's dense early ones
    n_es = max(1, args.engine_streams)
    engs, strs = [eng], [stream]
    for _ in range(n_es - 1):
        s2 = km.Stream(device)
        e2 = km.CheckEngine(snap, s2, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
        e2.check_batch_device(dq, len(q), da, de, sync=True)  # (its speculation depth: one synchronous batch)
        engs.append(e2)
        strs.append(s2)
    for k in range(max(1, args.warmup)):
        engs[k % n_es].check_batch_async(qb[k % nb].array, ab[k % nb].array, eb[k % nb].array)
    for s_ in strs:
        s_.sync()
    stream.kernel_time(reset=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        engs[k % n_es].check_batch_async(qb[k % nb].array, ab[k % nb].array, eb[k % nb].array)
    for s_ in strs:
        s_.sync()
    if dist_on:
        dist.barrier()
    elapsed_local = time.perf_counter() - t_start
    value, elapsed, total = job_rate(elapsed_local, args.batch * args.steps, dev)
    ranks_ms = per_rank_ms(elapsed_local / args.steps * 1e3, dev)
    pipe_kernel = [stream.kernel_time(reset=True)]
    pipe_allowed = [ab[k].array.copy() for k in range(nb)]
    pipe_err = np.concatenate([eb[k].array for k in range(nb)])
    assert (pipe_err == 0).all(), "unexpected query errors"
    # the pipeline's first batch again, synchronously on the device-resident path: same decisions
    dq.upload(stream, qh[0])
    eng.check_batch_device(dq, len(q), da, de, sync=True)
    pipe_vs_resident = int((da.download(stream, np.zeros(len(q), np.uint8)) != pipe_allowed[0]).sum())
    # every distinct timed batch against the DFS interpreter (a counted rerun of the same queries:
    # the reference recursion in its canonical order, pinned to the oracle by the GPU suite)
    pipe_vs_dfs = 0
    for k in range(nb):
        dq.upload(stream, qh[k])
        eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
        pipe_vs_dfs += int((da.download(stream, np.zeros(len(q), np.uint8)) != pipe_allowed[k]).sum())
    stream.counters(reset=True)
    log(f"[rank {rank}] pipelined: {elapsed_local / args.steps * 1e3:.2f} ms/step "
        f"({time.perf_counter() - t_setup:.1f}s since start)")
    # p99 batch latency over >= 100 batches of 64Ki queries (one rank's stream)
    lat = []
    nl = min(args.latency_batch, len(q))
    dql = km.DeviceBuffer(device, q[:nl].nbytes)
    for i in range(args.latency_iters):
        off = (i * nl) % max(1, len(q) - nl + 1)
        dql.upload(stream, q[off:off + nl])
        stream.sync()
        t1 = time.perf_counter()
        eng.check_batch_device(dql, nl, da, de, sync=True)
        lat.append(time.perf_counter() - t1)
    p99_ms = float(np.percentile(np.array(lat) * 1e3, 99)) if lat else None

    log(f"[rank {rank}] latency probe done ({time.perf_counter() - t_setup:.1f}s since start)")
    expand = expand_probe(km, snap, wl, stream) if args.workload in ("c3", "c4") else None
    serving = serving_probe(km, snap, q, wl, args.serve_clients, args.serve_request, args.serve_seconds) \
        if args.serve_clients > 0 else None
    log(f"[rank {rank}] expand + serving probes done ({time.perf_counter() - t_setup:.1f}s since start)")
    store = None
    if rank == 0 and world == 1 and not args.no_store_probe and args.workload in ("c3", "c4"):
        # the probe is a deployment's write path: the store, its served snapshot and the next one.
        # The bench's own snapshot, streams and buffers are not part of it and are released first
        # (in a deployment the served snapshot is the store's own)
        if os.environ.get("KETO_BENCH_STORE_KEEP") is None:
            for b_ in (dq, da, de, dql):
                b_.free()
            for s_ in strs:
                s_.close()
            snap.close()
            torch.cuda.empty_cache()
        store = store_probe(km, wl, q)
        log(f"[rank {rank}] store probe: advance {store['advance_ms']:.1f} ms (advanced {store['advanced']}), copy patch "
            f"{store['patch_ms']:.1f} ms (patched {store['patched']}), full build "
            f"{store['full_build_ms']:.0f} ms ({time.perf_counter() - t_setup:.1f}s since start)")

    achieved = bytes_t0 / (kernel_ms * 1e-3) / 1e9
    kname = "frontier"
    traffic, traffic_src = committed_traffic(args.workload, kname)
    if args.workload == "c2":
        data, cfgno = "nested-group graph", 2
        desc = (f"C2 nested groups: {info['n_tuples']} tuples, 5 levels, union-only, max_read_depth 8, "
                f"{args.batch} checks/batch/GPU, 50% random-walk positives, 1% depth 1-4")
    else:
        data, cfgno = "Drive-style folder forest", 4 if args.workload == "c4" else 3
        desc = (f"{args.workload.upper()} Drive-style: {info['n_tuples']} tuples, {wl.meta['roots']} forest(s) of fanout 5, "
                f"depth 10, view = (viewers | editors | owners | parents.traverse(view)) & !banned, "
                f"max_read_depth 16, {args.batch} checks/batch/GPU")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "checks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "per_rank_ms_per_step": ranks_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": f"synthetic (seeded {data}, BASELINE config {cfgno}; generated on the host, no dataset)",
        "config": {"workload": desc, "tuples": int(info["n_tuples"]), "batch_per_gpu": args.batch,
                   "parallelism": f"replica x{world} (query batch sharded, no data-path collective)"},
        "p99_batch_latency_ms": p99_ms,
        "latency_batch": nl,
        "allowed_fraction": float(allowed.mean()),
        "timed_vs_dfs": {"n": int(len(q)), "mismatches": dfs_mismatches,
                         "note": "device-resident batches' decisions vs the counted batch's DFS interpreter, same queries"},
        "pipeline": {"what": "value: per step a fresh seeded batch in pinned host memory, H2D + check kernels + D2H "
                             "enqueued (KETO_F_ASYNC) on one engine stream -- the library runs the copies on two copy "
                             "streams through two staging slots, overlapping the neighbouring batches' kernels; timed "
                             "from the first enqueue until the stream drained",
                     "distinct_batches": nb, "streams": f"{n_es} engine stream(s), each 1 compute + 2 copy",
                     "query_record_bytes": 16 if rec16 else 32,
                     "kernel_ms_per_batch": [ks / max(1, kn) for ks, kn in pipe_kernel],
                     "first_batch_vs_device_resident_mismatches": pipe_vs_resident,
                     "mismatches": pipe_vs_dfs,
                     "mismatches_what": f"all {nb} distinct timed batches ({nb * args.batch} queries) vs the DFS "
                                        "interpreter on a counted rerun of the same queries",
                     "allowed_fraction": float(np.mean([a.mean() for a in pipe_allowed]))},
        "device_resident": {"checks_per_s": resident_rate, "ms_per_step": resident_el / args.steps * 1e3,
                            "kernel_ms": kernel_ms,
                            "what": "the same step with the queries already in HBM and outputs left there, one "
                                    "synchronous batch per step (KETO_F_DEVICE_PTRS): the roofline's timing"},
        "serving": serving,
        "expand": expand,
        "incremental_snapshot": store,
        "snapshot_build_s": info["build_seconds"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": ("check path: resolve_kernel + fr_block (one launch) + DFS on routed"
                                if os.environ.get("KETO_FR_ENGINE", "b" if args.batch <= int(os.environ.get(
                                    "KETO_FR_BLOCK_MAX", 1 << 16)) else "g")[0] == "b" else
                                "check path: resolve_kernel + frontier generations (fr_init, fr_expand, fr_reduce, "
                                "fr_repeat) + DFS on routed"),
                     "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": int(bytes_t0),
                     "bytes_model": "8*rows + 4*edges + 8*probes + 17*queries (BASELINE.md) of the REFERENCE's "
                                    "traversal -- the rows, edges and probes Keto's engine reads for these queries "
                                    "(the DFS interpreter's counters of a counted batch, equal to the oracle's) -- "
                                    "over the engine's measured check-path time; the engine itself reads a "
                                    "different (unpruned, breadth-first) set",
                     "work": {"rows": pt["rows"][0], "edges": pt["edges"][0], "probes": pt["probes"][0],
                              "queries_tier0": pt["queries"][0], "queries_tier1": pt["queries"][1],
                              "queries_tier2": pt["queries"][2]}},
        "cpu_baseline": None,
    }
    if fr["batches"]:
        out["frontier"] = {"goals_per_batch": fr["goals"] / fr["batches"], "generations_max": fr["max_generations"],
                           "routed_fraction": fr["routed"] / max(1, fr["queries"]), "budget": 1024}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sched, cb, dec = cpu_baseline(wl, q, wl.max_depth, wl.max_width, args.cpu_budget, gpu_allowed=allowed,
                                      pipe=[(qh[k], pipe_allowed[k]) for k in range(nb)])
        out["cpu_baseline"] = cb
        if cpu_baseline.pipe is not None:
            out["pipeline"]["oracle_mismatches"] = cpu_baseline.pipe["mismatches"]
            out["pipeline"]["oracle_sample"] = cpu_baseline.pipe
        out["cpu_baseline_sql_mode"] = getattr(cpu_baseline, "sql", None)
        ns = len(dec)
        out["cpu_parity_sample"] = {"n": ns, "mismatches": int((dec != allowed[:ns]).sum())}
        out["schedule_sensitivity"] = sched
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
