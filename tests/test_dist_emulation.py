"""The distributed frontier (djy-keto_amd/csrc/frontier_dist.hip: a graph partitioned by object,
each rank's partition resident, the goals that cross to another rank's objects exchanged once per
generation and their values returned bottom-up) on the CPU, no GPU: the kernel SOURCES built for
the host by tools/cpuemu (one lane at a time), on 2 and 3 gloo ranks, each holding only the tuples
keto_object_owner gives it.

Every query the engine decides itself must equal the oracle over the whole graph
(oracle/refsem.c; internal/check/engine.go:65-266): random worlds with every rewrite kind,
undeclared relations, cycles, depth and width truncation and strict mode (tests/randworld.py),
and a small Drive forest.  The queries it routes to the closure path (visited-set repeats across
ranks, the goal budget) come back flagged here (err -1: the closure path is GPU-only, its answers
are tests/test_gpu_partition.py's); they must stay a small share."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tools", "cpuemu")


@pytest.fixture(scope="module")
def emu_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("emu")
    lib = d / "libketo_emu_dist.so"
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", EMU, f"OBJDIR={d / 'obj'}", f"LIB={lib}", "OPT=-O1"], check=True,
                   timeout=900)
    return str(lib)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lib, case, seeds, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KETO_MI355X_ALLOW_OVERRIDE="tools",
                      KETO_MI355X_LIB_OVERRIDE=lib)
    if case == "drive_chunked":  # the batch in chunks of 700 queries (the ranks' chunk counts differ)
        os.environ["KETO_PART_CHUNK"] = "700"
    for p in (ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json

        import refsem
        from keto_mi355x import partition, synth
        import keto_mi355x as km
        from product_helpers import queries_to_oracle, queries_to_product, tuples_to_product, world_from_workload
        from randworld import random_world
        from torch_collective import TorchCollective

        coll = TorchCollective()
        res = []
        for seed in seeds:
            if case == "random":
                w, t, q_rs, expands = random_world(seed)
                roots = np.array([(w.ns_names.ids[a], w.uuids.ids[b], w.rel_names.ids[r], d) for a, b, r, d in expands],
                                 dtype=km.SUBJSET_DT)
                tup = tuples_to_product(t)
                q = queries_to_product(q_rs)
                ns_cfg, ns_names, rel_names = json.dumps(w.namespaces), w.ns_names.names, w.rel_names.names
                n_uuids, strict, depth, width = max(1, len(w.uuids.names)), w.strict, w.max_depth, w.max_width
                orc = refsem.Oracle(w, t)
                orc.set_limits(depth, width)
                oq = q_rs
            else:
                wl = synth.drive(depth=4, fanout=3, acl_per_node=6, n_groups=200, members_per_group=6, n_users=600,
                                 seed=seed, roots=6 if case.startswith("drive_placed") else 1)
                tup = wl.tuples
                q = synth.drive_queries(wl, 3000 - 500 * rank * (case == "drive_chunked"), seed=seed + 7)
                ns_cfg, ns_names, rel_names = wl.namespaces, wl.ns_names, wl.rel_names
                n_uuids, strict, depth, width = wl.n_uuids, wl.strict, wl.max_depth, wl.max_width
                w, _ = world_from_workload(wl, with_tuples=False)
                orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
                orc.set_limits(depth, width)
                oq = queries_to_oracle(q)
                rng = np.random.default_rng(seed + rank)
                roots = np.zeros(24, dtype=km.SUBJSET_DT)
                roots["ns"][:12], roots["rel"][:12] = wl.ns_names.index("Group"), wl.rel_names.index("members")
                roots["obj"][:12] = wl.meta["gbase"] + rng.integers(0, wl.meta["n_groups"], 12)
                roots["ns"][12:], roots["rel"][12:] = wl.ns_names.index("Folder"), wl.rel_names.index("viewers")
                roots["obj"][12:] = rng.integers(0, wl.meta["folders_per_root"], 12)
            # drive_placed: every root's folder tree on one rank (keto_placement), groups hashed;
            # drive_placed_repl: the same with the groups replicated on every rank (KETO_PLACE_ALL)
            place = synth.drive_placement(wl, replicate_groups=case == "drive_placed_repl") \
                if case.startswith("drive_placed") else None
            o = partition.object_owner(tup["ns"], tup["obj"], world, place)
            own = (o == rank) | (o == partition.OWNER_ALL)
            # (world 1: KETO_F_PART_DIST, the distributed frontier with every exchange to this rank)
            eng = partition.PartitionedEngine(ns_cfg, ns_names, rel_names, n_uuids, tup[own], strict=strict,
                                              max_read_depth=depth, max_read_width=width, collective=coll,
                                              distributed=world == 1, placement=place)
            allowed, err = eng.check_batch(q)  # every rank checks the whole batch: each root at its owner
            st = dict(eng.last)
            lv = eng.generation_stats()
            dec, oerr, _ = orc.check_batch(oq, threads=1)
            ok = err != -1
            # Expand: rows fetched from their owners, walked here (csrc/expand_dist.hip): exact trees
            nodes, offs, xerr = eng.expand_batch(roots)
            xst = dict(eng.last)
            tree_mis = 0
            for i, r in enumerate(roots):
                on, _ = orc.expand(1, int(r["obj"]), int(r["ns"]), int(r["rel"]), int(r["max_depth"]))
                mine = nodes[int(offs[i]):int(offs[i + 1])]
                same = len(mine) == len(on)
                for a, b in (("type", "type"), ("subj_kind", "kind"), ("s_obj", "sid"), ("s_ns", "sns"), ("s_rel", "srel"),
                             ("n_children", "n_children")):
                    same = same and np.array_equal(mine[a], on[b])
                tree_mis += 0 if same else 1
            res.append(dict(seed=seed, n=len(q), routed=int((~ok).sum()), st_routed=int(st["routed"]),
                            dmis=int((allowed[ok] != dec[ok]).sum()), emis=int((err[ok] != oerr[ok]).sum()),
                            gens=int(st["generations"]), levels=len(lv), sent=int(st["exchange_bytes"]),
                            allowed=int(allowed[ok].sum()), tree_mis=int(tree_mis), xerr=int((xerr != 0).sum()),
                            tree_nodes=int(offs[-1]), x_levels=int(xst["levels"])))
            orc.close()
            eng.close()
        out[rank] = res
    finally:
        dist.destroy_process_group()


def _run(lib, world, case, seeds):
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), lib, case, seeds, out), nprocs=world, join=True)
        return dict(out)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_random_worlds_match_oracle(emu_lib, world):
    res = _run(emu_lib, world, "random", list(range(300, 330)))
    total = routed = 0
    for r in range(world):
        for x in res[r]:
            assert x["dmis"] == 0 and x["emis"] == 0, (r, x)
            assert x["tree_mis"] == 0 and x["xerr"] == 0, (r, x)
            assert x["routed"] == x["st_routed"] and x["levels"] == x["gens"], (r, x)
            total += x["n"]
            routed += x["routed"]
    assert routed < 0.25 * total, (routed, total)


@pytest.mark.parametrize("world,case", [(2, "drive"), (3, "drive"), (3, "drive_chunked"), (2, "drive_placed"),
                                        (3, "drive_placed"), (2, "drive_placed_repl"), (3, "drive_placed_repl")])
def test_small_drive_matches_oracle(emu_lib, world, case):
    res = _run(emu_lib, world, case, [5])
    for r in range(world):
        for x in res[r]:
            assert x["dmis"] == 0 and x["emis"] == 0, (r, x)
            assert x["tree_mis"] == 0 and x["xerr"] == 0 and x["tree_nodes"] > 24 and x["x_levels"] > 1, (r, x)
            assert x["routed"] < 0.02 * x["n"], (r, x)
            assert x["sent"] > 0 and x["gens"] > 3 and x["allowed"] > 0, (r, x)


def test_scratch_cache_never_waits_on_a_dead_stream(emu_lib):
    """keto_stream_destroy retires the scratch-cache events recorded on its streams (compute, H2D,
    D2H) before destroying them: a builder temporary released on each, then taken again after the
    stream object is gone, must not be fenced by its dead stream's event (the round-4 end-of-suite
    failure: hipEventSynchronize on an event of a destroyed stream).  tools/cpuemu models stream
    liveness; tools/cpuemu/emu_probe.cpp is the probe (it fails with KETO_E_DEVICE without the
    retirement)."""
    import ctypes
    lib = ctypes.CDLL(emu_lib)
    assert lib.keto_emu_scratch_dead_stream_probe() == 0
