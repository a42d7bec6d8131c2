"""Random-world parity sweep (tool, test infrastructure): the suite's random worlds
(tests/randworld.py) over many more seeds and two sizes, on the GPU, against the oracle.

Per world: Check decisions and errors equal the canonical DFS (rs_check); the frontier's routed
count equals rs_check_u's and, with nothing routed, so does its goal count (the spawn rules,
goal for goal); Expand trees equal the oracle's, child order included.  Prints a progress line
per 50 worlds and a final JSON summary; failing (seed, size, rewrites) triples are listed.
usage: parity_sweep.py --seeds 60:1060 [--sizes small,big] [--kind random|spine]
(KETO_FR_ENGINE=gen forces the generation engine)"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("djy-keto_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(R, p))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
import refsem  # noqa: E402
from product_helpers import product_snapshot, product_tree_to_nested, queries_to_product  # noqa: E402
from randworld import random_world  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", default="60:560")
ap.add_argument("--sizes", default="small,big")
ap.add_argument("--budget", type=int, default=1024)
ap.add_argument("--kind", default="random", choices=["random", "spine"],
                help="spine: tests/test_gpu_spine.py's folder-chain worlds (sizes = width limits 10 / 2 / 1)")
a = ap.parse_args()
lo, hi = (int(x) for x in a.seeds.split(":"))
SIZES = {"small": {}, "big": {"n_obj": 24, "n_users": 10, "n_tuples": 260}}
if a.kind == "spine":
    from test_gpu_spine import spine_world  # noqa: E402
    a.sizes = "10,2,1" if a.sizes == "small,big" else a.sizes


def world(seed, size, rewrites):
    if a.kind == "spine":
        w, t, q = spine_world(seed, int(size))
        return w, t, q, []
    return random_world(seed, rewrites=rewrites, **SIZES[size])

os.environ["KETO_FR_BUDGET"] = str(a.budget)
stream = km.Stream(0)
tot = {"worlds": 0, "queries": 0, "routed": 0, "goals": 0, "expand_roots": 0, "goal_checked_worlds": 0}
fails = []
t0 = time.time()
for seed in range(lo, hi):
    for size in a.sizes.split(","):
        for rewrites in ((True,) if a.kind == "spine" else (True, False)):
            w, t, q, expands = world(seed, size, rewrites)
            orc = refsem.Oracle(w, t)
            orc.set_limits(w.max_depth, w.max_width)
            dec, err, _ = orc.check_batch(q, threads=8)
            _, _, routed, goals, _ = orc.check_u_batch(q, threads=8, budget=a.budget)
            snap = product_snapshot(w, t)
            what = []
            try:
                eng = km.CheckEngine(snap, stream, max_read_depth=w.max_depth, max_read_width=w.max_width)
                stream.frontier_stats(reset=True)
                allowed, gerr = eng.check_batch(queries_to_product(q))
                fs = stream.frontier_stats(reset=True)
                if not np.array_equal(gerr, err):
                    what.append("errors")
                if not np.array_equal(allowed, dec):
                    what.append("decisions")
                if fs["batches"] and fs["routed"] != int(routed.sum()):
                    what.append("routed %d vs %d" % (fs["routed"], int(routed.sum())))
                if fs["batches"] and not routed.any():
                    tot["goal_checked_worlds"] += 1
                    if fs["goals"] != int(goals.sum()):
                        what.append("goals %d vs %d" % (fs["goals"], int(goals.sum())))
                xe = km.ExpandEngine(snap, stream, max_read_depth=w.max_depth)
                if expands:
                    roots = np.array([(w.ns_names.ids[x], w.uuids.ids[b], w.rel_names.ids[r], d)
                                      for x, b, r, d in expands], dtype=km.SUBJSET_DT)
                    nodes, offs, xerr = xe.build_trees(roots)
                    if (xerr != 0).any():
                        what.append("expand errors")
                for i, (x, b, r, d) in enumerate(expands):
                    on, _ = orc.expand(1, w.uuids.ids[b], w.ns_names.ids[x], w.rel_names.ids[r], d)
                    if product_tree_to_nested(w, nodes[int(offs[i]):int(offs[i + 1])]) != refsem.tree_to_nested(w, on):
                        what.append("tree %d" % i)
                        break
                tot["queries"] += len(q)
                tot["routed"] += int(fs["routed"])
                tot["goals"] += int(fs["goals"])
                tot["expand_roots"] += len(expands)
            finally:
                snap.close()
            tot["worlds"] += 1
            if what:
                fails.append({"seed": seed, "size": size, "rewrites": rewrites, "what": what})
                print("FAIL", fails[-1], flush=True)
            if tot["worlds"] % 50 == 0:
                print("worlds %d  queries %d  fails %d  %.0f s" % (tot["worlds"], tot["queries"], len(fails), time.time() - t0),
                      flush=True)
stream.close()
print(json.dumps({"kind": a.kind, "seeds": a.seeds, "sizes": a.sizes, "budget": a.budget,
                  "engine": os.environ.get("KETO_FR_ENGINE", "auto"), **tot, "fails": fails,
                  "seconds": round(time.time() - t0, 1)}))
sys.exit(1 if fails else 0)
