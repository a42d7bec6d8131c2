"""Per-query interpreter step counts (tool, not product): run a sample of a synthetic batch
one query at a time through the CPU emulation build (tools/cpuemu) with work counting,
so lane_steps of each call = load-slot iterations of that query in tier 0.  Then simulate
the persistent grid's schedule (waves x 64 lanes, longest-first work order) to see how much
of a batch is bound by its longest queries.

  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=tools/cpuemu/libketo_emu.so \
      python tools/query_steps.py --workload c2 --sample 20000
"""
import argparse
import heapq
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--sample", type=int, default=20000)
ap.add_argument("--tuples", type=int, default=10_000_000)
ap.add_argument("--out", default="gpurun_out/query_steps.npz")
a = ap.parse_args()
if a.workload == "c2":
    wl = synth.nested_groups(a.tuples, seed=1)
    q = synth.nested_groups_queries(wl, 1 << 20, seed=7)
else:
    wl = synth.drive(depth=8, n_groups=200_000, n_users=2_000_000, seed=3)
    q = synth.drive_queries(wl, 1 << 20, seed=11)
snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
rng = np.random.Generator(np.random.PCG64(0))
idx = np.sort(rng.choice(len(q), size=min(a.sample, len(q)), replace=False))
steps = np.zeros(len(idx), np.int64)
rows = np.zeros(len(idx), np.int64)
st.counters(reset=True)
for k, i in enumerate(idx):
    eng.check_batch(q[i:i + 1], count_work=True)
    c = st.counters(reset=True)
    steps[k] = c["lane_steps"]
    rows[k] = c["rows"]
os.makedirs(os.path.dirname(a.out), exist_ok=True)
np.savez(a.out, idx=idx, steps=steps, rows=rows)
pct = [50, 90, 99, 99.9, 100]
print("steps/query mean %.1f" % steps.mean(), {p: int(np.percentile(steps, p)) for p in pct})
print("rows/query  mean %.1f" % rows.mean(), {p: int(np.percentile(rows, p)) for p in pct})


def simulate(steps_all, lanes, order_desc=True):
    """persistent lanes pull queries in order; returns (makespan in steps, mean busy fraction)"""
    work = np.sort(steps_all)[::-1] if order_desc else steps_all
    heap = [0] * lanes
    for w in work:
        t = heapq.heappop(heap)
        heapq.heappush(heap, t + int(w))
    mk = max(heap)
    return mk, work.sum() / (mk * lanes)


full = np.resize(steps, len(q))  # the sample's distribution at batch size
for lanes in (6144 * 64,):
    for desc in (True, False):
        mk, util = simulate(full, lanes, desc)
        print(f"lanes {lanes} longest-first={desc}: makespan {mk} steps, lane utilisation {util:.3f}, "
              f"ideal {full.sum() / lanes:.0f} steps")
