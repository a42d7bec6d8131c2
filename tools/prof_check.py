"""Profiling driver: C2 snapshot + a few 2^20-query check batches (no counting pass),
short enough for one rocprofv3 --pmc pass.  KETO_MI355X_LIB_OVERRIDE selects an A/B build."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, default=3)
ap.add_argument("--tuples", type=int, default=10_000_000)
ap.add_argument("--workload", default="c2")
ap.add_argument("--count", action="store_true", help="one counted batch first: per-tier work and step counters")
ap.add_argument("--single", type=int, default=-1, help="time one query alone, x64 and x(full grid) copies")
ap.add_argument("--compare", action="store_true", help="frontier vs DFS interpreter: decisions and times")
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
dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
dq.upload(st, q)
if a.single >= 0:
    for copies in (1, 64, 6144 * 64):
        qq = np.repeat(q[a.single:a.single + 1], copies)
        d2 = km.DeviceBuffer(0, qq.nbytes)
        d2.upload(st, qq)
        st.counters(reset=True)
        eng.check_batch_device(d2, copies, da, de, sync=True, count_work=True)
        c = st.counters(reset=True)
        ms = []
        for _ in range(3):
            eng.check_batch_device(d2, copies, da, de, sync=True)
            ms.append(st.last_kernel_ms())
        print(f"query {a.single} x{copies}: tier-0 kernel {min(ms):.3f} ms, lane_steps/query "
              f"{c['lane_steps'] / copies:.0f}, wave_steps {c['wave_steps']}, "
              f"us/step {min(ms) * 1e3 * ((copies + 63) // 64) / max(1, c['wave_steps']):.2f}",
              flush=True)
if a.count:
    st.counters(reset=True)
    eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
    c = st.counters(reset=True)["per_tier"]
    for t in range(3):
        ws, ls = c["wave_steps"][t], c["lane_steps"][t]
        print(f"tier {t}: queries {c['queries'][t]} rows {c['rows'][t]} edges {c['edges'][t]} probes {c['probes'][t]} "
              f"wave_steps {ws} lane_steps {ls} util {ls / max(1, 64 * ws):.3f}", flush=True)
for i in range(a.batches):
    t0 = time.perf_counter()
    eng.check_batch_device(dq, len(q), da, de, sync=True)
    print(f"batch {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms, tier-0 kernel {st.last_kernel_ms():.2f} ms",
          flush=True)
if a.compare:
    res = {}
    for mode in ("0", "1"):
        os.environ["KETO_FRONTIER"] = mode
        ms = []
        for i in range(3):
            t0 = time.perf_counter()
            eng.check_batch_device(dq, len(q), da, de, sync=True)
            ms.append((time.perf_counter() - t0) * 1e3)
        res[mode] = (da.download(st, np.zeros(len(q), np.uint8)), de.download(st, np.zeros(len(q), np.int32)), min(ms),
                     st.last_kernel_ms())
        print(f"KETO_FRONTIER={mode}: batch {min(ms):.2f} ms, device path {res[mode][3]:.2f} ms", flush=True)
    fs = st.frontier_stats(reset=True)
    print("frontier stats", fs, flush=True)
    same = (res["0"][0] == res["1"][0]).all() and (res["0"][1] == res["1"][1]).all()
    print("decisions identical:", bool(same), "allowed", int(res["1"][0].sum()), flush=True)
    if not same:
        sys.exit(1)
