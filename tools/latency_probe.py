"""Batch latency vs batch size (profiling tool): device-pointer batches of n queries on the
C3 (or C4) Drive graph, wall time per batch and the main kernel's HIP-event time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "djy-keto_amd"))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 1
wl = synth.drive_scaled(scale)
snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
s = km.Stream(0)
eng = km.CheckEngine(snap, s, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
q = synth.drive_queries(wl, 1 << 16, seed=5)
dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
dq.upload(s, q)
for n in (1, 16, 128, 512, 4096, 65536):
    ws, ks = [], []
    for it in range(30):
        t0 = time.perf_counter()
        eng.check_batch_device(dq, n, da, de, sync=True)
        ws.append((time.perf_counter() - t0) * 1e3)
        ks.append(s.last_kernel_ms())
    ws, ks = np.array(ws[5:]), np.array(ks[5:])
    print(f"n={n:6d} wall p50 {np.median(ws):7.3f} ms  p99 {np.percentile(ws, 99):7.3f}  kernel p50 {np.median(ks):7.3f} ms",
          flush=True)
