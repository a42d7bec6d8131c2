"""Time generation + device snapshot build of the Drive workload at a scale (C3 = 1, C4 = 10),
then one 2^20-query Check batch (tool, not product)."""
import argparse
import os
import resource
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=1)
ap.add_argument("--batches", type=int, default=3)
a = ap.parse_args()
t0 = time.time()
w = synth.drive_scaled(a.scale)
print(f"gen {len(w.tuples)} tuples {time.time() - t0:.1f}s rss {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6:.1f} GB", flush=True)
t0 = time.time()
snap = km.Snapshot(w.namespaces, w.tuples, w.ns_names, w.rel_names, w.n_uuids, strict=w.strict, device=0)
print(f"build {time.time() - t0:.1f}s {snap.info()} rss {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6:.1f} GB", flush=True)
q = synth.drive_queries(w, 1 << 20, seed=11)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=w.max_depth, max_read_width=w.max_width)
dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
dq.upload(st, q)
for i in range(a.batches):
    t1 = time.perf_counter()
    eng.check_batch_device(dq, len(q), da, de, sync=True)
    print(f"batch {i}: {(time.perf_counter() - t1) * 1e3:.2f} ms kernel {st.last_kernel_ms():.2f} ms", flush=True)
allowed = da.download(st, np.zeros(len(q), np.uint8))
print("allowed fraction", allowed.mean())
