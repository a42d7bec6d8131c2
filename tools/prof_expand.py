"""Batched Expand timing (tool, not product): the bench's expand probe on the C3 graph,
per-call wall time; run under rocprofv3 --kernel-trace --stats for the kernel share."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402
import bench  # noqa: E402

w = synth.drive_scaled(int(os.environ.get("SCALE", "1")))
snap = km.Snapshot(w.namespaces, w.tuples, w.ns_names, w.rel_names, w.n_uuids, strict=w.strict, device=0)
st = km.Stream(0)
print(bench.expand_probe(km, snap, w, st), flush=True)
rng = np.random.default_rng(5)
n = 4096
r = np.zeros(n, dtype=km.SUBJSET_DT)
h = n // 2
r["ns"][:h], r["rel"][:h] = 1, w.rel_names.index("members")
r["obj"][:h] = w.meta["gbase"] + rng.integers(0, w.meta["n_groups"], h)
r["ns"][h:], r["rel"][h:] = 2, w.rel_names.index("viewers")
r["obj"][h:] = rng.integers(0, w.meta["folders_per_root"], n - h)
xe = km.ExpandEngine(snap, st, max_read_depth=w.max_depth)
for half, sl in (("members", slice(0, h)), ("viewers", slice(h, n))):
    xe.build_trees(r[sl])
    t0 = time.perf_counter()
    nodes, offs, err = xe.build_trees(r[sl])
    print(f"{half}: {(time.perf_counter() - t0) * 1e3:.2f} ms, {int(offs[-1])} nodes, max tree "
          f"{int(np.diff(offs.astype(np.int64)).max())}", flush=True)
