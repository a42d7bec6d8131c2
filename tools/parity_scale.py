"""Parity at full scale (tool): GPU decisions vs the oracle over the same Drive/C2 graph and
query batch; prints mismatches (query, both answers, oracle work).  Test/debug only."""
import argparse
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "djy-keto_amd"))
sys.path.insert(0, os.path.join(R, "oracle"))
import numpy as np  # noqa: E402

import keto_mi355x as km  # noqa: E402
import refsem  # noqa: E402
from keto_mi355x import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=1)
ap.add_argument("--n", type=int, default=1 << 16)
ap.add_argument("--out", default="gpurun_out/parity_mismatch.npz")
ap.add_argument("--check", type=int, default=0, help="oracle on this many queries from the batch tail too")
a = ap.parse_args()
wl = synth.drive_scaled(a.scale)
q = synth.drive_queries(wl, a.n, seed=11)
snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict, device=0)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
allowed, err = eng.check_batch(q)
dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
dq.upload(st, q)
for cnt in (True, False):
    eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=cnt)
    a2 = da.download(st, np.zeros(len(q), np.uint8))
    print(f"device path count={cnt}: allowed {a2.mean():.4f}, differs from host path on {(a2 != allowed).sum()}"
          f" (tail half {a2[len(q)//2:].mean():.4f} vs {allowed[len(q)//2:].mean():.4f})", flush=True)
if a.check:
    sel = np.r_[0:a.check, len(q) - a.check:len(q)]
    q, allowed, err = q[sel], allowed[sel], err[sel]
w = refsem.World(namespaces=wl.namespaces, strict=wl.strict, max_depth=wl.max_depth, max_width=wl.max_width)
w.ns_names, w.rel_names, w.uuids = refsem.Interner(), refsem.Interner(), refsem.Interner()
for n in wl.ns_names:
    w.ns_names(n)
for r in wl.rel_names:
    w.rel_names(r)
w._walk_names()
t0 = time.time()
orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
print(f"oracle build {time.time() - t0:.1f}s", flush=True)
dec, oerr, _ = orc.check_batch(q.view(refsem.QUERY_DT), threads=16)
mm = np.nonzero((dec != allowed) | (oerr != err))[0]
print(f"scale {a.scale}: {len(mm)} mismatches of {len(q)} (gpu allowed {allowed.mean():.4f}, oracle {dec.mean():.4f})")
for i in mm[:20]:
    one = q[i:i + 1]
    m1, e1, s1 = orc.check(one.view(refsem.QUERY_DT))
    print(i, one[0], "gpu", allowed[i], err[i], "oracle", dec[i], oerr[i], "mem", m1[0], "rows/edges/probes",
          s1.rows, s1.edges, s1.probes)
os.makedirs(os.path.dirname(a.out), exist_ok=True)
np.savez(a.out, idx=mm, q=q[mm], gpu=allowed[mm], orc=dec[mm])
