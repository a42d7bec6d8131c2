"""Process-exit probe (tool): the library's copy patterns, then a normal exit, meant
to run under `rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/exit_probe.py MODE`.
  sync    host-pointer batches (the library's staging buffers, synchronous)
  async   KETO_F_ASYNC batches over pinned host memory on the engine stream's two copy streams
          (bench.py's pipelined path), then the usual atexit teardown (handles closed, keto_shutdown)
  leak    the same as async, and no teardown at all (KETO_MI355X_NO_TEARDOWN=1): every stream, event
          and pinned buffer of the library left to the runtime
Prints the addresses of the library's pinned buffers and the process's mappings of them, so a
fault address from the run can be matched against them (KETO_BENCH_MAPS-style: /proc/self/maps
is written to gpurun_out/exit_probe_maps_<MODE>.txt at the end of main)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "djy-keto_amd")]
MODE = sys.argv[1] if len(sys.argv) > 1 else "async"
if MODE == "leak":
    os.environ["KETO_MI355X_NO_TEARDOWN"] = "1"

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402


def main():
    wl = synth.nested_groups(200_000, seed=1)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids)
    q = synth.nested_groups_queries(wl, 1 << 16, seed=2)
    stream = km.Stream(0)
    eng = km.CheckEngine(snap, stream, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    if MODE == "sync":
        for _ in range(8):
            a, e = eng.check_batch(q)
    else:
        qb = [km.PinnedArray(len(q), km.QUERY_DT) for _ in range(4)]
        ab = [km.PinnedArray(len(q), np.uint8) for _ in range(4)]
        eb = [km.PinnedArray(len(q), np.int32) for _ in range(4)]
        for b in qb:
            b.array[:] = q
        for k in range(16):
            eng.check_batch_async(qb[k % 4].array, ab[k % 4].array, eb[k % 4].array)
        stream.sync()
        a = ab[0].array
        for name, bufs in (("queries", qb), ("allowed", ab), ("errors", eb)):
            print(name, [hex(b.array.ctypes.data) for b in bufs])
    print("allowed", int(np.asarray(a).sum()), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open("/proc/self/maps") as f, open(os.path.join(ROOT, "gpurun_out", f"exit_probe_maps_{MODE}.txt"), "w") as o:
        o.write(f.read())


if __name__ == "__main__":
    main()
    print("main returned", flush=True)
