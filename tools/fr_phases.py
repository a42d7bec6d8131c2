"""fr_expand phase profile of a KETO_FR_PROF build (tools/ab_build.sh): wave-cycles spent between
the kernel's phase marks over one frontier batch of the Drive profiling workload.
usage: KETO_MI355X_LIB_OVERRIDE=tools/ab/libketo_frprof.so python3 tools/fr_phases.py [--c4]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

if "--c4" in sys.argv:  # bench.py's C4 graph and batch
    wl = synth.drive_scaled(10)
else:
    wl = synth.drive(depth=8, n_groups=200_000, n_users=2_000_000, seed=3)
q = synth.drive_queries(wl, 1 << 20, seed=11)
snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
eng.check_batch(q)
st.counters(reset=True)
eng.check_batch(q)
c = st.counters(reset=True)["per_tier"]
vals = [c["rows"][0], c["edges"][0], c["probes"][0], c["out_nodes"][0], c["queries"][0], c["wave_steps"][0],
        c["lane_steps"][0]]
names = ["loads (g0, qgoals, row, subject)", "phase A (decide / count)", "budget + qgoals atomics",
         "allocation (goals, occurrences) + gfn/gval stores", "phase B (spawn children, occurrences)", "-", "-"]
tot = sum(vals)
for n, v in zip(names, vals):
    print(f"{n:28s} {v:16d} {100 * v / max(1, tot):6.1f}%")
