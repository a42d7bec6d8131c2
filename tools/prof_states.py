"""Per-dispatch-key profile of the Check interpreter (tool, not product).  Needs an A/B build
with -DKETO_PROF_STATES=1 (rounds in which a wave runs each key: the union cost) or =2 (lanes
in each key), selected through KETO_MI355X_LIB_OVERRIDE; prints the 16 slots."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

w = synth.drive_scaled(1)
snap = km.Snapshot(w.namespaces, w.tuples, w.ns_names, w.rel_names, w.n_uuids, strict=w.strict, device=0)
q = synth.drive_queries(w, 1 << 20, seed=11)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=w.max_depth, max_read_width=w.max_width)
dq, da, de = km.DeviceBuffer(0, q.nbytes), km.DeviceBuffer(0, len(q)), km.DeviceBuffer(0, 4 * len(q))
dq.upload(st, q)
st.counters(reset=True)
eng.check_batch_device(dq, len(q), da, de, sync=True, count_work=True)
c = st.counters(reset=True)["per_tier"]
names = ["RET", "POP", "ROWOFF", "FSCAN", "ESDONE", "CNEXT", "VIS",  # slot 7 (CEDGE) not exported
         "TNEXT", "IA", "ES", "RW", "SC", "TTU", "INV"]  # slot 15 (TEDGE) not exported
fields = ["rows", "edges", "probes", "out_nodes", "queries", "wave_steps", "lane_steps"]
flat = [c[k][t] for t in (1, 2) for k in fields]  # counters[8..14], [16..22]
print("wave_steps", c["wave_steps"][0], "lane_steps", c["lane_steps"][0])
for n, v in zip(names, flat):
    print(f"{n:8s} {v}")
