"""fr_expand's global accesses by site (tool, not product): a KETO_FR_LOADPROF build counts, for
every load / store site of the goal code, the distinct 128-byte lines each wave touches -- the
L2 requests the site costs when it misses the L1 -- over one C4 batch (bench.py's graph and batch).
usage: KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=tools/ab/libketo_lp.so python3 tools/fr_loads.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd"))
import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

SITES = ["g0 read", "subject record", "goal row (ES / TTU)", "candidate set_row (ROW_LOAD)",
         "item rows (TTU item / chain)", "edge windows", "probe hash", "vkey", "routed bit", "child goal writes",
         "gfn + gvs writes", "occurrence writes"]
wl = synth.drive_scaled(10)
q = synth.drive_queries(wl, 1 << 20, seed=int(os.environ.get("SEED", "11")))
snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
st = km.Stream(0)
eng = km.CheckEngine(snap, st, max_read_depth=wl.max_depth, max_read_width=wl.max_width)
eng.check_batch(q)
st.counters(reset=True)
st.frontier_stats(reset=True)
eng.check_batch(q)
pt = st.counters(reset=True)["per_tier"]
goals = st.frontier_stats(reset=True)["goals"]
fields = ["rows", "edges", "probes", "out_nodes", "queries", "wave_steps", "lane_steps"]
vals = [pt[f][1] for f in fields] + [pt[f][2] for f in fields]
out = {"goals": goals, "queries": len(q), "lines_per_site": {}}
tot = sum(vals[:len(SITES)])
for name, v in zip(SITES, vals):
    out["lines_per_site"][name] = {"lines": v, "per_goal": v / max(1, goals), "per_check": v / len(q),
                                   "share": v / max(1, tot)}
    print(f"{name:32s} {v:14d}  {v / max(1, goals):6.2f}/goal  {v / len(q):7.2f}/check  {100 * v / max(1, tot):5.1f}%")
print(f"{'total':32s} {tot:14d}  {tot / max(1, goals):6.2f}/goal  {tot / len(q):7.2f}/check")
json.dump(out, open(os.environ.get("OUT", "/dev/null"), "w"), indent=1)
