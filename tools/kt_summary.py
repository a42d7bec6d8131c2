"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace run (rocpd .db or kernel_trace.csv):
calls, average / min / max duration.  The tier-0 launch of a 2^20 batch is the row with the
largest grid of the uncounted interpreter.   usage: kt_summary.py <db-or-csv> [out.csv]"""
import csv
import sqlite3
import sys
from collections import defaultdict

src = sys.argv[1]
rows = []
if src.endswith(".db"):
    c = sqlite3.connect(src)
    for name, grid, wg, dur in c.execute("select name, grid_x, workgroup_x, duration from kernels"):
        rows.append((name, int(grid), int(wg), float(dur)))
else:
    for r in csv.DictReader(open(src)):
        rows.append((r["Kernel_Name"], int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"]),
                     int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0))),
                     float(r["End_Timestamp"]) - float(r["Start_Timestamp"])))
agg = defaultdict(list)
for name, grid, wg, dur in rows:
    short = name.replace("keto::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    agg[(short, grid, wg)].append(dur)
out = [("kernel", "grid", "block", "calls", "avg_us", "min_us", "max_us", "total_us")]
for (k, g, w), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    out.append((k, g, w, len(d), f"{sum(d) / len(d) / 1e3:.2f}", f"{min(d) / 1e3:.2f}", f"{max(d) / 1e3:.2f}",
                f"{sum(d) / 1e3:.1f}"))
w = csv.writer(open(sys.argv[2], "w", newline="")) if len(sys.argv) > 2 else None
for r in out:
    print(",".join(map(str, r)))
    if w:
        w.writerow(r)
