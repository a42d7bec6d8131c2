"""Counter sums per dispatch of the Check interpreter's tier-0 launch from one rocprofv3 --pmc
output directory (tool).  usage: pmc_sum.py gpurun_out/pmc_x [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "check_kernel")
vals = defaultdict(lambda: defaultdict(float))
info = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        info[k] = (r["Kernel_Name"][:70], int(r["Grid_Size"]))
big = max(vals, key=lambda k: info[k][1] * 1e12 + sum(vals[k].values()) * 0, default=None)
cands = [k for k in vals if info[k][1] == info[big][1]] if big else []
best = max(cands, key=lambda k: vals[k].get("SQ_WAVE_CYCLES", 0)) if cands else None
if best:
    print(info[best])
    for c, v in sorted(vals[best].items()):
        print(f"   {c:28s} {v:14.4g}")
