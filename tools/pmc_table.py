"""Summarise rocprofv3 --pmc passes (rocprofv3 --pmc output) per kernel: counter sums per
dispatch for the Check interpreters' tier-0 launches.  usage: pmc_table.py gpurun_out/pmc_c2"""
import csv
import glob
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(float))
names = {}
for f in glob.glob(f"{sys.argv[1]}/p*/**/*counter_collection.csv", recursive=True) + \
        glob.glob(f"{sys.argv[1]}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = (f.split("/p")[-1][:1], r["Dispatch_Id"])
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = (r["Kernel_Name"][:60], int(r["Grid_Size"]))
agg = defaultdict(lambda: defaultdict(list))
for k, cs in vals.items():
    nm = names[k]
    for c, v in cs.items():
        agg[nm][c].append(v)
for nm, cs in sorted(agg.items(), key=lambda x: -max(max(v) for v in x[1].values())):
    print(nm)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {max(v):16.4g}  (n={len(v)})")
