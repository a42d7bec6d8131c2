"""Counter totals per kernel name over every dispatch in one or more rocprofv3 --pmc output
directories (tool).  usage: pmc_kernels.py dir [dir ...]  ->  kernel: counter = sum"""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[name].add(r["Dispatch_Id"])
for name in sorted(tot, key=lambda n: -max(tot[n].values())):
    print(f"{name}  ({len(calls[name])} dispatches)")
    for c, v in sorted(tot[name].items()):
        print(f"   {c:28s} {v:14.4g}")
