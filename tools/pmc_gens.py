"""Per-generation SQ counters of the frontier's fr_expand dispatches from rocprofv3 --pmc passes
(tool): a batch is an fr_init followed by its fr_expand dispatches (generation 0, 1, ...).
usage: pmc_gens.py DIR [DIR ...]  ->  per generation: mean of each counter over the batches"""
import csv
import glob
import sys
from collections import defaultdict

per = defaultdict(lambda: defaultdict(list))  # gen -> counter -> values
for d in sys.argv[1:]:
    rows = defaultdict(dict)  # dispatch -> {name, counters}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            rows[k]["name"] = r["Kernel_Name"]
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
    gen = None
    for k in sorted(rows):
        n = rows[k]["name"]
        if "fr_init" in n:
            gen = 0
        elif "fr_expand" in n and gen is not None:
            for c, v in rows[k].items():
                if c != "name":
                    per[gen][c].append(v)
            gen += 1
        elif "fr_reduce" in n:
            gen = None
cs = sorted({c for g in per for c in per[g]})
print("gen  " + " ".join(f"{c[3:]:>14s}" for c in cs))
for g in sorted(per):
    print(f"{g:3d}  " + " ".join(f"{sum(per[g][c]) / max(1, len(per[g][c])):14.4g}" for c in cs))
