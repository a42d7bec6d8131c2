"""Per-kernel split of rocprofv3 --pmc passes over bench.py's check path (tool).

usage: pmc_split.py OUT_JSON DIR [DIR ...]
Every DIR is one rocprofv3 --pmc pass (its own counter set).  Per kernel name: dispatches, and
each counter summed over its dispatches; per check batch: the sum divided by the number of
batches (dispatches of the batch's first kernel: fr_init / fb_check).  FETCH_SIZE is reported
x2 and both sizes in bytes (MI355X_MICROARCH.md HBM: gfx950 tallies 128-B requests at 64 B;
rocprofv3 reports KB)."""
import csv
import glob
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

out, dirs = sys.argv[1], sys.argv[2:]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            name = re.sub(r"\(.*$", "", name).replace("keto::", "")
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add((d, r["Dispatch_Id"]))
first = [n for n in tot if n.startswith("fr_init") or n.startswith("fb_check")]
batches = max((len({x[1] for x in disp[n]}) for n in first), default=1)
kern = {}
for name in sorted(tot, key=lambda n: -sum(tot[n].values())):
    c = tot[name]
    nd = len({x[1] for x in disp[name]})
    e = {"dispatches": nd, "per_batch": {}}
    for k, v in sorted(c.items()):
        if k == "FETCH_SIZE":
            e["per_batch"]["fetch_bytes"] = 2 * 1024 * v / batches
        elif k == "WRITE_SIZE":
            e["per_batch"]["write_bytes"] = 1024 * v / batches
        else:
            e["per_batch"][k] = v / batches
    kern[name] = e
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "djy-keto_amd", "keto_mi355x",
                   "libketo_mi355x.so")
res = {"batches": batches, "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
       "correction": "FETCH_SIZE x2 x1024, WRITE_SIZE x1024 (bytes); SQ cycle counters in quad-cycles",
       "kernels": kern}
json.dump(res, open(out, "w"), indent=1)
for name, e in kern.items():
    pb = e["per_batch"]
    s = "  ".join(f"{k}={v:.4g}" for k, v in pb.items())
    print(f"{name[:60]:60s} n={e['dispatches']:5d}  {s}")
