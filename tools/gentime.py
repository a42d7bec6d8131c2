"""Median per-generation expansion time of the 2^20-query batches in a log written under
KETO_FR_GENTIME=1 (tool).  usage: gentime.py LOG [n]"""
import sys

import numpy as np

n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
rows = []
for line in open(sys.argv[1]):
    if line.startswith("[gentime]") and f" n {n} " in line:
        rows.append([float(x) for x in line.split("us:")[1].split()])
if not rows:
    print("no gentime lines")
    sys.exit(0)
G = max(len(r) for r in rows)
m = [float(np.median([r[g] for r in rows if len(r) > g])) for g in range(G)]
print(f"batches {len(rows)} total {sum(m):.0f} us | " + " ".join(f"{x:.0f}" for x in m))
