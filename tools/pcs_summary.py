"""Sum rocprofv3 PC samples (csv) per source line and per instruction (tool)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", list(rows[0].keys()) if rows else None, "samples:", len(rows))
if not rows:
    sys.exit(0)
keys = rows[0].keys()
line_k = next((k for k in keys if "Comment" in k), None)
inst_k = next((k for k in keys if k.lower() == "instruction"), None)
stall_k = next((k for k in keys if "Stall" in k or "stall" in k), None)
for name, k in (("source line", line_k), ("instruction", inst_k), ("stall reason", stall_k)):
    if not k:
        continue
    c = collections.Counter(r[k] for r in rows)
    tot = sum(c.values())
    print(f"\n== by {name} ({k}) ==")
    for v, n in c.most_common(40):
        print(f"{100.0 * n / tot:6.2f}%  {v[:150]}")
