"""Config-5 batch breakdown from a rocprofv3 kernel trace (tool): phases (closure, id remap, build,
check) of the last full batch, the heaviest kernels of each, and the largest idle gaps.
  usage: tools/c5_trace.py <kernel_trace.csv> [batch]  (batch: index of the k_query_keys launch
  that starts it; default 2, one of the one-call-per-batch runs before bench.py's timed region)"""
import collections
import csv
import sys


def nm(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)", "anon")
    if "rocprim" in n:
        for k in ("radix", "scan", "select", "unique"):
            if k in n.lower():
                return "cub_" + k
        return "cub"
    return n.split("(")[0].split("::")[-1]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_query_keys" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
seg = rows[starts[k]:starts[k + 1]]
first = {}
for i, r in enumerate(seg):
    first.setdefault(nm(r), i)
cuts = [("closure", 0), ("remap", first["k_ids_tuples"]), ("build", first["k_validate"]), ("check", first["resolve_kernel"])]
for k, (name, a) in enumerate(cuts):
    b = cuts[k + 1][1] if k + 1 < len(cuts) else len(seg)
    s = seg[a:b]
    st = int(s[0]["Start_Timestamp"])
    en = int(seg[b]["Start_Timestamp"]) if b < len(seg) else max(int(r["End_Timestamp"]) for r in s)
    agg = collections.Counter()
    for r in s:
        agg[nm(r)] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"{name:8s} span {(en - st) / 1e6:6.2f} ms, kernels {sum(agg.values()) / 1e6:6.2f} ms: " +
          ", ".join(f"{k} {v / 1e6:.2f}" for k, v in agg.most_common(6)))
gaps = sorted(((int(seg[i]["Start_Timestamp"]) - int(seg[i - 1]["End_Timestamp"]), nm(seg[i - 1]), nm(seg[i]))
               for i in range(1, len(seg))), reverse=True)
print("largest gaps:", "; ".join(f"{g / 1e6:.2f} ms {a} -> {b}" for g, a, b in gaps[:8]))
