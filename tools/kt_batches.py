"""Per-batch device time of the frontier check path from a rocprofv3 --kernel-trace run (rocpd
.db or kernel_trace.csv), to set beside bench.py's roofline.kernel_ms (HIP events around the
check path of every timed batch).

A batch of the frontier path is the request resolution pass, fr_init, one fr_expand per
generation, one fr_reduce per generation (deepest first) with fr_repeat before generation 0, and
the DFS interpreter on any routed queries.  Batches are split at each resolve pass whose grid
covers `--n` queries and that an fr_init follows (bench.py's 2^20: the latency probe's smaller
batches and the counted DFS batch are left out).  Reported per batch: the summed kernel
durations ("busy") and the span from the resolve pass's start to the last kernel's end before
the next batch ("span", what the HIP events see).   usage: kt_batches.py <db-or-csv> [--n 1048576] [--out summary.csv]"""
import argparse
import csv
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--out")
a = ap.parse_args()

rows = []  # (start, end, short name, grid)
if a.src.endswith(".db"):
    c = sqlite3.connect(a.src)
    for name, grid, st, en in c.execute("select name, grid_x, start, end from kernels order by start"):
        rows.append((int(st), int(en), name, int(grid)))
else:
    for r in csv.DictReader(open(a.src)):
        g = int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], g))
rows.sort()
PATH = ("fr_init", "fr_expand", "fr_reduce", "fr_repeat", "check_kernel<false")


def short(n):
    return n.replace("keto::(anonymous namespace)::", "").replace("void ", "").split("(")[0]


batches = []  # list of lists of rows
cur = None
pending = None  # a full-size resolve pass, until the kernel after it shows which path it starts
for r in rows:
    nm = r[2]
    if "resolve_kernel" in nm:  # the next batch's resolve pass: this batch is over
        cur = None
        pending = r if r[3] >= a.n else None
        continue
    if "fr_init" in nm:
        cur = ([pending, r] if pending else [r]) if r[3] >= a.n else None
        pending = None
        if cur is not None:
            batches.append(cur)
        continue
    if "__amd_rocclr" in nm:  # (the frontier's control memsets between resolve and fr_init)
        continue
    pending = None
    if cur is None:
        continue
    if any(p in nm for p in PATH):
        cur.append(r)

per_kernel = defaultdict(list)
busy, span, gens = [], [], []
for b in batches:
    busy.append(sum(e - s for s, e, _, _ in b))
    span.append(max(e for _, e, _, _ in b) - b[0][0])
    gens.append(sum(1 for r in b if "fr_expand" in r[2]))
    acc = defaultdict(int)
    for s, e, nm, _ in b:
        acc[short(nm)] += e - s
    for k, v in acc.items():
        per_kernel[k].append(v)
out = [("quantity", "value")]
if batches:
    nb = len(batches)
    out += [("batches", nb), ("avg_generations", f"{sum(gens) / nb:.1f}"),
            ("avg_busy_ms", f"{sum(busy) / nb / 1e6:.3f}"), ("avg_span_ms", f"{sum(span) / nb / 1e6:.3f}"),
            ("min_span_ms", f"{min(span) / 1e6:.3f}"), ("max_span_ms", f"{max(span) / 1e6:.3f}")]
    for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1])):
        out.append((f"busy_ms[{k}]", f"{sum(v) / nb / 1e6:.3f}"))
w = csv.writer(open(a.out, "w", newline="")) if a.out else None
for r in out:
    print(",".join(map(str, r)))
    if w:
        w.writerow(r)
