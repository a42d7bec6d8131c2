"""Kernel summary of a rocprofv3 SQLite result (rocpd *_results.db): per kernel name the
launches, total / average / max duration, sorted by total time."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration), max(duration) from kernels "
                  "group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'max_us':>10s} {'pct':>6s}")
for name, n, s, a, m in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{name[:60]:60s} {n:6d} {s / 1e6:10.3f} {a / 1e3:10.1f} {m / 1e3:10.1f} {100 * s / tot:6.1f}")
