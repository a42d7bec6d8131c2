"""Debug tool: run one golden fixture's checks one query at a time (prints progress)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, os.path.join(R, "djy-keto_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import keto_mi355x as km  # noqa: E402
from fixtures import load, world_for  # noqa: E402
from product_helpers import product_snapshot, queries_to_product  # noqa: E402

fx = load(sys.argv[1] if len(sys.argv) > 1 else "rewrites")
w, t, q = world_for(fx)
snap = product_snapshot(w, t)
st = km.Stream(0)
for i, c in enumerate(fx["checks"][: int(sys.argv[2]) if len(sys.argv) > 2 else 3]):
    eng = km.CheckEngine(snap, st, max_read_depth=c.get("global", fx.get("global", 5)), max_read_width=100)
    print("query", i, c, flush=True)
    a, e = eng.check_batch(queries_to_product(q[i:i + 1]))
    print(" ->", a, e, "expected", c["allowed"], flush=True)
