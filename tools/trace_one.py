"""Run one golden check through a chosen library build (debug aid)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", d) for d in ("djy-keto_amd", "oracle", "tests")]
import numpy as np
import keto_mi355x as km
from fixtures import load, world_for
from product_helpers import product_snapshot, queries_to_product
fx = load(sys.argv[1]); i = int(sys.argv[2])
w, t, q = world_for(fx)
snap = product_snapshot(w, t)
print("ids: ns", w.ns_names.ids, "rel", w.rel_names.ids)
eng = km.CheckEngine(snap, km.Stream(0), max_read_depth=fx.get("global", 5))
a, e = eng.check_batch(queries_to_product(q[i:i + 1]))
print("query", fx["checks"][i]["query"], "allowed", a, "err", e, "expected", fx["checks"][i]["allowed"])
