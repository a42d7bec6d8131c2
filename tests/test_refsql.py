"""The SQL-mode restatement (oracle/refsql.py: the engine recursion issuing the reference's
own four statements against in-memory SQLite, bench.py's second CPU baseline) agrees with the
in-memory oracle (refsem.c) -- two independent restatements -- on the reference's known
answers, random worlds and a Drive sample; and it loads only the rows the sample can read."""
import numpy as np
import pytest

import refsem
import refsql
from fixtures import fixture_names, load, world_for
from randworld import random_world


def _engine(w, t, q, orc, depth):
    rows = refsql.closure_rows(orc, q["ns"], q["obj"], depth + 1)
    return refsql.SqlEngine(rows, w.namespaces, w.ns_names.names, w.rel_names.names, max_depth=depth,
                            max_width=w.max_width, strict=w.strict)


def _run(eng, w, q):
    out = []
    for r in q:
        subj = (0, int(r["sid"])) if r["kind"] == 0 else (1, w.ns_names.names[r["sns"]], int(r["sid"]),
                                                          w.rel_names.names[r["srel"]])
        m, e = eng.check(w.ns_names.names[r["ns"]], int(r["obj"]), w.rel_names.names[r["rel"]], subj, int(r["depth"]))
        out.append((int(e == 0 and m == refsql.IS_MEMBER), e))
    return np.array([a for a, _ in out], np.uint8), np.array([e for _, e in out], np.int32)


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("checks")])
def test_sql_mode_golden(name):
    fx = load(name)
    w, t, q = world_for(fx)
    orc = refsem.Oracle(w, t)
    for i, c in enumerate(fx["checks"]):
        g = c.get("global", fx.get("global", 5))
        orc.set_limits(g, fx.get("max_width", 100))
        eng = _engine(w, t, q[i:i + 1], orc, g)
        eng.max_width = fx.get("max_width", 100)
        a, e = _run(eng, w, q[i:i + 1])
        assert int(e[0]) == c.get("err", 0), (name, c)
        assert bool(a[0]) == c["allowed"], (name, c)


@pytest.mark.parametrize("seed", list(range(0, 40, 2)))
def test_sql_mode_random_worlds(seed):
    w, t, q, _ = random_world(seed, rewrites=seed % 4 == 0)
    orc = refsem.Oracle(w, t)
    orc.set_limits(w.max_depth, w.max_width)
    dec, err, _ = orc.check_batch(q, threads=2)
    eng = _engine(w, t, q, orc, w.max_depth)
    a, e = _run(eng, w, q)
    np.testing.assert_array_equal(e, err)
    np.testing.assert_array_equal(a, dec)



def test_sql_mode_drive_sample():
    from keto_mi355x import synth
    from product_helpers import queries_to_oracle, world_from_workload
    wl = synth.drive(depth=6, n_groups=5000, n_users=20000, seed=11)
    q = queries_to_oracle(synth.drive_queries(wl, 400, seed=4))
    q["depth"][:40] = np.random.default_rng(0).integers(1, 5, 40)
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, err, _ = orc.check_batch(q, threads=4)
    rows = refsql.closure_rows(orc, q["ns"], q["obj"], wl.max_depth + 1)
    assert 0 < len(rows) < len(wl.tuples)
    eng = refsql.SqlEngine(rows, wl.namespaces, wl.ns_names, wl.rel_names, max_depth=wl.max_depth,
                           max_width=wl.max_width, strict=wl.strict)
    a, e = _run(eng, w, q)
    np.testing.assert_array_equal(a, dec)
    np.testing.assert_array_equal(e, err)
