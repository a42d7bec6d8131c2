"""Snapshot loader from Keto's SQLite store (keto_mi355x/loader.py), checked on the CPU
through the oracle: the reference's known answers (tests/golden) must hold on the loaded
snapshot, whose ids, order and names all came from the database."""
import os

import numpy as np
import pytest

import refsem
from fixtures import fixture_names, load
from keto_mi355x.loader import KetoStore
from keto_sqlite import oracle_world, subject_of, write_store


def _store(tmp_path, fx, **kw):
    path = os.path.join(tmp_path, "keto.sqlite")
    nid = write_store(path, fx["tuples"], **kw)
    return KetoStore(path, fx["namespaces"], nid=nid if kw.get("networks", 1) > 1 else None,
                     strict=fx.get("strict", False)), nid


def _queries(store, fx):
    out = []
    for c in fx.get("checks", []):
        t = refsem.parse_tuple(c["query"])
        out.append(store.query(t["ns"], t["obj"], t["rel"], subject_of(t), c.get("depth", 0))[0])
    return np.array(out, dtype=out[0].dtype) if out else None


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("checks")])
def test_loaded_snapshot_keeps_the_reference_answers(tmp_path, name):
    fx = load(name)
    store, _ = _store(tmp_path, fx, seed=len(name))
    assert len(store.tuples) == len(fx["tuples"])
    # ORDER BY shard_id restored the fixture order from a shuffled insertion
    sh = store.tuples["shard_id"]
    assert all(bytes(sh[i]) < bytes(sh[i + 1]) for i in range(len(sh) - 1))
    w, t = oracle_world(store)
    orc = refsem.Oracle(w, t, shard_bytes=True)
    q = _queries(store, fx).view(refsem.QUERY_DT)
    for i, c in enumerate(fx["checks"]):
        orc.set_limits(c.get("global", fx.get("global", 5)), fx.get("max_width", 100))
        mem, err, _ = orc.check(q[i:i + 1])
        assert err[0] == c.get("err", 0), (name, c)
        assert bool(err[0] == 0 and mem[0] == refsem.IS_MEMBER) == c["allowed"], (name, c)


def test_network_filter_names_and_watermark(tmp_path):
    fx = load("docs_expand_beach")
    store, nid = _store(tmp_path, fx, networks=3)
    assert len(store.tuples) == len(fx["tuples"])  # other networks' rows are not read
    assert store.watermark == "2024-01-01 00:00:08"
    # every object/subject string comes back through keto_uuid_mappings
    objs = {refsem.parse_tuple(s)["obj"] for s in fx["tuples"]}
    assert objs <= set(store.strings)
    q = store.query("files", "/photos/beach.jpg", "access", "maureen")[0]
    assert store.strings[int(q["obj"])] == "/photos/beach.jpg" and store.strings[int(q["s_obj"])] == "maureen"
    unknown = store.query("nope", "never-written", "no-such-relation", "nobody")[0]
    assert unknown["obj"] >= store.n_uuids and unknown["s_obj"] >= store.n_uuids
    assert store.ns.names[int(unknown["ns"])].startswith("\x00") and store.rel.names[int(unknown["rel"])].startswith("\x00")
