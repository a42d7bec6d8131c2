"""The oracle against the reference's own known-answer vectors (tests/golden).

This is what pins the CPU restatement: every expected value was asserted by
the reference's tests (file:line in each fixture's "src")."""
import numpy as np
import pytest

import refsem
from fixtures import fixture_names, load, world_for


@pytest.mark.parametrize("name", fixture_names())
def test_oracle_checks(name):
    fx = load(name)
    w, tuples, q = world_for(fx)
    orc = refsem.Oracle(w, tuples)
    for i, c in enumerate(fx.get("checks", [])):
        orc.set_limits(c.get("global", fx.get("global", 5)), fx.get("max_width", 100))
        mem, err, _ = orc.check(q[i:i + 1])
        allowed = bool(err[0] == 0 and mem[0] == refsem.IS_MEMBER)
        assert err[0] == c.get("err", 0), (name, c)
        assert allowed == c["allowed"], (name, c)


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n).get("expands")])
def test_oracle_expands(name):
    fx = load(name)
    w, tuples, _ = world_for(fx)
    orc = refsem.Oracle(w, tuples)
    for e in fx["expands"]:
        if "subject_id" in e:  # expand/handler.go:119-126: a subject id is its own leaf
            continue
        ns, obj, rel = refsem.parse_subject_set(e["subject"])
        nodes, _ = orc.expand(1, w.uuids.ids[obj], w.ns_names.ids[ns], w.rel_names.ids[rel], e["depth"])
        got = refsem.tree_to_nested(w, nodes)
        if e.get("exact"):
            assert got == e["tree"], (name, e["src"])
        assert refsem.trees_equal_unordered(got, e["tree"]), (name, e["src"], got)
