"""Schedule sensitivity (hard part 1).

The reference runs sibling sub-checks through checkgroup (concurrent_checkgroup.go:66-159):
results are taken in add order, but which siblings are already marked visited when a child
runs depends on goroutine timing.  The oracle's canonical order (refsem.c SCHED_EAGER, which
the kernels follow) marks the next sibling before child k runs -- what engine.go:151-162 does
in practice.  rs_check_ex re-runs each query under the other extreme (SCHED_SEQUENTIAL: child
k finishes before its sibling is marked) and flags a query as schedule-sensitive when some
visited scope both pruned a sibling and saw depth / width truncation, an error or AND / NOT.
These tests pin that the flag is sound for the two schedules (every disagreement is flagged)
and that it stays rare on the BASELINE workloads."""
import numpy as np
import pytest

import refsem
from fixtures import load, world_for
from product_helpers import queries_to_oracle, world_from_workload
from randworld import random_world


def test_sibling_marking_fixture_is_flagged():
    fx = load("sibling_marking_order")
    w, t, q = world_for(fx)
    orc = refsem.Oracle(w, t)
    orc.set_limits(5, 100)
    dec, err, flags, _ = orc.check_batch_ex(q, threads=1)
    assert list(dec) == [c["allowed"] for c in fx["checks"]]
    # depth 3: the sequential schedule denies what the eager one allows -> flagged
    assert flags[0] & refsem.F_SEQ_DIFFERS and flags[0] & refsem.F_SENSITIVE
    # depth 4: both schedules allow, and no truncation inside the scope -> not flagged
    assert flags[2] == 0


@pytest.mark.parametrize("rewrites", [True, False])
def test_flag_covers_every_disagreement_random_worlds(rewrites):
    n_diff = n_flag = n = 0
    for seed in range(60):
        w, t, q, _ = random_world(seed, rewrites=rewrites)
        orc = refsem.Oracle(w, t)
        orc.set_limits(w.max_depth, w.max_width)
        dec, err, flags, _ = orc.check_batch_ex(q, threads=4)
        d0, e0, _ = orc.check_batch(q, threads=4)
        np.testing.assert_array_equal(dec, d0)  # the canonical result is rs_check's
        np.testing.assert_array_equal(err, e0)
        diff = (flags & refsem.F_SEQ_DIFFERS) != 0
        sens = (flags & refsem.F_SENSITIVE) != 0
        assert not (diff & ~sens).any(), f"seed {seed}: a disagreement the criterion missed"
        n_diff += int(diff.sum())
        n_flag += int(sens.sum())
        n += len(q)
    assert n_flag >= n_diff
    assert n_flag < n  # the criterion is not vacuous


@pytest.mark.parametrize("wl_name", ["nested_groups", "drive"])
def test_sensitivity_rate_on_baseline_generators(wl_name):
    """small instances of the C2 / C3 generators: every disagreement between the two schedules
    is flagged; the conservative flag stays a minority and actual disagreements are rare (on
    these seeds: none)"""
    from keto_mi355x import synth
    if wl_name == "nested_groups":
        wl = synth.nested_groups(200_000, seed=5)
        q = synth.nested_groups_queries(wl, 20_000, seed=9, trunc_frac=0.05)
    else:
        wl = synth.drive(depth=6, n_groups=5000, n_users=20000, seed=11)
        q = synth.drive_queries(wl, 20_000, seed=4)
        q["max_depth"][:1000] = np.random.default_rng(0).integers(1, 5, 1000)
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    dec, err, flags, _ = orc.check_batch_ex(queries_to_oracle(q), threads=8)
    diff = (flags & refsem.F_SEQ_DIFFERS) != 0
    sens = (flags & refsem.F_SENSITIVE) != 0
    assert not (diff & ~sens).any()
    assert sens.mean() < 0.25
    assert diff.mean() < 0.01
