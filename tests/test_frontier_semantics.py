"""The frontier engine's semantics on the CPU (oracle/refsem.c "Frontier semantics").

rs_check_u evaluates every query without visited pruning and routes a query when a key some
visited scope receives twice has a decisive occurrence, or when it spawns more than `budget`
goals.  Claim: every query it does not route decides exactly as the canonical DFS (rs_check).
These tests check the claim on the random worlds and on small instances of the BASELINE
generators, and that routing stays rare there."""
import numpy as np
import pytest

import refsem
from product_helpers import queries_to_oracle, world_from_workload
from randworld import random_world


@pytest.mark.parametrize("rewrites", [True, False])
@pytest.mark.parametrize("budget", [1024, 8])
def test_unrouted_queries_decide_as_the_dfs_random_worlds(rewrites, budget):
    n = n_routed = 0
    for seed in range(60):
        w, t, q, _ = random_world(seed, rewrites=rewrites)
        orc = refsem.Oracle(w, t)
        orc.set_limits(w.max_depth, w.max_width)
        dec, err, _ = orc.check_batch(q, threads=4)
        udec, uerr, routed, goals, gens = orc.check_u_batch(q, threads=4, budget=budget)
        ok = routed == 0
        np.testing.assert_array_equal(udec[ok], dec[ok], err_msg=f"seed {seed}")
        np.testing.assert_array_equal(uerr[ok], err[ok], err_msg=f"seed {seed}")
        assert (goals[ok] <= budget).all()
        n += len(q)
        n_routed += int(routed.sum())
    assert n_routed < n * (0.05 if budget > 100 else 0.9)


@pytest.mark.parametrize("wl_name", ["nested_groups", "drive"])
def test_routing_is_rare_on_baseline_generators(wl_name):
    from keto_mi355x import synth
    if wl_name == "nested_groups":
        wl = synth.nested_groups(300_000, seed=5)
        q = synth.nested_groups_queries(wl, 20_000, seed=9, trunc_frac=0.05)
    else:
        wl = synth.drive(depth=8, n_groups=20_000, n_users=100_000, seed=3)
        q = synth.drive_queries(wl, 20_000, seed=4)
        q["max_depth"][:1000] = np.random.default_rng(0).integers(1, 5, 1000)
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    qo = queries_to_oracle(q)
    dec, err, _ = orc.check_batch(qo, threads=8)
    udec, uerr, routed, goals, gens = orc.check_u_batch(qo, threads=8, budget=1024)
    ok = routed == 0
    np.testing.assert_array_equal(udec[ok], dec[ok])
    np.testing.assert_array_equal(uerr[ok], err[ok])
    assert routed.mean() < 0.01


def test_spawn_shaping_keeps_drive_goals_few():
    """Regression guard for the frontier's spawn-time shaping (oracle/refsem.c u_sub node_check,
    u_es chains, u_and_merge), which the product mirrors goal for goal: on a Drive world the
    restatement spawns under 20 goals per query (46 without the round-2 rules) and most queries
    finish within a handful of generations, with their decisions still the DFS's."""
    from keto_mi355x import synth
    wl = synth.drive(depth=8, n_groups=20_000, n_users=100_000, seed=3)
    q = synth.drive_queries(wl, 20_000, seed=4)
    w, _ = world_from_workload(wl, with_tuples=False)
    orc = refsem.Oracle(w, wl.tuples.view(refsem.TUPLE_DT), shard_bytes=True)
    orc.set_limits(wl.max_depth, wl.max_width)
    qo = queries_to_oracle(q)
    dec, err, _ = orc.check_batch(qo, threads=8)
    udec, uerr, routed, goals, gens = orc.check_u_batch(qo, threads=8, budget=1024)
    ok = routed == 0
    np.testing.assert_array_equal(udec[ok], dec[ok])
    assert goals.mean() < 20.0
    assert gens.mean() < 8.0

