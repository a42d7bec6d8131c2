"""Divergence model of the Check interpreter (tool, not product).

Runs a sample of a Drive batch through the CPU emulation built with -DKETO_EMU_TRACE
(tools/cpuemu/trace.h), which records every query's steps (load slots) and the dispatch key of
every transition.  Then simulates the persistent grid: 64-lane waves, each lane pulling the next
query; a wave-step costs the number of DISTINCT keys its live lanes run (the divergent switch
executes each taken case body once per wave).  Compared with the same steps regrouped across
the waves of a block before every step (lanes sorted by their next key), which is what a
block-level regroup through LDS would buy.

  make -C tools/cpuemu OBJDIR=/tmp/emu_trace_obj LIB=/tmp/libketo_emu_trace.so "OPT=-O2 -DKETO_EMU_TRACE"
  KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=/tmp/libketo_emu_trace.so \
      KETO_EMU_TRACE_FILE=/tmp/trace.bin python tools/sim_regroup.py --run
  python tools/sim_regroup.py --sim /tmp/trace.bin
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "djy-keto_amd"))


def run(n, depth, trunc):
    import keto_mi355x as km
    from keto_mi355x import synth
    wl = synth.drive(depth=depth, n_groups=200_000, n_users=2_000_000, seed=3)
    q = synth.drive_queries(wl, n, seed=11)
    if trunc:
        q["max_depth"][: n // 100] = np.random.default_rng(0).integers(1, 5, n // 100)
    snap = km.Snapshot(wl.namespaces, wl.tuples, wl.ns_names, wl.rel_names, wl.n_uuids, strict=wl.strict)
    eng = km.CheckEngine(snap, km.Stream(0), max_read_depth=wl.max_depth, max_read_width=wl.max_width)
    a, e = eng.check_batch(q)
    print("allowed", a.mean())


def parse(path):
    b = np.fromfile(path, dtype=np.uint8)
    queries, cur, step = [], None, None
    i = 0
    n = len(b)
    while i < n:
        x = b[i]
        if x == 0xFE:
            cur = []
            queries.append(cur)
            step = []
            cur.append(step)
            i += 5
        elif x == 0xFF:
            step = []
            cur.append(step)
            i += 1
        else:
            step.append(int(x))
            i += 1
    return [[frozenset(s) for s in qs] for qs in queries], [[tuple(s) for s in qs] for qs in queries]


def simulate(queries, lanes_per_wave=64, n_lanes=64 * 64, regroup_block=0, key_fn=None):
    """returns (wave_steps, bodies, lane_steps); queries: list of lists of key sets"""
    rng = np.random.default_rng(0)
    order = list(rng.permutation(len(queries)))
    lane_q = [None] * n_lanes
    lane_s = [0] * n_lanes
    nxt = 0
    wave_steps = bodies = lane_steps = 0
    while True:
        for l in range(n_lanes):
            if lane_q[l] is None and nxt < len(order):
                lane_q[l] = order[nxt]
                lane_s[l] = 0
                nxt += 1
        live = [l for l in range(n_lanes) if lane_q[l] is not None]
        if not live:
            break
        steps = {l: queries[lane_q[l]][lane_s[l]] for l in live}
        if regroup_block:
            for b0 in range(0, n_lanes, regroup_block):
                blk = [l for l in live if b0 <= l < b0 + regroup_block]
                blk.sort(key=lambda l: key_fn(steps[l]))
                for w0 in range(0, len(blk), lanes_per_wave):
                    u = set()
                    for l in blk[w0:w0 + lanes_per_wave]:
                        u |= steps[l]
                    bodies += len(u)
                    wave_steps += 1
        else:
            for w0 in range(0, n_lanes, lanes_per_wave):
                u = set()
                any_live = False
                for l in range(w0, w0 + lanes_per_wave):
                    if lane_q[l] is not None:
                        u |= steps[l]
                        any_live = True
                if any_live:
                    bodies += len(u)
                    wave_steps += 1
        lane_steps += len(live)
        for l in live:
            lane_s[l] += 1
            if lane_s[l] >= len(queries[lane_q[l]]):
                lane_q[l] = None
    return wave_steps, bodies, lane_steps


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--sim")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--trunc", action="store_true")
    ap.add_argument("--lanes", type=int, default=64 * 32)
    a = ap.parse_args()
    if a.run:
        run(a.n, a.depth, a.trunc)
    if a.sim:
        sets, seqs = parse(a.sim)
        ntr = sum(len(s) for qs in seqs for s in qs)
        nst = sum(len(qs) for qs in seqs)
        print(f"{len(sets)} queries, {nst / len(sets):.1f} steps/query, {ntr / len(sets):.1f} transitions/query")
        ws, bo, ls = simulate(sets, n_lanes=a.lanes)
        print(f"baseline: wave_steps {ws}, bodies {bo}, bodies/wave-step {bo / ws:.1f}, lanes/wave-step {ls / ws:.1f}, "
              f"bodies per lane-step {bo / ls:.3f}")
        for blk in (256, 1024):
            for name, fn in (("first key", lambda s: min(s) if s else -1), ("key set", lambda s: tuple(sorted(s)))):
                ws2, bo2, ls2 = simulate(sets, n_lanes=a.lanes, regroup_block=blk, key_fn=fn)
                print(f"regroup block {blk} by {name}: bodies/wave-step {bo2 / ws2:.1f}, bodies per lane-step "
                      f"{bo2 / ls2:.3f} ({bo / bo2:.2f}x fewer bodies)")
