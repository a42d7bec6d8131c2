"""Incremental-snapshot probe alone (tool): bench.store_probe on the Drive forest x scale (C4: 10).
Run with KETO_PATCH_VERBOSE=1 for the patch's phase times.   usage: tools/patch_probe.py [scale]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "djy-keto_amd")]

import keto_mi355x as km  # noqa: E402
from keto_mi355x import synth  # noqa: E402

import bench  # noqa: E402

wl = synth.drive_scaled(int(sys.argv[1]) if len(sys.argv) > 1 else 10, materialize=True)
q = synth.drive_queries(wl, 1 << 16, seed=3)
print(bench.store_probe(km, wl, q), flush=True)
