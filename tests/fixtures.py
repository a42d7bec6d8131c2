"""Shared loaders for the golden fixtures (test infrastructure)."""
import glob
import json
import os

import numpy as np

import refsem

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "*.json")))


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def world_for(fx):
    w = refsem.World(namespaces=fx["namespaces"], strict=fx.get("strict", False),
                     max_depth=fx.get("global", 5), max_width=fx.get("max_width", 100))
    tuples = w.tuple_array(fx["tuples"])
    checks = fx.get("checks", [])
    q = w.query_array([(c["query"], c.get("depth", 0)) for c in checks])
    # intern expand subjects up-front so every id is known at build time
    for e in fx.get("expands", []):
        if "subject" in e:
            ns, obj, rel = refsem.parse_subject_set(e["subject"])
            w.ns_names(ns), w.uuids(obj), w.rel_names(rel)
        else:
            w.uuids(e["subject_id"])
    return w, tuples, q
