"""Snapshot A/B (debug tool, not product): build the random-world snapshots named on the command
line with the library this process loads (KETO_MI355X_LIB_OVERRIDE for another build), save
each (keto_snapshot_save), and with --compare, diff two such files array by array.
  usage: tools/snapdiff.py save OUTDIR seed:rewrites ...   |   tools/snapdiff.py compare A B"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["set_row", "set_dst", "weight", "ent_obj", "slot_rel", "vkey", "all_off", "all_subj", "rev_off", "rev_nodes",
         "ns", "relinfo", "nsrel", "ops", "op_children", "op_items", "or_items", "ent_rank", "probe"]
INFO_BYTES, DEV_BYTES = 64, 232  # sizeof(keto_snapshot_info), sizeof(DevSnapshot)


def parse(path):
    b = open(path, "rb").read()
    o = 8 + 24 + INFO_BYTES + DEV_BYTES
    host = {}
    for name in ("ns_names", "rel_names"):
        n = struct.unpack_from("<Q", b, o)[0]
        o += 8
        for _ in range(n):
            ln = struct.unpack_from("<Q", b, o)[0]
            o += 8 + ln
    for name, size in (("ns", 16), ("ent_obj", 4), ("slot_rel", 4), ("relinfo", 4), ("nsrel", 4), ("ops", None),
                       ("op_children", 4), ("op_items", 4), ("or_items", 8)):
        n = struct.unpack_from("<Q", b, o)[0]
        o += 8
        if size is None:  # ops: element size from the next vector's position is unknown; read as bytes
            size = 16
        host[name] = b[o:o + n * size]
        o += n * size
    n = struct.unpack_from("<Q", b, o)[0]
    idx = struct.unpack_from(f"<{n}q", b, o + 8)
    o += 8 + 8 * n
    n = struct.unpack_from("<Q", b, o)[0]
    sizes = struct.unpack_from(f"<{n}Q", b, o + 8)
    o += 8 + 8 * n
    allocs = []
    for s in sizes:
        allocs.append(b[o:o + s])
        o += s
    dev = {NAMES[k]: (allocs[i] if i >= 0 else b"") for k, i in enumerate(idx)}
    return host, dev


def compare(a, b):
    ha, da = parse(a)
    hb, db = parse(b)
    for k in ha:
        print(f"host {k:12s} {'same' if ha[k] == hb[k] else 'DIFF'} ({len(ha[k])} / {len(hb[k])} B)")
    for k in NAMES:
        x, y = da[k], db[k]
        if k in ("rev_nodes", "probe"):  # unordered within a row / by insertion: compare as multisets
            same = len(x) == len(y) and np.array_equal(np.sort(np.frombuffer(x[:len(x) // 4 * 4], np.uint32)),
                                                       np.sort(np.frombuffer(y[:len(y) // 4 * 4], np.uint32)))
        else:
            same = x == y
        extra = ""
        if not same and len(x) == len(y) and len(x) % 4 == 0:
            u, v = np.frombuffer(x, np.uint32), np.frombuffer(y, np.uint32)
            d = np.nonzero(u != v)[0]
            extra = f" first diffs at u32 {d[:8].tolist()}: {u[d[:8]].tolist()} vs {v[d[:8]].tolist()}"
        print(f"dev  {k:12s} {'same' if same else 'DIFF'} ({len(x)} / {len(y)} B){extra}")


def save(outdir, specs):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "djy-keto_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    from product_helpers import product_snapshot
    from randworld import random_world
    os.makedirs(outdir, exist_ok=True)
    for spec in specs:
        seed, rw = spec.split(":")
        w, t, q, _ = random_world(int(seed), rewrites=rw == "1")
        snap = product_snapshot(w, t)
        snap.save(os.path.join(outdir, f"{seed}_{rw}.bin"))
        snap.close()
        print("saved", spec, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2], sys.argv[3:])
    else:
        compare(sys.argv[2], sys.argv[3])
