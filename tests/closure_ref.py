"""numpy restatement of the config-5 closure (csrc/partition.hip), test infrastructure: every
tuple of every object within `levels` subject-set hops of the batch's objects; with `subjects`
(a Check batch) subject-id tuples are kept only if they name one of those subjects.

The rows of an object come from `tuples`: a TUPLE_DT array (searched by object key), or a
function keys -> rows (synth.drive_object_tuples: the generator's own rows, for graphs that are
never held whole, e.g. config 5 at x40)."""
import numpy as np


def _keys(ns, obj):
    return (np.asarray(ns).astype(np.uint64) << np.uint64(32)) | np.asarray(obj).astype(np.uint64)


def _array_rows(tuples):
    k = _keys(tuples["ns"], tuples["obj"])
    order = np.argsort(k, kind="stable")
    ks = k[order]

    def rows(front):
        lo = np.searchsorted(ks, front, "left")
        hi = np.searchsorted(ks, front, "right")
        idx = np.concatenate([order[a:b] for a, b in zip(lo, hi)]) if len(front) else np.zeros(0, np.int64)
        return tuples[np.sort(idx)]
    return rows, tuples[:0]


def closure(tuples, ns, obj, levels, subjects=None):
    if callable(tuples):
        rows_of, empty = tuples, tuples(np.zeros(0, np.uint64))
    else:
        rows_of, empty = _array_rows(tuples)
    seen = np.zeros(0, np.uint64)
    front = np.unique(_keys(ns, obj))
    out = []
    subj = None if subjects is None else np.unique(np.asarray(subjects, np.uint32))
    for _ in range(levels):
        front = front[~np.isin(front, seen)]
        if not len(front):
            break
        seen = np.union1d(seen, front)
        rows = rows_of(front)
        if subj is not None:
            rows = rows[(rows["subj_kind"] == 1) | np.isin(rows["s_obj"], subj)]
        out.append(rows)
        ss = rows[rows["subj_kind"] == 1]
        front = np.unique(_keys(ss["s_ns"], ss["s_obj"]))
    return np.concatenate(out) if out else empty
