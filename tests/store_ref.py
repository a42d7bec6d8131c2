"""Test infrastructure: TransactRelationTuples restated on host arrays
(persistence/sql/relationtuples.go:277-287 -> WriteRelationTuples :262-275, then
DeleteRelationTuples :168-189 with whereSubject :128-150)."""
import numpy as np


def content_keys(t: np.ndarray) -> np.ndarray:
    """(ns, obj, rel, kind, s_obj, s_ns|0, s_rel|0) rows: a subject id matches on its id only"""
    k = np.zeros((len(t), 7), dtype=np.uint64)
    is_set = t["subj_kind"] == 1
    k[:, 0], k[:, 1], k[:, 2] = t["ns"], t["obj"], t["rel"]
    k[:, 3] = is_set
    k[:, 4] = t["s_obj"]
    k[:, 5] = np.where(is_set, t["s_ns"], 0)
    k[:, 6] = np.where(is_set, t["s_rel"], 0)
    return k


def transact(tuples: np.ndarray, ins: np.ndarray, dele: np.ndarray) -> np.ndarray:
    allt = np.concatenate([tuples, ins])
    if len(dele) == 0:
        return allt
    kd = {tuple(r) for r in content_keys(dele).tolist()}
    keep = np.array([tuple(r) not in kd for r in content_keys(allt).tolist()], dtype=bool)
    return allt[keep]
