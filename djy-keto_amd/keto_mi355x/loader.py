"""Snapshot loader from a live Keto SQL store, host side.

Reads a network's relation tuples from Keto's SQLite database in the reference's own
iteration order.  The schema is
`internal/persistence/sql/migrations/sql/20230228091200000000_add-on-delete-cascade-to-relationship.sqlite.up.sql:14-49`:
`keto_relation_tuples(shard_id, nid, namespace, object, relation, subject_id,
subject_set_namespace, subject_set_object, subject_set_relation, commit_time)`.

- The read is `... WHERE nid = ? ORDER BY shard_id`, the order of every row scan in
  `persistence/sql/traverser.go:88` and `relationtuples.go:216-230`.
- UUID columns hold gofrs/uuid's `Value()`, the canonical text form.  Its text order is
  the byte order the device builder sorts rows by.
- Strings for output come from `keto_uuid_mappings(id, string_representation)`
  (`persistence/sql/uuid_mapping.go:19-33`).
- Query strings map to UUIDs the way `Mapper.FromTuple` does for reads: `UUIDv5(nid, s)`
  without writing (`uuid_mapping.go:35-74`, readOnly).

The result interns everything to the C ABI's dense ids:
- namespaces: the config's first, then any others the table holds;
- relations: `""` first, then the config's, then the table's, plus one reserved name that
  stands for "a relation name the snapshot has never seen";
- UUIDs: every UUID that appears in a tuple.

A query naming an unknown UUID gets an id >= n_uuids. The kernels treat that as an absent
entity and still evaluate it.
"""
from __future__ import annotations

import sqlite3
import uuid as _uuid

import numpy as np

from . import _abi
from .engine import Interner, Snapshot

UNKNOWN_RELATION = "\x00unknown-relation"  # never declared, so its status is the reference's
# "relation does not exist" in configured namespaces and nil in legacy ones
UNKNOWN_NAMESPACE = "\x00unknown-namespace"  # a namespace without configuration, like any
# name a query brings that the snapshot has never seen

_SQL = ("SELECT shard_id, namespace, object, relation, subject_id, subject_set_namespace, "
        "subject_set_object, subject_set_relation, commit_time FROM keto_relation_tuples "
        "WHERE nid = ? ORDER BY shard_id")


def _uuid_text(v) -> str:
    if isinstance(v, (bytes, bytearray, memoryview)) and len(v) == 16:
        return str(_uuid.UUID(bytes=bytes(v)))
    return str(_uuid.UUID(str(v)))


class KetoStore:
    """One network's tuples at read time, interned for keto_snapshot_build."""

    def __init__(self, path: str, namespaces: dict, nid: str | None = None, strict: bool = False,
                 chunk: int = 1 << 16):
        con = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
        try:
            if nid is None:
                ids = [r[0] for r in con.execute("SELECT DISTINCT nid FROM keto_relation_tuples")]
                if len(ids) != 1:
                    raise ValueError(f"database holds {len(ids)} networks: pass nid")
                nid = ids[0]
            self.nid = _uuid.UUID(_uuid_text(nid))
            self.namespaces, self.strict = namespaces, strict
            self.ns = Interner(list(namespaces))
            self.rel = Interner([""])
            for rels in namespaces.values():
                for r in rels:
                    self.rel(r["name"])
            self.uuids = Interner()
            recs, self.watermark = [], None
            cur = con.execute(_SQL, (str(nid) if not isinstance(nid, (bytes, bytearray)) else nid,))
            while True:
                rows = cur.fetchmany(chunk)
                if not rows:
                    break
                recs.append(self._intern(rows))
            self.tuples = np.concatenate(recs) if recs else np.zeros(0, dtype=_abi.TUPLE_DT)
            self.rel(UNKNOWN_RELATION)
            self.ns(UNKNOWN_NAMESPACE)
            self.n_uuids = len(self.uuids.names)
            strings = dict(con.execute("SELECT id, string_representation FROM keto_uuid_mappings"))
            norm = {}
            for k, v in strings.items():
                try:
                    norm[_uuid_text(k)] = v
                except ValueError:
                    continue
            # Mapper.ToTree output: the mapped string, or the UUID text itself if unmapped
            self.strings = [norm.get(u, u) for u in self.uuids.names]
        finally:
            con.close()

    def _intern(self, rows) -> np.ndarray:
        t = np.zeros(len(rows), dtype=_abi.TUPLE_DT)
        ns, rel, u = self.ns, self.rel, self.uuids
        sh = bytearray()
        for i, (shard, n, obj, r, sid, sns, sobj, srel, ct) in enumerate(rows):
            sh += _uuid.UUID(_uuid_text(shard)).bytes
            t["ns"][i], t["obj"][i], t["rel"][i] = ns(n), u(_uuid_text(obj)), rel(r)
            if sid is not None:
                t["s_obj"][i] = u(_uuid_text(sid))
            else:
                t["subj_kind"][i] = 1
                t["s_ns"][i], t["s_obj"][i], t["s_rel"][i] = ns(sns), u(_uuid_text(sobj)), rel(srel)
            if ct is not None and (self.watermark is None or str(ct) > self.watermark):
                self.watermark = str(ct)
        t["shard_id"] = np.frombuffer(bytes(sh), dtype=np.uint8).reshape(-1, 16)
        return t

    # ---- the shim's Mapper for requests (uuid_mapping.go:269-317, read-only) --------------

    def uuid_id(self, s: str) -> int:
        """API string -> dense id of UUIDv5(nid, s).  A UUID the snapshot does not hold is
        looked up, never interned (a long-running service sees unboundedly many): it maps to
        the one sentinel id n_uuids, which every kernel treats as absent."""
        i = self.uuids.ids.get(str(_uuid.uuid5(self.nid, s)))
        return self.n_uuids if i is None else i

    def rel_id(self, r: str) -> int:
        i = self.rel.ids.get(r)
        return self.rel.ids[UNKNOWN_RELATION] if i is None else i

    def ns_id(self, n: str) -> int:
        """a namespace neither configured nor in the table maps to the reserved unconfigured
        one (the REST handler answers such checks itself, check/handler.go:167-172)"""
        i = self.ns.ids.get(n)
        return self.ns.ids[UNKNOWN_NAMESPACE] if i is None else i

    def query(self, ns: str, obj: str, rel: str, subject, max_depth: int = 0) -> np.ndarray:
        """one QUERY_DT record; subject = "id" or (ns, obj, rel)"""
        q = np.zeros(1, dtype=_abi.QUERY_DT)
        q["ns"] = self.ns_id(ns)
        q["obj"], q["rel"], q["max_depth"] = self.uuid_id(obj), self.rel_id(rel), max_depth
        if isinstance(subject, str):
            q["s_obj"] = self.uuid_id(subject)
        else:
            q["subj_kind"], q["s_ns"] = 1, self.ns_id(subject[0])
            q["s_obj"], q["s_rel"] = self.uuid_id(subject[1]), self.rel_id(subject[2])
        return q

    def snapshot(self, device: int = 0) -> Snapshot:
        return Snapshot(self.namespaces, self.tuples, self.ns.names, self.rel.names, self.n_uuids,
                        strict=self.strict, device=device)

    def name_tables(self):
        """id -> string tables for keto_trees_to_json / keto_trees_to_proto"""
        from .api import NameTables
        return NameTables(self.ns.names, self.rel.names, self.strings)
