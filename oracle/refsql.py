"""TEST / BENCH INFRASTRUCTURE ONLY -- "restated reference (SQL mode)": the Check engine with
every storage read issued as the reference's own SQL against an in-memory SQLite store.

bench.py's CPU baseline beside the in-memory port (refsem.c).  The reference engine (Go) cannot
run here, but its cost model is: one goroutine recursion whose every hop is one of four
statements against the persister -- with the in-memory SQLite DSN of its tests
(internal/x/dbx/dsn_sqlite.go:24-29) that is SQLite in the same process.  This module restates
the recursion of internal/check/{engine,rewrites,binop}.go in Python (schedule: refsem.c
SCHED_EAGER) and issues, per hop, the statement the reference issues:

  ES rows        TraverseSubjectSetExpansion  persistence/sql/traverser.go:68-92 (pages of 1000)
  OR shortcut    TraverseSubjectSetRewrite    traverser.go:146-154 (relation IN (...) LIMIT 1)
  TTU rows       GetRelationTuples            persistence/sql/relationtuples.go:216-227 (pages of 100)
  direct         ExistsRelationTuples         relationtuples.go:253-260

against the reference's table and indexes (migrations/sql/...sqlite.up.sql:14-80).  UUID
columns hold integer ids and shard_id the row's shard rank: every predicate and ORDER BY
compares them exactly as the UUIDs would.  Only the rows the sampled queries can read are
loaded (refsem.h rs_closure: objects within max_depth + 1 subject-set hops), so a 1B-tuple
graph's sample fits in memory; rows of an object are complete, so the answers are the whole
graph's (tests/test_partition.py pins that closure argument).
"""
from __future__ import annotations

import ctypes
import sqlite3
import sys

import numpy as np

ROW_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("kind", "<u4"), ("sid", "<u4"), ("sns", "<u4"),
                   ("srel", "<u4"), ("pad", "<u4"), ("pos", "<u8")])

DDL = """
CREATE TABLE keto_relation_tuples (
  shard_id INTEGER NOT NULL, nid INTEGER NOT NULL, namespace VARCHAR(200) NOT NULL, object INTEGER NOT NULL,
  relation VARCHAR(64) NOT NULL, subject_id INTEGER NULL, subject_set_namespace VARCHAR(200) NULL,
  subject_set_object INTEGER NULL, subject_set_relation VARCHAR(64) NULL, commit_time TIMESTAMP NOT NULL,
  PRIMARY KEY (shard_id, nid));
CREATE INDEX keto_relation_tuples_uuid_subject_ids_idx ON keto_relation_tuples (nid, namespace, object, relation,
  subject_id) WHERE subject_set_namespace IS NULL AND subject_set_object IS NULL AND subject_set_relation IS NULL;
CREATE INDEX keto_relation_tuples_uuid_subject_sets_idx ON keto_relation_tuples (nid, namespace, object, relation,
  subject_set_namespace, subject_set_object, subject_set_relation) WHERE subject_id IS NULL;
CREATE INDEX keto_relation_tuples_uuid_full_idx ON keto_relation_tuples (nid, namespace, object, relation, subject_id,
  subject_set_namespace, subject_set_object, subject_set_relation, commit_time);
"""
NID = 1
UNKNOWN, IS_MEMBER, NOT_MEMBER = 0, 1, 2
ERR_NO_RELATION, ERR_INTERNAL, ERR_NOT_IMPLEMENTED = 1, 2, 3
MAX_RECURSION = 4096  # refsem.c's guard: a zero-cost rewrite cycle never returns in the reference


def closure_rows(orc, ns, obj, levels: int, max_rows: int = 0):
    """rows an oracle (refsem.Oracle) holds for every object within `levels` hops (None when
    there are more than max_rows > 0 of them)"""
    import refsem
    L = refsem.lib()
    L.rs_closure.restype = ctypes.c_size_t
    L.rs_closure.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_size_t]
    ns = np.ascontiguousarray(ns, np.uint32)
    obj = np.ascontiguousarray(obj, np.uint32)
    need = L.rs_closure(orc.db, ns.ctypes.data, obj.ctypes.data, len(ns), levels, None, 0)
    if max_rows and need > max_rows:
        return None
    out = np.zeros(max(1, need), ROW_DT)
    L.rs_closure(orc.db, ns.ctypes.data, obj.ctypes.data, len(ns), levels, out.ctypes.data, need)
    return out[:need]


class SqlEngine:
    """check.Engine restated over SQL.  ns_names / rel_names: id -> name of the rows' ids."""

    def __init__(self, rows: np.ndarray, namespaces: dict, ns_names, rel_names, max_depth=5, max_width=100,
                 strict=False):
        self.ns_names, self.rel_names = list(ns_names), list(rel_names)
        self.config = namespaces
        self.max_depth, self.max_width, self.strict = max_depth, max_width, strict
        self.con = sqlite3.connect(":memory:")
        self.con.executescript(DDL)
        ns, rel = self.ns_names, self.rel_names
        data = [(int(r["pos"]), NID, ns[r["ns"]], int(r["obj"]), rel[r["rel"]],
                 int(r["sid"]) if r["kind"] == 0 else None, ns[r["sns"]] if r["kind"] == 1 else None,
                 int(r["sid"]) if r["kind"] == 1 else None, rel[r["srel"]] if r["kind"] == 1 else None, 0)
                for r in rows]
        self.con.executemany("INSERT INTO keto_relation_tuples VALUES (?,?,?,?,?,?,?,?,?,?)", data)
        self.con.commit()
        self.statements = 0
        self.guard = 0
        sys.setrecursionlimit(max(sys.getrecursionlimit(), 8 * MAX_RECURSION + 1000))

    # -- namespace.ASTRelationFor (internal/namespace/definitions.go:37-62) ---------------
    def ast_relation_for(self, ns, rel):
        if rel == "":
            return None, 0
        rels = self.config.get(ns)
        if not rels:  # unknown namespace, or one without relation config
            return None, 0
        for r in rels:
            if r["name"] == rel:
                return r, 0
        return None, ERR_NO_RELATION

    # -- the four statements -----------------------------------------------------------------
    @staticmethod
    def _subject(subj):
        if subj[0] == 0:
            return ("subject_id = ? AND subject_set_namespace IS NULL AND subject_set_object IS NULL AND "
                    "subject_set_relation IS NULL", [subj[1]])
        return ("subject_id IS NULL AND subject_set_namespace = ? AND subject_set_object = ? AND "
                "subject_set_relation = ?", [subj[1], subj[2], subj[3]])

    def traverse_subject_set_expansion(self, ns, obj, rel, subj):
        """traverser.go:53-121: [(sns, sobj, srel, found)] in shard order, stops at found"""
        where, args = self._subject(subj)
        out, shard = [], -1
        while True:
            self.statements += 1
            rows = self.con.execute(f"""
SELECT current.shard_id, current.subject_set_namespace, current.subject_set_object, current.subject_set_relation,
       EXISTS(SELECT 1 FROM keto_relation_tuples WHERE nid = current.nid AND namespace = current.subject_set_namespace
              AND object = current.subject_set_object AND relation = current.subject_set_relation AND {where}) AS found
FROM keto_relation_tuples AS current
WHERE current.nid = ? AND current.shard_id > ? AND current.namespace = ? AND current.object = ? AND
      current.relation = ? AND current.subject_id IS NULL
ORDER BY current.nid, current.shard_id LIMIT ?""", args + [NID, shard, ns, obj, rel, 1000]).fetchall()
            for r in rows:
                out.append((r[1], r[2], r[3], bool(r[4])))
                if r[4]:
                    return out
            if len(rows) == 1000:
                shard = rows[-1][0]
            else:
                return out

    def traverse_subject_set_rewrite(self, ns, obj, subj, relations):
        """traverser.go:123-191: found (relation IN (...) LIMIT 1)"""
        if not relations:
            return False
        where, args = self._subject(subj)
        self.statements += 1
        q = (f"SELECT 1 FROM keto_relation_tuples WHERE nid = ? AND namespace = ? AND object = ? AND {where} AND "
             f"relation IN ({','.join('?' * len(relations))}) LIMIT 1")
        return self.con.execute(q, [NID, ns, obj] + args + list(relations)).fetchone() is not None

    def get_relation_tuples(self, ns, obj, rel):
        """relationtuples.go:207-247, pages of 100 (persister.go:44): subjects in shard order"""
        out, shard = [], -1
        while True:
            self.statements += 1
            rows = self.con.execute(
                "SELECT shard_id, subject_id, subject_set_namespace, subject_set_object, subject_set_relation "
                "FROM keto_relation_tuples WHERE nid = ? AND shard_id > ? AND namespace = ? AND object = ? AND "
                "relation = ? ORDER BY shard_id, nid LIMIT ?", (NID, shard, ns, obj, rel, 101)).fetchall()
            page = rows[:100]
            out += page
            if len(rows) > 100:
                shard = page[-1][0]
            else:
                return out

    def exists(self, ns, obj, rel, subj):
        """relationtuples.go:249-261"""
        where, args = self._subject(subj)
        self.statements += 1
        return self.con.execute(f"SELECT EXISTS(SELECT 1 FROM keto_relation_tuples WHERE nid = ? AND namespace = ? "
                                f"AND object = ? AND relation = ? AND {where})",
                                [NID, ns, obj, rel] + args).fetchone()[0] == 1

    # -- the engine (internal/check/engine.go, rewrites.go, binop.go) -------------------------
    def check(self, ns, obj, rel, subj, depth=0):
        """CheckRelationTuple (engine.go:76-95) -> (membership, err); subj = (0, id) or
        (1, ns, obj, rel) with names for namespaces / relations"""
        d = depth if 0 < depth <= self.max_depth else self.max_depth
        self.guard = 0
        return self._is_allowed(ns, obj, rel, subj, d, False, None)

    def _is_allowed(self, ns, obj, rel, subj, d, skip_direct, vs):
        if d <= 0:
            return UNKNOWN, 0
        self.guard += 1
        try:
            if self.guard > MAX_RECURSION:
                return UNKNOWN, ERR_INTERNAL
            return self._is_allowed_body(ns, obj, rel, subj, d, skip_direct, vs)
        finally:
            self.guard -= 1

    def _is_allowed_body(self, ns, obj, rel, subj, d, skip_direct, vs):
        r, err = self.ast_relation_for(ns, rel)
        if err:
            return UNKNOWN, err
        has_rw = r is not None and r.get("rewrite") is not None
        can_ss = not self.strict or r is None or any(t.get("relation") for t in (r.get("types") or []))
        if has_rw:
            res = self._rewrite(ns, obj, r["rewrite"], subj, d, vs)
            if res[1] or res[0] == IS_MEMBER:
                return res
        if (not self.strict or not has_rw) and not skip_direct and d - 1 > 0:
            if self.exists(ns, obj, rel, subj):
                return IS_MEMBER, 0
        if can_ss:
            res = self._expand_subject(ns, obj, rel, subj, d - 1, vs)
            if res[1] or res[0] == IS_MEMBER:
                return res
        return NOT_MEMBER, 0

    def _expand_subject(self, ns, obj, rel, subj, d, vs):
        if d <= 0:
            return UNKNOWN, 0
        own = vs is None
        if own:
            vs = set()  # graph.InitVisited; key = ns-rel + object (UniqueID, definitions.go:114-116)
        rows = self.traverse_subject_set_expansion(ns, obj, rel, subj)
        if any(f for *_, f in rows):
            return IS_MEMBER, 0
        if len(rows) > self.max_width:
            rows = rows[:self.max_width - 1]
        it = iter(rows)

        def advance():
            for sns, sobj, srel, _ in it:
                k = (sns + "-" + srel, sobj)
                if k in vs:
                    continue
                vs.add(k)
                return (sns, sobj, srel)
            return None

        nxt = advance()  # eager sibling marking (refsem.c SCHED_EAGER)
        while nxt is not None:
            cur, nxt = nxt, advance()
            res = self._is_allowed(cur[0], cur[1], cur[2], subj, d, True, vs)
            if res[1] or res[0] == IS_MEMBER:
                if not own:
                    while advance() is not None:
                        pass
                return res
        return NOT_MEMBER, 0

    def _rewrite(self, ns, obj, rw, subj, d, vs):
        if d <= 0:
            return UNKNOWN, 0
        op = rw.get("operator", "or")
        if op not in ("or", "and"):
            return UNKNOWN, ERR_NOT_IMPLEMENTED
        self.guard += 1
        try:
            if self.guard > MAX_RECURSION:
                return UNKNOWN, ERR_INTERNAL
            return self._rewrite_body(ns, obj, rw, subj, d, vs, op)
        finally:
            self.guard -= 1

    def _rewrite_body(self, ns, obj, rw, subj, d, vs, op):
        children = rw.get("children") or []
        n = 0
        if op == "or":
            css = [c["relation"] for c in children if self._kind(c) == "css"]
            if css:
                n += 1
                rels = []
                for rn in css:
                    ar, _ = self.ast_relation_for(ns, rn)
                    if self.strict and ar is not None and ar.get("rewrite") is not None:
                        continue
                    rels.append(rn)
                if self.traverse_subject_set_rewrite(ns, obj, subj, rels):
                    return IS_MEMBER, 0
                for rn in css:
                    res = self._is_allowed(ns, obj, rn, subj, d - 1, True, vs)
                    if res[1] or res[0] == IS_MEMBER:
                        return res
        for c in children:
            if op == "or" and self._kind(c) == "css":
                continue
            n += 1
            res = self._child(ns, obj, c, subj, d, 1, vs)
            if op == "or":
                if res[1] or res[0] == IS_MEMBER:
                    return res
            elif res[1] or res[0] != IS_MEMBER:
                return NOT_MEMBER, res[1]
        return (IS_MEMBER, 0) if op == "and" and n else (NOT_MEMBER, 0)

    @staticmethod
    def _kind(c):
        if "operator" in c or "children" in c:
            return "rw"
        if "inverted" in c:
            return "not"
        if "computed_subject_set_relation" in c:
            return "ttu"
        return "css"

    def _child(self, ns, obj, c, subj, d, nested_cost, vs):
        k = self._kind(c)
        if k == "ttu":
            if d < 0:
                return UNKNOWN, 0
            for row in self.get_relation_tuples(ns, obj, c["relation"]):
                if row[1] is not None:  # subject ids are skipped (rewrites.go:280)
                    continue
                res = self._is_allowed(row[2], row[3], c["computed_subject_set_relation"], subj, d - 1, False, vs)
                if res[1] or res[0] == IS_MEMBER:
                    return res
            return NOT_MEMBER, 0
        if k == "css":
            if d < 0:
                return UNKNOWN, 0
            return self._is_allowed(ns, obj, c["relation"], subj, d, False, vs)
        if k == "rw":
            return self._rewrite(ns, obj, c, subj, d - nested_cost, vs)
        if d < 0:  # inverted (rewrites.go:136-200)
            return UNKNOWN, 0
        self.guard += 1
        try:
            if self.guard > MAX_RECURSION:
                return UNKNOWN, ERR_INTERNAL
            m, e = self._child(ns, obj, c["inverted"], subj, d, 0, vs)
        finally:
            self.guard -= 1
        return (NOT_MEMBER if m == IS_MEMBER else IS_MEMBER if m == NOT_MEMBER else m), e
