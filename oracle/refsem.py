"""TEST INFRASTRUCTURE ONLY -- Python driver for the C oracle (refsem.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It plays the part of the reference's Mapper
(internal/relationtuple/uuid_mapping.go:199-399: strings <-> ids) and of
namespace loading (internal/namespace/ast JSON, the format of
internal/schema/.snapshots/TestParser-*.json), independently of the
product's own C++ snapshot builder.
"""
from __future__ import annotations

import ctypes
import json
import os
import uuid as _uuid
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "librefsem.so")

TUPLE_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("kind", "<u4"), ("sid", "<u4"),
                     ("sns", "<u4"), ("srel", "<u4"), ("pad", "<u4"), ("shard_hi", "<u8"),
                     ("shard_lo", "<u8")])
QUERY_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("kind", "<u4"), ("sid", "<u4"),
                     ("sns", "<u4"), ("srel", "<u4"), ("depth", "<i4")])
AST_DT = np.dtype([("type", "<i4"), ("op", "<i4"), ("rel", "<u4"), ("computed", "<u4"),
                   ("child_begin", "<i4"), ("child_count", "<i4")])
REL_DT = np.dtype([("name", "<u4"), ("rewrite", "<i4"), ("has_ss_type", "<i4"), ("pad", "<i4")])
NS_DT = np.dtype([("configured", "<i4"), ("rel_begin", "<i4"), ("rel_count", "<i4"), ("pad", "<i4")])
TREE_DT = np.dtype([("type", "<u4"), ("kind", "<u4"), ("sid", "<u4"), ("sns", "<u4"), ("srel", "<u4"),
                    ("n_children", "<u4")])

REWRITE, CSS, TTU, INVERT = 0, 1, 2, 3
F_SENSITIVE, F_SEQ_DIFFERS, F_MAXEXP = 1, 2, 4  # rs_check_ex flags
IS_MEMBER, NOT_MEMBER, UNKNOWN = 1, 2, 0


class _Cfg(ctypes.Structure):
    _fields_ = [("n_ns", ctypes.c_uint32), ("n_relnames", ctypes.c_uint32), ("empty_rel", ctypes.c_uint32),
                ("ns", ctypes.c_void_p), ("rels", ctypes.c_void_p), ("n_rels", ctypes.c_uint32),
                ("ast", ctypes.c_void_p), ("n_ast", ctypes.c_uint32), ("children", ctypes.c_void_p),
                ("n_children", ctypes.c_uint32), ("vclass", ctypes.c_void_p), ("strict", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("max_width", ctypes.c_int32), ("shard_bytes", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_uint64), ("edges", ctypes.c_uint64), ("probes", ctypes.c_uint64),
                ("out_nodes", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run `make -C oracle`)")
        L = ctypes.CDLL(LIB_PATH)
        L.rs_build.restype = ctypes.c_void_p
        L.rs_build.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Cfg)]
        L.rs_free.argtypes = [ctypes.c_void_p]
        L.rs_set_limits.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.rs_set_reach.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.rs_check.restype = ctypes.c_int
        L.rs_check.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(Stats)]
        L.rs_check_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.rs_check_batch_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.rs_check_u_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.rs_expand.restype = ctypes.c_long
        L.rs_expand.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.POINTER(Stats)]
        _lib = L
    return _lib


# --------------------------------------------------------------------------
# tuple strings (ketoapi/enc_string.go:40-94)

def parse_tuple(s: str) -> dict:
    ns, rest = s.split(":", 1)
    obj, rest = rest.split("#", 1)
    rel, subj = rest.split("@", 1)
    subj = subj.strip("()")
    t = {"ns": ns, "obj": obj, "rel": rel}
    if ":" in subj:
        nso, _, srel = subj.partition("#")
        sns, sobj = nso.split(":", 1)
        t["subject_set"] = (sns, sobj, srel)
    else:
        t["subject_id"] = subj
    return t


def parse_subject_set(s: str):
    nso, _, rel = s.partition("#")
    ns, obj = nso.split(":", 1)
    return ns, obj, rel


class Interner:
    def __init__(self):
        self.ids: dict[str, int] = {}
        self.names: list[str] = []

    def __call__(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.names)
            self.ids[s] = i
            self.names.append(s)
        return i


def seeded_shard_ids(n: int, seed: int):
    """UUIDv4-shaped shard ids from a seeded generator (reference assigns uuid.NewV4()
    at insert, relationtuples.go:113).  Returns (hi, lo) uint64 arrays."""
    rng = np.random.Generator(np.random.PCG64(seed))
    hi = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64) << np.uint64(1)
    hi |= rng.integers(0, 2, size=n, dtype=np.int64).astype(np.uint64)
    lo = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64) << np.uint64(1)
    lo |= rng.integers(0, 2, size=n, dtype=np.int64).astype(np.uint64)
    # version 4 / variant bits, as in a real UUIDv4
    hi = (hi & ~np.uint64(0xF000)) | np.uint64(0x4000)
    lo = (lo & ~np.uint64(0xC000000000000000)) | np.uint64(0x8000000000000000)
    return hi, lo


@dataclass
class World:
    """Interned snapshot input: namespaces (AST JSON) + tuples, as the Go shim would hold them."""
    namespaces: dict
    strict: bool = False
    max_depth: int = 5
    max_width: int = 100
    ns_names: Interner = field(default_factory=Interner)
    rel_names: Interner = field(default_factory=Interner)
    uuids: Interner = field(default_factory=Interner)  # objects and subject ids share the UUID space

    def __post_init__(self):
        self.rel_names("")
        for n in self.namespaces:
            self.ns_names(n)
        self._walk_names()

    def _walk_names(self):
        def walk(node):
            if node is None:
                return
            if "operator" in node or "children" in node:
                for c in node.get("children") or []:
                    walk(c)
            elif "inverted" in node:
                walk(node["inverted"])
            else:
                self.rel_names(node["relation"])
                if "computed_subject_set_relation" in node:
                    self.rel_names(node["computed_subject_set_relation"])
        for rels in self.namespaces.values():
            for r in rels:
                self.rel_names(r["name"])
                for t in r.get("types") or []:
                    self.ns_names(t["namespace"])
                    if t.get("relation"):
                        self.rel_names(t["relation"])
                walk(r.get("rewrite"))

    # -- tuples ---------------------------------------------------------------
    def tuple_array(self, tuples: list, shard_hi=None, shard_lo=None) -> np.ndarray:
        out = np.zeros(len(tuples), dtype=TUPLE_DT)
        for i, t in enumerate(tuples):
            if isinstance(t, str):
                t = parse_tuple(t)
            out[i]["ns"] = self.ns_names(t["ns"])
            out[i]["obj"] = self.uuids(t["obj"])
            out[i]["rel"] = self.rel_names(t["rel"])
            if "subject_set" in t:
                sns, sobj, srel = t["subject_set"]
                out[i]["kind"] = 1
                out[i]["sid"] = self.uuids(sobj)
                out[i]["sns"] = self.ns_names(sns)
                out[i]["srel"] = self.rel_names(srel)
            else:
                out[i]["sid"] = self.uuids(t["subject_id"])
        if shard_hi is None:
            # insertion order == shard order for hand-written fixtures
            out["shard_hi"] = np.arange(len(tuples), dtype=np.uint64)
            out["shard_lo"] = 0
        else:
            out["shard_hi"] = shard_hi
            out["shard_lo"] = shard_lo
        return out

    def query_array(self, queries: list) -> np.ndarray:
        out = np.zeros(len(queries), dtype=QUERY_DT)
        for i, q in enumerate(queries):
            s, depth = (q, 0) if isinstance(q, str) else q
            t = parse_tuple(s)
            out[i]["ns"] = self.ns_names(t["ns"])
            out[i]["obj"] = self.uuids(t["obj"])
            out[i]["rel"] = self.rel_names(t["rel"])
            if "subject_set" in t:
                sns, sobj, srel = t["subject_set"]
                out[i]["kind"] = 1
                out[i]["sid"] = self.uuids(sobj)
                out[i]["sns"] = self.ns_names(sns)
                out[i]["srel"] = self.rel_names(srel)
            else:
                out[i]["sid"] = self.uuids(t["subject_id"])
            out[i]["depth"] = depth
        return out

    # -- namespace AST flattening (oracle-private) -------------------------------
    def flatten(self):
        n_ns = len(self.ns_names.names)
        nsarr = np.zeros(n_ns, dtype=NS_DT)
        rels, ast, children = [], [], []

        def add(node):
            """append one AST node; returns its index"""
            idx = len(ast)
            if "operator" in node or "children" in node:
                ast.append([REWRITE, 0 if node.get("operator", "or") == "or" else
                            (1 if node.get("operator") == "and" else 2), 0, 0, 0, 0])
                kids = [add(c) for c in (node.get("children") or [])]
                ast[idx][4] = len(children)
                ast[idx][5] = len(kids)
                children.extend(kids)
            elif "inverted" in node:
                ast.append([INVERT, 0, 0, 0, 0, 1])
                k = add(node["inverted"])
                ast[idx][4] = len(children)
                children.append(k)
            elif "computed_subject_set_relation" in node:
                ast.append([TTU, 0, self.rel_names(node["relation"]),
                            self.rel_names(node["computed_subject_set_relation"]), 0, 0])
            else:
                ast.append([CSS, 0, self.rel_names(node["relation"]), 0, 0, 0])
            return idx

        for name, rlist in self.namespaces.items():
            i = self.ns_names.ids[name]
            nsarr[i]["configured"] = 1
            nsarr[i]["rel_begin"] = len(rels)
            nsarr[i]["rel_count"] = len(rlist)
            for r in rlist:
                rw = add(r["rewrite"]) if r.get("rewrite") is not None else -1
                ss = int(any(t.get("relation") for t in (r.get("types") or [])))
                rels.append((self.rel_names(r["name"]), rw, ss, 0))
        self._n_ns_cfg = n_ns
        return nsarr, np.array(rels, dtype=REL_DT) if rels else np.zeros(0, REL_DT), \
            np.array([tuple(a) for a in ast], dtype=AST_DT) if ast else np.zeros(0, AST_DT), \
            np.array(children, dtype=np.int32)

    def vclass(self):
        n_ns, n_rel = len(self.ns_names.names), len(self.rel_names.names)
        cls = {}
        out = np.zeros((n_ns, n_rel), dtype=np.uint32)
        for a, ns in enumerate(self.ns_names.names):
            for b, rel in enumerate(self.rel_names.names):
                out[a, b] = cls.setdefault(ns + "-" + rel, len(cls))
        return out


class Oracle:
    """The oracle DB over a World + tuple array."""

    def __init__(self, world: World, tuples: np.ndarray, shard_bytes: bool = False):
        """tuples: TUPLE_DT, or the engine's keto_tuple layout (same 48-byte record with the
        shard_id as raw UUID bytes) with shard_bytes=True.  Not copied: kept referenced."""
        self.world = world
        self._keep = []
        nsarr, rels, ast, children = world.flatten()
        # any id interned after this point cannot appear in tuples: make sure the
        # vclass table covers names used later by queries by reserving room.
        vcls = world.vclass()
        cfg = _Cfg()
        cfg.n_ns = vcls.shape[0]
        cfg.n_relnames = vcls.shape[1]
        cfg.empty_rel = world.rel_names.ids[""]
        nsfull = np.zeros(vcls.shape[0], dtype=NS_DT)
        nsfull[: len(nsarr)] = nsarr
        for arr in (nsfull, rels, ast, children, vcls):
            self._keep.append(np.ascontiguousarray(arr))
        cfg.ns = self._keep[0].ctypes.data
        cfg.rels = self._keep[1].ctypes.data if len(rels) else None
        cfg.n_rels = len(rels)
        cfg.ast = self._keep[2].ctypes.data if len(ast) else None
        cfg.n_ast = len(ast)
        cfg.children = self._keep[3].ctypes.data if len(children) else None
        cfg.n_children = len(children)
        cfg.vclass = self._keep[4].ctypes.data
        cfg.strict = int(world.strict)
        cfg.max_depth = world.max_depth
        cfg.max_width = world.max_width
        self.n_ns, self.n_rel = vcls.shape
        cfg.shard_bytes = int(shard_bytes)
        tuples = np.ascontiguousarray(tuples)
        if tuples.dtype.itemsize != TUPLE_DT.itemsize:
            raise ValueError("tuple records must be 48 bytes")
        self._tuples = tuples  # rs_build indexes the caller's array in place
        self.db = lib().rs_build(tuples.ctypes.data, len(tuples), ctypes.byref(cfg))

    def close(self):
        if self.db:
            lib().rs_free(self.db)
            self.db = None

    def __del__(self):
        self.close()

    def set_limits(self, max_depth: int, max_width: int):
        lib().rs_set_limits(self.db, max_depth, max_width)

    def set_reach(self, on: bool):
        """the frontier restatement's reachability rule (rs_check_u): on by default"""
        lib().rs_set_reach(self.db, int(bool(on)))

    def _check_ids(self, q: np.ndarray):
        if len(q) and (int(q["ns"].max()) >= self.n_ns or int(q["rel"].max()) >= self.n_rel or
                       int((q["sns"] * (q["kind"] == 1)).max()) >= self.n_ns or
                       int((q["srel"] * (q["kind"] == 1)).max()) >= self.n_rel):
            raise ValueError("query names an id unknown when the oracle was built")

    def check(self, queries: np.ndarray):
        """returns (membership[], err[], Stats) one query at a time (single thread)"""
        q = np.ascontiguousarray(queries)
        self._check_ids(q)
        mem = np.zeros(len(q), dtype=np.int32)
        err = np.zeros(len(q), dtype=np.int32)
        st = Stats()
        e = ctypes.c_int32()
        for i in range(len(q)):
            mem[i] = lib().rs_check(self.db, q[i:i + 1].ctypes.data, ctypes.byref(e), ctypes.byref(st))
            err[i] = e.value
        return mem, err, st

    def check_batch(self, queries: np.ndarray, threads: int):
        q = np.ascontiguousarray(queries)
        self._check_ids(q)
        dec = np.zeros(len(q), dtype=np.uint8)
        err = np.zeros(len(q), dtype=np.int32)
        st = Stats()
        lib().rs_check_batch(self.db, q.ctypes.data, len(q), threads, dec.ctypes.data, err.ctypes.data,
                             ctypes.byref(st))
        return dec, err, st

    def check_batch_ex(self, queries: np.ndarray, threads: int):
        """canonical decisions plus the schedule-sensitivity flags (F_SENSITIVE, F_SEQ_DIFFERS):
        each query also runs under the sequential schedule (refsem.h rs_check_ex)"""
        q = np.ascontiguousarray(queries)
        self._check_ids(q)
        dec = np.zeros(len(q), dtype=np.uint8)
        err = np.zeros(len(q), dtype=np.int32)
        flags = np.zeros(len(q), dtype=np.uint32)
        st = Stats()
        lib().rs_check_batch_ex(self.db, q.ctypes.data, len(q), threads, dec.ctypes.data, err.ctypes.data,
                                flags.ctypes.data, ctypes.byref(st))
        return dec, err, flags, st

    def check_u_batch(self, queries: np.ndarray, threads: int, budget: int = 1024):
        """frontier semantics (refsem.h rs_check_u): decisions, errors, routed flags, goals and
        goal-tree generations per query"""
        q = np.ascontiguousarray(queries)
        self._check_ids(q)
        n = len(q)
        dec = np.zeros(n, dtype=np.uint8)
        err = np.zeros(n, dtype=np.int32)
        routed, goals, gens = (np.zeros(n, dtype=np.uint32) for _ in range(3))
        lib().rs_check_u_batch(self.db, q.ctypes.data, n, threads, budget, dec.ctypes.data, err.ctypes.data,
                               routed.ctypes.data, goals.ctypes.data, gens.ctypes.data)
        return dec, err, routed, goals, gens

    def expand(self, kind, sid, sns, srel, depth, cap=1 << 16):
        out = np.zeros(cap, dtype=TREE_DT)
        st = Stats()
        n = lib().rs_expand(self.db, kind, sid, sns, srel, depth, out.ctypes.data, cap, ctypes.byref(st))
        if n < 0:
            return self.expand(kind, sid, sns, srel, depth, cap * 4)
        return out[:n].copy(), st


def tree_to_nested(world: World, nodes: np.ndarray):
    """pre-order node array -> nested dict in ketoapi JSON shape (type, tuple subject, children)."""
    pos = [0]

    def subj(n):
        if n["kind"] == 0:
            return {"subject_id": world.uuids.names[n["sid"]]}
        return {"subject_set": {"namespace": world.ns_names.names[n["sns"]],
                                "object": world.uuids.names[n["sid"]],
                                "relation": world.rel_names.names[n["srel"]]}}

    def rec():
        n = nodes[pos[0]]
        pos[0] += 1
        d = {"type": "union" if n["type"] == 1 else "leaf", "tuple": subj(n)}
        kids = [rec() for _ in range(int(n["n_children"]))]
        if kids:
            d["children"] = kids
        return d

    if len(nodes) == 0:
        return None
    return rec()


def trees_equal_unordered(a, b) -> bool:
    """expand/testhelper.go:23-53 -- equality disregarding child order."""
    if a is None or b is None:
        return a is b
    if a["type"] != b["type"] or a["tuple"] != b["tuple"]:
        return False
    ca, cb = a.get("children") or [], b.get("children") or []
    if len(ca) != len(cb):
        return False
    return all(any(trees_equal_unordered(x, y) for y in cb) for x in ca)


def uuid5_nil(s: str) -> str:
    """uuid.NewV5(uuid.Nil, s) as used by the reference tests (engine_test.go:52-54)."""
    return str(_uuid.uuid5(_uuid.UUID(int=0), s))


def load_fixture(path: str) -> dict:
    with open(path) as f:
        return json.load(f)
