"""Host-side mirror of the reference engine API over the C ABI.

  CheckEngine.check_is_member(tuple, rest_depth)  ~ check.Engine.CheckIsMember   (internal/check/engine.go:65-71)
  CheckEngine.check_relation_tuple(...)            ~ check.Engine.CheckRelationTuple (engine.go:76-95)
  CheckEngine.check_batch(queries)                 ~ the batched form the Go shim's dispatcher uses
  ExpandEngine.build_tree(subject, rest_depth)     ~ expand.Engine.BuildTree       (internal/expand/engine.go:43-52)

Every evaluation runs in libketo_mi355x's gfx950 kernels; this module only
interns strings (the Mapper role, internal/relationtuple/uuid_mapping.go) and
moves buffers.  A missing library or device raises -- there is no CPU path.
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass, field

import numpy as np

from . import _abi
from ._abi import KetoError, check, lib

IS_MEMBER, NOT_MEMBER = 1, 2


def shard_bytes(hi: np.ndarray, lo: np.ndarray) -> np.ndarray:
    """(hi, lo) uint64 halves -> big-endian 16-byte UUIDs (ORDER BY shard_id byte order)."""
    out = np.empty((len(hi), 16), dtype=np.uint8)
    out[:, :8] = hi.astype(">u8").view(np.uint8).reshape(-1, 8)
    out[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(-1, 8)
    return out


class Interner:
    def __init__(self, names=()):
        self.ids: dict[str, int] = {}
        self.names: list[str] = []
        for n in names:
            self(n)

    def __call__(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.names)
            self.ids[s] = i
            self.names.append(s)
        return i


@dataclass
class Mapper:
    """String <-> dense id tables (the Go shim's job; uuid_mapping.go:199-399)."""
    namespaces: Interner = field(default_factory=Interner)
    relations: Interner = field(default_factory=Interner)
    uuids: Interner = field(default_factory=Interner)


class Snapshot:
    """Immutable device-resident snapshot (CSR rows + compiled rewrite program)."""

    def __init__(self, namespaces_json: str | dict, tuples: np.ndarray, ns_names: list, rel_names: list,
                 n_uuids: int, strict: bool = False, device: int = 0, device_tuples: tuple | None = None,
                 store: "TupleStore | None" = None, base: "Snapshot | None" = None):
        """tuples: host TUPLE_DT array; or tuples=None and device_tuples=(device pointer, count)
        for records already resident on `device` (keto_snapshot_build_device); or tuples=None
        and store=TupleStore for its current content (keto_store_snapshot) -- with base= an
        earlier snapshot of that store, by patching it (keto_store_snapshot_patch; `patched`
        says whether the patch ran or the full build)."""
        if isinstance(namespaces_json, dict):
            namespaces_json = json.dumps(namespaces_json)
        self._ns = (ctypes.c_char_p * max(1, len(ns_names)))(*[n.encode() for n in ns_names])
        self._rel = (ctypes.c_char_p * max(1, len(rel_names)))(*[r.encode() for r in rel_names])
        self._json = namespaces_json.encode()
        cfg = _abi.SnapshotConfig(len(ns_names), self._ns, len(rel_names), self._rel, n_uuids, self._json,
                                  int(strict), device)
        h = ctypes.c_void_p()
        self.patched = False
        if store is not None and base is not None:
            p = ctypes.c_int32()
            check(lib().keto_store_snapshot_patch(store.handle, base.handle, ctypes.byref(cfg), ctypes.byref(h),
                                                  ctypes.byref(p)))
            self.patched = bool(p.value)
        elif store is not None:
            check(lib().keto_store_snapshot(store.handle, ctypes.byref(cfg), ctypes.byref(h)))
        elif device_tuples is not None:
            ptr, count = device_tuples
            check(lib().keto_snapshot_build_device(ctypes.byref(cfg), ptr, count, ctypes.byref(h)))
        else:
            tuples = np.ascontiguousarray(tuples, dtype=_abi.TUPLE_DT)
            check(lib().keto_snapshot_build(ctypes.byref(cfg), tuples.ctypes.data, len(tuples), ctypes.byref(h)))
        self.handle = h
        self.device = device
        self.ns_names, self.rel_names = list(ns_names), list(rel_names)
        _abi.track(self)

    def info(self) -> dict:
        inf = _abi.SnapshotInfo()
        check(lib().keto_snapshot_info_get(self.handle, ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in inf._fields_}

    def advance(self, store: "TupleStore") -> bool:
        """this store snapshot advanced in place to the store's current version
        (keto_store_snapshot_advance): False = unchanged, the delta needs a full build.  No batch
        may be in flight on it."""
        a = ctypes.c_int32()
        check(lib().keto_store_snapshot_advance(store.handle, self.handle, ctypes.byref(a)))
        return bool(a.value)

    def save(self, path: str):
        """the snapshot to a file (keto_snapshot_save): the restart artefact"""
        check(lib().keto_snapshot_save(self.handle, str(path).encode()))

    @classmethod
    def load(cls, path: str, ns_names: list, rel_names: list, device: int = 0) -> "Snapshot":
        """a saved snapshot back onto `device` (keto_snapshot_load), without a rebuild"""
        self = cls.__new__(cls)
        h = ctypes.c_void_p()
        check(lib().keto_snapshot_load(str(path).encode(), device, ctypes.byref(h)))
        self.handle, self.device = h, device
        self.ns_names, self.rel_names = list(ns_names), list(rel_names)
        _abi.track(self)
        return self

    def close(self):
        if getattr(self, "handle", None):
            lib().keto_snapshot_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class TupleStore:
    """Device-resident tuple store of one network (keto_store_*): TransactRelationTuples
    deltas, versioned snapshots (the version is the snaptoken)."""

    def __init__(self, tuples: np.ndarray, device: int = 0):
        t = np.ascontiguousarray(tuples, dtype=_abi.TUPLE_DT)
        h = ctypes.c_void_p()
        check(lib().keto_store_create(device, t.ctypes.data if len(t) else None, len(t), 0, ctypes.byref(h)))
        self.handle, self.device = h, device
        _abi.track(self)

    def transact(self, insert: np.ndarray | None = None, delete: np.ndarray | None = None):
        ins = np.ascontiguousarray(insert if insert is not None else np.zeros(0, _abi.TUPLE_DT), dtype=_abi.TUPLE_DT)
        dele = np.ascontiguousarray(delete if delete is not None else np.zeros(0, _abi.TUPLE_DT), dtype=_abi.TUPLE_DT)
        check(lib().keto_store_transact(self.handle, ins.ctypes.data if len(ins) else None, len(ins),
                                        dele.ctypes.data if len(dele) else None, len(dele), 0))

    def info(self) -> tuple:
        n, v = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().keto_store_info(self.handle, ctypes.byref(n), ctypes.byref(v)))
        return n.value, v.value

    def close(self):
        if getattr(self, "handle", None):
            lib().keto_store_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class Stream:
    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().keto_stream_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device
        _abi.track(self)

    def sync(self):
        check(lib().keto_stream_sync(self.handle))

    def counters(self, reset: bool = False) -> dict:
        """{'rows': total, ..., 'per_tier': {'rows': [t0, t1, t2], ...}}"""
        c = _abi.WorkCounters()
        check(lib().keto_stream_counters(self.handle, ctypes.byref(c), int(reset)))
        per = {k: list(getattr(c, k)) for k, _ in c._fields_}
        out = {k: sum(v) for k, v in per.items()}
        out["per_tier"] = per
        return out

    def frontier_stats(self, reset: bool = False) -> dict:
        """frontier-engine activity on this stream (keto_stream_frontier_stats)"""
        c = _abi.FrontierStats()
        check(lib().keto_stream_frontier_stats(self.handle, ctypes.byref(c), int(reset)))
        return {k: int(getattr(c, k)) for k, _ in c._fields_}

    def expand_time(self, reset: bool = False) -> tuple:
        """(ms summed, batches) of the Expand traversals on this stream (keto_stream_expand_time)"""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        check(lib().keto_stream_expand_time(self.handle, ctypes.byref(ms), ctypes.byref(n), int(reset)))
        return ms.value, n.value

    def kernel_time(self, reset: bool = False) -> tuple:
        """(summed main-kernel ms, launches) timed with HIP events on this stream"""
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        check(lib().keto_stream_kernel_time(self.handle, ctypes.byref(ms), ctypes.byref(n), int(reset)))
        return ms.value, n.value

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_double()
        check(lib().keto_stream_last_kernel_ms(self.handle, ctypes.byref(ms)))
        return ms.value

    def close(self):
        if getattr(self, "handle", None):
            lib().keto_stream_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class DeviceBuffer:
    """Raw device allocation (keto_device_alloc) for HBM-resident batches."""

    def __init__(self, device: int, nbytes: int):
        p = ctypes.c_void_p()
        check(lib().keto_device_alloc(device, max(1, nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p, nbytes
        _abi.track(self)

    def upload(self, stream: Stream, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(lib().keto_memcpy_h2d(stream.handle, self.ptr, arr.ctypes.data, arr.nbytes))

    def download(self, stream: Stream, arr: np.ndarray):
        check(lib().keto_memcpy_d2h(stream.handle, arr.ctypes.data, self.ptr, arr.nbytes))
        return arr

    def free(self):
        if self.ptr:
            lib().keto_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class PinnedArray:
    """numpy array over pinned host memory (keto_host_alloc): the buffers of KETO_F_ASYNC batches,
    whose copies then run asynchronously on the stream."""

    def __init__(self, n: int, dtype):
        dtype = np.dtype(dtype)
        self.nbytes = max(1, n * dtype.itemsize)
        p = ctypes.c_void_p()
        check(lib().keto_host_alloc(self.nbytes, ctypes.byref(p)))
        self.ptr = p
        buf = (ctypes.c_uint8 * self.nbytes).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=np.uint8, count=n * dtype.itemsize).view(dtype)
        _abi.track(self)

    def free(self):
        if self.ptr:
            self.array = None
            lib().keto_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class CheckEngine:
    """check.Engine over the GPU snapshot (limits = limit.max_read_depth/max_read_width)."""

    def __init__(self, snapshot: Snapshot, stream: Stream | None = None, max_read_depth: int = 5,
                 max_read_width: int = 100):
        self.snapshot = snapshot
        self.stream = stream or Stream(snapshot.device)
        self.limits = _abi.Limits(max_read_depth, max_read_width)

    def check_batch(self, queries: np.ndarray, count_work: bool = False, err_detail: bool = False):
        """queries: QUERY_DT array (host).  Returns (allowed uint8[n], err int32[n]); with
        err_detail, err = 1 | relation-name id << 8 for `relation %q does not exist`."""
        q = np.ascontiguousarray(queries, dtype=_abi.QUERY_DT)
        allowed = np.zeros(len(q), dtype=np.uint8)
        err = np.zeros(len(q), dtype=np.int32)
        flags = (_abi.F_COUNT_WORK if count_work else 0) | (_abi.F_ERR_DETAIL if err_detail else 0)
        check(lib().keto_check_batch(self.snapshot.handle, self.stream.handle, q.ctypes.data, len(q),
                                     ctypes.byref(self.limits), allowed.ctypes.data, err.ctypes.data, flags))
        return allowed, err

    def check_batch_async(self, queries: np.ndarray, allowed: np.ndarray, err: np.ndarray):
        """KETO_F_ASYNC over host buffers (pinned: PinnedArray): H2D of the queries, the kernels
        and D2H of the decisions are enqueued on the stream and the call returns; the outputs are
        valid after stream.sync().  queries: QUERY_DT, or QUERY16_DT records (keto_check_batch16:
        half the H2D bytes)."""
        assert queries.dtype in (_abi.QUERY_DT, _abi.QUERY16_DT) and queries.flags.c_contiguous
        assert len(allowed) >= len(queries) and len(err) >= len(queries)
        fn = lib().keto_check_batch16 if queries.dtype == _abi.QUERY16_DT else lib().keto_check_batch
        check(fn(self.snapshot.handle, self.stream.handle, queries.ctypes.data, len(queries), ctypes.byref(self.limits),
                 allowed.ctypes.data, err.ctypes.data, _abi.F_ASYNC))

    def check_batch16(self, queries16: np.ndarray, err_detail: bool = False):
        """keto_check_batch16: QUERY16_DT records (pack_queries16) -> (allowed uint8[n], err int32[n])"""
        q = np.ascontiguousarray(queries16, dtype=_abi.QUERY16_DT)
        allowed = np.zeros(len(q), dtype=np.uint8)
        err = np.zeros(len(q), dtype=np.int32)
        check(lib().keto_check_batch16(self.snapshot.handle, self.stream.handle, q.ctypes.data, len(q),
                                       ctypes.byref(self.limits), allowed.ctypes.data, err.ctypes.data,
                                       _abi.F_ERR_DETAIL if err_detail else 0))
        return allowed, err

    def check_batch_device(self, d_queries: DeviceBuffer, n: int, d_allowed: DeviceBuffer, d_err: DeviceBuffer,
                           sync: bool = True, count_work: bool = False):
        flags = _abi.F_DEVICE_PTRS | (0 if sync else _abi.F_ASYNC) | (_abi.F_COUNT_WORK if count_work else 0)
        check(lib().keto_check_batch(self.snapshot.handle, self.stream.handle, d_queries.ptr, n,
                                     ctypes.byref(self.limits), d_allowed.ptr, d_err.ptr, flags))

    def check_relation_tuple(self, query_rec: np.ndarray):
        """-> (membership-as-bool, error code) for one QUERY_DT record."""
        a, e = self.check_batch(np.atleast_1d(query_rec))
        return bool(a[0]), int(e[0])

    def check_is_member(self, query_rec: np.ndarray) -> bool:
        """CheckIsMember (engine.go:65-71): the bool, or the reference's error -- for an
        undeclared relation its exact text `relation %q does not exist`
        (namespace/definitions.go:61), naming the relation the walk rejected."""
        a, e = self.check_batch(np.atleast_1d(query_rec), err_detail=True)
        code, rel = int(e[0]) & 0xFF, int(e[0]) >> 8
        if code == _abi.QERR_NO_RELATION:
            names = self.snapshot.rel_names
            name = names[rel] if rel < len(names) else names[int(np.atleast_1d(query_rec)["rel"][0])] \
                if int(np.atleast_1d(query_rec)["rel"][0]) < len(names) else ""
            raise KetoError(code, f"relation {json.dumps(name)} does not exist")
        if code:
            raise KetoError(code, "not implemented" if code == _abi.QERR_NOT_IMPLEMENTED else "check failed")
        return bool(a[0])


def pack_queries16(queries: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
    """QUERY_DT records -> QUERY16_DT (keto_pack_query16): KetoError(KETO_E_LIMIT) for a request
    outside the 16-byte form (namespace >= 4096, relation >= 1024, depth outside int16)"""
    q = np.ascontiguousarray(queries, dtype=_abi.QUERY_DT)
    if out is None:
        out = np.zeros(len(q), dtype=_abi.QUERY16_DT)
    assert out.dtype == _abi.QUERY16_DT and out.flags.c_contiguous and len(out) >= len(q)
    check(lib().keto_pack_query16(q.ctypes.data if len(q) else None, len(q), out.ctypes.data if len(out) else None))
    return out


class ExpandEngine:
    """expand.Engine.BuildTree over the GPU snapshot."""

    def __init__(self, snapshot: Snapshot, stream: Stream | None = None, max_read_depth: int = 5):
        self.snapshot = snapshot
        self.stream = stream or Stream(snapshot.device)
        self.limits = _abi.Limits(max_read_depth, 100)
        self._cap = 0  # output nodes the last batch needed: sizes the next one (no count-pass retry)

    def build_trees(self, roots: np.ndarray, out: "PinnedArray | None" = None):
        """roots: SUBJSET_DT array -> (nodes TREE_DT, offsets uint64[n+1], err int32[n]).
        out: a PinnedArray of TREE_DT (keto_host_alloc) the trees are copied into -- one DMA
        instead of a staged pageable copy -- while it holds them."""
        r = np.ascontiguousarray(roots, dtype=_abi.SUBJSET_DT)
        n = len(r)
        offs = np.zeros(n + 1, dtype=np.uint64)
        err = np.zeros(max(1, n), dtype=np.int32)
        cap = max(64, 16 * n, self._cap)
        while True:
            if out is not None and len(out.array) >= cap:
                nodes, cap = out.array, len(out.array)
            else:
                nodes = np.empty(cap, dtype=_abi.TREE_DT)  # filled by the library up to offs[n]
            rc = lib().keto_expand_batch(self.snapshot.handle, self.stream.handle, r.ctypes.data, n,
                                         ctypes.byref(self.limits), nodes.ctypes.data, cap, offs.ctypes.data,
                                         err.ctypes.data)
            if rc == _abi.KETO_E_CAPACITY:
                cap = self._cap = int(offs[n]) + 1
                continue
            check(rc)
            return nodes[: int(offs[n])], offs, err[:n]

    def build_trees_spans(self, roots: np.ndarray, out: "PinnedArray | None" = None):
        """keto_expand_batch_spans: the same trees in completion order -> (nodes TREE_DT, first
        uint64[n], count uint32[n], err int32[n]); root i's tree is nodes[first[i]:first[i] + count[i]].
        With out (a PinnedArray, keto_host_alloc) the library writes each tree into it as its walk
        ends, over PCIe, while the other roots still walk."""
        r = np.ascontiguousarray(roots, dtype=_abi.SUBJSET_DT)
        n = len(r)
        first = np.zeros(max(1, n), dtype=np.uint64)
        count = np.zeros(max(1, n), dtype=np.uint32)
        err = np.zeros(max(1, n), dtype=np.int32)
        total = ctypes.c_uint64(0)
        cap = max(64, 16 * n, self._cap)
        while True:
            if out is not None and len(out.array) >= cap:
                nodes, cap = out.array, len(out.array)
            else:
                nodes = np.empty(cap, dtype=_abi.TREE_DT)
            rc = lib().keto_expand_batch_spans(self.snapshot.handle, self.stream.handle, r.ctypes.data, n,
                                               ctypes.byref(self.limits), nodes.ctypes.data, cap, first.ctypes.data,
                                               count.ctypes.data, err.ctypes.data, ctypes.byref(total))
            if rc == _abi.KETO_E_CAPACITY:
                cap = self._cap = int(total.value) + 1
                continue
            check(rc)
            return nodes[: int(total.value)], first[:n], count[:n], err[:n]

    def build_tree(self, ns: int, obj: int, rel: int, rest_depth: int = 0):
        """expand.Engine.BuildTree (expand/engine.go:43-52) for one subject-set root:
        the pre-order TREE_DT nodes, or None for a nil tree."""
        nodes, offs, err = self.build_trees(np.array([(ns, obj, rel, rest_depth)], dtype=_abi.SUBJSET_DT))
        if err[0]:
            raise KetoError(int(err[0]), "expand failed")
        return nodes[int(offs[0]):int(offs[1])] if offs[1] > offs[0] else None


class Dispatcher:
    """Request coalescing (keto_dispatcher_*): many threads call check(); one dispatcher
    thread in the library batches whatever is queued into each launch.  ctypes releases the
    GIL for the blocking call, so Python threads coalesce like goroutines in the Go shim."""

    def __init__(self, snapshot: Snapshot, max_read_depth: int = 5, max_read_width: int = 100,
                 max_batch: int = 1 << 16, max_wait_us: int = 0, inflight: int = 4, err_detail: bool = False,
                 on_batch=None):
        """on_batch(event dict): called by the library's slot threads after every batch
        (keto_dispatcher_config.on_batch) -- where a Go shim feeds its Prometheus histograms"""
        self._hook = None
        if on_batch is not None:
            def hook(_ctx, ev):
                e = ev.contents
                on_batch({k: getattr(e, k) for k, _ in e._fields_})
            self._hook = _abi.BATCH_HOOK_FN(hook)
        cfg = _abi.DispatcherConfig(_abi.Limits(max_read_depth, max_read_width), max_batch, max_wait_us, inflight,
                                    _abi.F_ERR_DETAIL if err_detail else 0,
                                    self._hook if self._hook else _abi.BATCH_HOOK_FN(), None)
        h = ctypes.c_void_p()
        check(lib().keto_dispatcher_create(snapshot.handle, ctypes.byref(cfg), ctypes.byref(h)))
        self.handle = h
        self.snapshot = snapshot
        _abi.track(self)

    def check(self, queries: np.ndarray):
        q = np.ascontiguousarray(queries, dtype=_abi.QUERY_DT)
        allowed = np.zeros(len(q), dtype=np.uint8)
        err = np.zeros(max(1, len(q)), dtype=np.int32)
        check(lib().keto_dispatcher_check(self.handle, q.ctypes.data, len(q), allowed.ctypes.data, err.ctypes.data))
        return allowed, err[: len(q)]

    def expand(self, roots: np.ndarray, cap: int = 0):
        """ExpandService.Expand coalescing (expand/handler.go:115-152): SUBJSET_DT roots ->
        (nodes TREE_DT, offsets uint64[n+1], err int32[n]), like ExpandEngine.build_trees."""
        r = np.ascontiguousarray(roots, dtype=_abi.SUBJSET_DT)
        n = len(r)
        offs = np.zeros(n + 1, dtype=np.uint64)
        err = np.zeros(max(1, n), dtype=np.int32)
        cap = cap or max(64, 16 * n)
        while True:
            nodes = np.empty(max(1, cap), dtype=_abi.TREE_DT)
            rc = lib().keto_dispatcher_expand(self.handle, r.ctypes.data, n, nodes.ctypes.data, cap, offs.ctypes.data,
                                              err.ctypes.data)
            if rc == _abi.KETO_E_CAPACITY:
                cap = int(offs[n]) + 1
                continue
            check(rc)
            return nodes[: int(offs[n])], offs, err[:n]

    def set_snapshot(self, snapshot: Snapshot):
        check(lib().keto_dispatcher_set_snapshot(self.handle, snapshot.handle))
        self.snapshot = snapshot

    def stats(self) -> dict:
        st = _abi.DispatcherStats()
        check(lib().keto_dispatcher_stats_get(self.handle, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in st._fields_}

    def close(self):
        if getattr(self, "handle", None):
            lib().keto_dispatcher_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
