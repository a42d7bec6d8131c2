"""Partitioned graphs: BASELINE config 5 (second half) over the C ABI.

A graph too large to replicate is spread over the ranks of a job by object: every tuple of
`(ns, obj)` lives on rank `keto_object_owner(ns, obj, world)` (include/keto_mi355x.h).  Per
batch the library (csrc/partition.hip, `keto_partition_*`) gathers the closure of the batch's
objects from their owners -- one all-to-all pair per depth level, driven by device kernels
(hash-set dedup, counting-scatter routing, binary-search gathers) -- builds it into a device
snapshot and runs the unmodified kernels on it; see that file for why the result equals the
whole graph's.  The collective is the caller's: `collective` is any object with

    rank, world
    alltoall_u64(send: np.ndarray[world] uint64) -> np.ndarray[world] uint64
    alltoallv(send: np.ndarray uint8, send_bytes: list, recv: np.ndarray uint8, recv_bytes: list) -> None
    allreduce_max_u64(v: int) -> int

and optionally, to move the exchange's bytes device to device (keto_collective.alltoallv_device),

    alltoallv_device(send_ptr: int, send_bytes: list, recv_ptr: int, recv_bytes: list, stream: int) -> None

(tests/torch_collective.py wraps torch.distributed: gloo in the tests, RCCL in bench.py; a Go
host wraps its own communicator).  No collective = one rank.  This module imports no torch.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from ._abi import check, lib

_MULT = 0x9E3779B97F4A7C15


OWNER_ALL = 0xFFFFFFFF  # KETO_OWNER_ALL: a replicated namespace's objects (placement block PLACE_ALL)
PLACE_ALL = 0xFFFFFFFF


def object_owner(ns: np.ndarray, obj: np.ndarray, nparts: int, placement=None) -> np.ndarray:
    """keto_object_owner (include/keto_mi355x.h) over numpy arrays; with placement (16 block
    sizes per namespace, keto_placement) keto_object_owner_placed: OWNER_ALL for a replicated
    namespace (every rank holds its tuples)."""
    ns, obj = np.asarray(ns).astype(np.uint64), np.asarray(obj).astype(np.uint64)
    k = (ns << np.uint64(32)) | obj
    with np.errstate(over="ignore"):
        h = k * np.uint64(_MULT)
    own = ((h >> np.uint64(32)) % np.uint64(nparts)).astype(np.uint32)
    if placement is not None:
        blk = np.zeros(2 ** 16, np.uint64)
        blk[:16] = np.asarray(placement, dtype=np.uint64)[:16]
        b = blk[np.minimum(ns, 2 ** 16 - 1).astype(np.int64)]
        repl = b == PLACE_ALL
        placed = (b > 0) & ~repl
        own[placed] = ((obj[placed] // b[placed]) % np.uint64(nparts)).astype(np.uint32)
        own[repl] = OWNER_ALL
    return own


class _CCollective(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("alltoall_u64", _abi.ALLTOALL_U64_FN), ("alltoallv", _abi.ALLTOALLV_FN),
                ("allreduce_max_u64", _abi.ALLREDUCE_MAX_FN), ("alltoallv_device", _abi.ALLTOALLV_DEV_FN)]


def _c_collective(coll):
    """ctypes callbacks over a Python collective object (kept alive by the caller)."""
    W = int(coll.world)

    def a2a(_ctx, send, recv):
        try:
            s = np.ctypeslib.as_array(send, shape=(W,)).copy()
            np.ctypeslib.as_array(recv, shape=(W,))[:] = coll.alltoall_u64(s)
            return 0
        except Exception:  # surfaced to the library as a failed collective
            return -1

    def a2av(_ctx, send, send_bytes, recv, recv_bytes):
        try:
            sb = [int(x) for x in np.ctypeslib.as_array(send_bytes, shape=(W,))]
            rb = [int(x) for x in np.ctypeslib.as_array(recv_bytes, shape=(W,))]
            s = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, sum(sb))).from_address(send or 0)) if sum(sb) \
                else np.zeros(0, np.uint8)
            r = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, sum(rb))).from_address(recv or 0)) if sum(rb) \
                else np.zeros(0, np.uint8)
            coll.alltoallv(s[:sum(sb)], sb, r[:sum(rb)], rb)
            return 0
        except Exception:
            return -1

    def amax(_ctx, v):
        try:
            v[0] = int(coll.allreduce_max_u64(int(v[0])))
            return 0
        except Exception:
            return -1

    def a2av_dev(_ctx, send, send_bytes, recv, recv_bytes, stream):
        try:
            sb = [int(x) for x in np.ctypeslib.as_array(send_bytes, shape=(W,))]
            rb = [int(x) for x in np.ctypeslib.as_array(recv_bytes, shape=(W,))]
            coll.alltoallv_device(int(send or 0), sb, int(recv or 0), rb, int(stream or 0))
            return 0
        except Exception:
            return -1

    use_dev = callable(getattr(coll, "alltoallv_device", None)) and getattr(coll, "device_buffers", True)
    dev = _abi.ALLTOALLV_DEV_FN(a2av_dev) if use_dev else _abi.ALLTOALLV_DEV_FN()
    fns = (_abi.ALLTOALL_U64_FN(a2a), _abi.ALLTOALLV_FN(a2av), _abi.ALLREDUCE_MAX_FN(amax), dev)
    c = _CCollective(None, int(coll.rank), W, *fns)
    return c, fns


class PartitionedEngine:
    """check.Engine / expand.Engine over a graph partitioned by object across the ranks of a
    job: one rank per GPU, `part_tuples` = this rank's partition (keto_object_owner == rank),
    host TUPLE_DT records or device_tuples=(pointer, count).  Collective: every rank calls
    check_batch / expand_batch for each batch together."""

    def __init__(self, namespaces, ns_names, rel_names, n_uuids: int, part_tuples=None, *, strict: bool = False,
                 device: int = 0, max_read_depth: int = 5, max_read_width: int = 100, collective=None,
                 device_tuples: tuple | None = None, distributed: bool = False, placement=None):
        import json
        if isinstance(namespaces, dict):
            namespaces = json.dumps(namespaces)
        self._ns = (ctypes.c_char_p * max(1, len(ns_names)))(*[n.encode() for n in ns_names])
        self._rel = (ctypes.c_char_p * max(1, len(rel_names)))(*[r.encode() for r in rel_names])
        self._json = namespaces.encode()
        cfg = _abi.SnapshotConfig(len(ns_names), self._ns, len(rel_names), self._rel, n_uuids, self._json,
                                  int(strict), device)
        self.max_read_depth, self.max_read_width = max_read_depth, max_read_width
        lim = _abi.Limits(max_read_depth, max_read_width)
        self._coll = None
        # distributed=True (KETO_F_PART_DIST): the distributed frontier even at world 1, every
        # exchange going to this rank through the collective
        if collective is not None and (int(collective.world) > 1 or distributed):
            self._coll = _c_collective(collective)
        flags = _abi.F_PART_DIST if distributed else 0
        # placement: 16 block sizes per namespace (keto_placement; None: keto_object_owner)
        pl = None
        if placement is not None:
            self._pl = _abi.Placement((ctypes.c_uint32 * 16)(*[int(b) for b in list(placement)[:16]]))
            pl = ctypes.byref(self._pl)
        h = ctypes.c_void_p()
        if device_tuples is not None:
            ptr, count = device_tuples
            check(lib().keto_partition_create_placed(ctypes.byref(cfg), ptr, count, _abi.F_DEVICE_PTRS | flags,
                                                     ctypes.byref(self._coll[0]) if self._coll else None, ctypes.byref(lim),
                                                     pl, ctypes.byref(h)))
        else:
            t = np.ascontiguousarray(part_tuples, dtype=_abi.TUPLE_DT)
            check(lib().keto_partition_create_placed(ctypes.byref(cfg), t.ctypes.data if len(t) else None, len(t), flags,
                                                     ctypes.byref(self._coll[0]) if self._coll else None, ctypes.byref(lim),
                                                     pl, ctypes.byref(h)))
        self.handle = h
        self.last = {}
        _abi.track(self)

    def levels(self) -> int:
        return self.max_read_depth + 1

    def _stats(self):
        st = _abi.PartitionStats()
        check(lib().keto_partition_stats_get(self.handle, ctypes.byref(st)))
        self.last = {k: getattr(st, k) for k, _ in st._fields_}

    def level_stats(self) -> list:
        """the last batch's closure exchange level by level (keto_partition_levels_get)"""
        n = ctypes.c_uint32()
        check(lib().keto_partition_levels_get(self.handle, None, 0, ctypes.byref(n)))
        arr = (_abi.PartitionLevel * max(1, n.value))()
        check(lib().keto_partition_levels_get(self.handle, arr, n.value, ctypes.byref(n)))
        return [{k: getattr(arr[i], k) for k, _ in _abi.PartitionLevel._fields_} for i in range(n.value)]

    def generation_stats(self) -> list:
        """the last distributed-frontier batch generation by generation (keto_partition_generations_get):
        goals, record_bytes_out, records_in, value_bytes_back, ms"""
        n = ctypes.c_uint32()
        check(lib().keto_partition_generations_get(self.handle, None, 0, ctypes.byref(n)))
        arr = (_abi.PartitionGeneration * max(1, n.value))()
        check(lib().keto_partition_generations_get(self.handle, arr, n.value, ctypes.byref(n)))
        return [{k: getattr(arr[i], k) for k, _ in _abi.PartitionGeneration._fields_} for i in range(n.value)]

    def check_batch(self, queries: np.ndarray, count_work: bool = False):
        """queries: QUERY_DT (this rank's) -> (allowed u8[n], err i32[n])"""
        q = np.ascontiguousarray(queries, dtype=_abi.QUERY_DT)
        allowed = np.zeros(len(q), np.uint8)
        err = np.zeros(max(1, len(q)), np.int32)
        check(lib().keto_partition_check(self.handle, q.ctypes.data if len(q) else None, len(q), allowed.ctypes.data,
                                         err.ctypes.data, _abi.F_COUNT_WORK if count_work else 0))
        self._stats()
        if count_work:  # the check kernels' counters, keto_work_counters-shaped (tier 0 only)
            self.last_work = {k: [self.last[k], 0, 0] for k in ("rows", "edges", "probes", "queries")}
        return allowed, err[:len(q)]

    def check_batches(self, batches: list, count_work: bool = False, outs: list | None = None):
        """several batches in order, pipelined (keto_partition_check_many: batch k+1's closure
        runs while batch k is built and checked) -> [(allowed, err)] per batch.  outs: optional
        [(allowed u8[n], err i32[n])] to write into (e.g. pinned arrays, keto_host_alloc: the
        one-rank path's copies then run as straight DMA, as keto_check_batch's do)."""
        qs = [np.ascontiguousarray(b, dtype=_abi.QUERY_DT) for b in batches]
        if outs is None:
            outs = [(np.zeros(len(q), np.uint8), np.zeros(max(1, len(q)), np.int32)) for q in qs]
        k = len(qs)
        P = ctypes.c_void_p * max(1, k)
        qp = P(*[q.ctypes.data if len(q) else None for q in qs])
        ap = P(*[a.ctypes.data for a, _ in outs])
        ep = P(*[e.ctypes.data for _, e in outs])
        ns = (ctypes.c_uint64 * max(1, k))(*[len(q) for q in qs])
        check(lib().keto_partition_check_many(self.handle, k, qp, ns, ap, ep, _abi.F_COUNT_WORK if count_work else 0))
        self._stats()
        return [(a, e[:len(q)]) for (a, e), q in zip(outs, qs)]

    def expand_batch(self, roots: np.ndarray):
        """roots: SUBJSET_DT (this rank's) -> (nodes TREE_DT, offsets u64[n+1], err i32[n])"""
        r = np.ascontiguousarray(roots, dtype=_abi.SUBJSET_DT)
        need = ctypes.c_uint64()
        check(lib().keto_partition_expand(self.handle, r.ctypes.data if len(r) else None, len(r), ctypes.byref(need)))
        nodes = np.empty(max(1, need.value), dtype=_abi.TREE_DT)
        offs = np.zeros(len(r) + 1, np.uint64)
        err = np.zeros(max(1, len(r)), np.int32)
        check(lib().keto_partition_expand_result(self.handle, nodes.ctypes.data, need.value, offs.ctypes.data,
                                                 err.ctypes.data))
        self._stats()
        return nodes[:need.value], offs, err[:len(r)]

    def close(self):
        if getattr(self, "handle", None):
            lib().keto_partition_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
