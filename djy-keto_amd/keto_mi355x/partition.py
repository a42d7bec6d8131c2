"""Partitioned graphs: BASELINE config 5 (second half).

A graph too large to replicate is spread over the ranks of a job by object: every tuple of
`(ns, obj)` lives on rank `keto_object_owner(ns, obj, world)` (include/keto_mi355x.h).  All
relation slots of an object are therefore on one rank -- its direct rows, the rows its
computed usersets reach and its tuple-to-userset (`parents`) row.  Crossing to another
object only ever happens along a subject-set edge.

How a batch runs (each rank checks its own queries):

1. **Closure exchange.**  The reference reads rows only of objects reachable from the
   query's object along subject-set edges, and only up to the depth ledger
   (`check/engine.go:214-249` returns before reading anything at rest depth <= 0; the
   found-lookahead of `traverser.go:73-80` reads one level further).  So `max_depth + 1`
   levels of a level-synchronous object BFS collect every tuple any query of the batch can
   read.  Each level is two RCCL all-to-alls over xGMI: object requests go to their owners,
   and the owners' tuples for them come back.  Objects already fetched are not asked for
   again.
2. **Local snapshot.**  The batch's closure is built into an ordinary device snapshot
   (`keto_snapshot_build_device`, the same HIP builder as the replicated path).
3. **Unmodified kernels.**  The Check / Expand kernels run on it.

The closure holds every tuple of every object the reference engine could read for these
queries, in the same `shard_id` order.  The kernels therefore take exactly the decisions
(and build exactly the trees) they would take on the whole graph.  Exactness (H0-H6,
SURVEY.md 8.0) comes for free, with no distributed version of the sequential DFS.
`tests/test_partition.py` checks this against the oracle over the whole graph, on two gloo
ranks.

The exchange uses torch.distributed (RCCL on GPUs, gloo in the CPU tests) and torch tensor
ops for the request routing.  That is plumbing; the data path is the HIP builder and
kernels.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist

from . import _abi
from .engine import CheckEngine, DeviceBuffer, ExpandEngine, Snapshot, Stream

_MULT = 0x9E3779B97F4A7C15
_MULT_I64 = _MULT - (1 << 64)   # the same bits as a signed 64-bit multiplier
W = _abi.TUPLE_DT.itemsize // 4  # int32 words per keto_tuple record
F_NS, F_OBJ, F_KIND, F_SOBJ, F_SNS = 0, 1, 3, 4, 5


def object_owner(ns: np.ndarray, obj: np.ndarray, nparts: int) -> np.ndarray:
    """keto_object_owner (include/keto_mi355x.h) over numpy arrays."""
    k = (np.asarray(ns).astype(np.uint64) << np.uint64(32)) | np.asarray(obj).astype(np.uint64)
    with np.errstate(over="ignore"):
        h = k * np.uint64(_MULT)
    return ((h >> np.uint64(32)) % np.uint64(nparts)).astype(np.uint32)


def _keys(ns: torch.Tensor, obj: torch.Tensor) -> torch.Tensor:
    """object key (ns << 32 | obj) from int32 columns holding u32 bit patterns"""
    return ((ns.to(torch.int64) & 0xFFFFFFFF) << 32) | (obj.to(torch.int64) & 0xFFFFFFFF)


def _owner(keys: torch.Tensor, nparts: int) -> torch.Tensor:
    return (((keys * _MULT_I64) >> 32) & 0xFFFFFFFF) % nparts


def _as_rows(tuples, device) -> torch.Tensor:
    if isinstance(tuples, torch.Tensor):
        return tuples.view(torch.int32).reshape(-1, W).to(device)
    a = np.ascontiguousarray(tuples, dtype=_abi.TUPLE_DT)
    return torch.from_numpy(a.view(np.int32).reshape(-1, W)).to(device)


class ObjectStore:
    """One rank's partition: its tuple records grouped by object key."""

    def __init__(self, tuples, device):
        t = _as_rows(tuples, device)
        keys, perm = torch.sort(_keys(t[:, F_NS], t[:, F_OBJ]), stable=True)
        self.tuples = t[perm]
        del t, perm
        self.keys, self.count = torch.unique_consecutive(keys, return_counts=True)
        self.begin = torch.cumsum(self.count, 0) - self.count
        self.device = torch.device(device)

    def __len__(self):
        return int(self.tuples.shape[0])

    def rows_of(self, req: torch.Tensor):
        """every tuple of each requested object, in request order; and the count per object"""
        if len(self.keys) == 0 or len(req) == 0:
            return self.tuples[:0], torch.zeros(len(req), dtype=torch.int64, device=self.device)
        idx = torch.searchsorted(self.keys, req).clamp_(max=len(self.keys) - 1)
        cnt = torch.where(self.keys[idx] == req, self.count[idx], 0)
        beg = self.begin[idx]
        total = int(cnt.sum())
        rep = torch.repeat_interleave(torch.arange(len(req), device=self.device), cnt)
        start = torch.cumsum(cnt, 0) - cnt
        pos = beg[rep] + (torch.arange(total, device=self.device) - start[rep])
        return self.tuples[pos], cnt


class _Comm:
    """all-to-all with variable splits over the job's process group (or none)."""

    def __init__(self, group=None):
        self.group = group
        self.on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        self.dev = "cuda" if self.on and dist.get_backend(group) == "nccl" else "cpu"
        self.bytes_sent = 0

    def a2a(self, x: torch.Tensor, send_counts: torch.Tensor):
        """x: rows grouped by destination rank, send_counts[r] rows for rank r.  Returns the
        rows received (grouped by source rank) and the count from each source."""
        if self.world == 1:
            return x, send_counts
        sc = send_counts.to(self.dev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        sl, rl = sc.tolist(), rc.tolist()
        xin = x.to(self.dev).contiguous()
        out = torch.empty((sum(rl),) + tuple(x.shape[1:]), dtype=x.dtype, device=self.dev)
        dist.all_to_all_single(out, xin, rl, sl, group=self.group)
        self.bytes_sent += (sum(sl) - sl[self.rank]) * xin[:1].numel() * xin.element_size()
        return out.to(x.device), rc.to(x.device)

    def any_rank(self, n: int) -> bool:
        if self.world == 1:
            return n > 0
        t = torch.tensor([n], dtype=torch.int64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item()) > 0


def closure(store: ObjectStore, comm: _Comm, root_keys: torch.Tensor, levels: int):
    """Every tuple of every object within `levels` subject-set hops of the roots, gathered from
    the objects' owners (level-synchronous; collective: all ranks call it together).
    Returns (rows int32[n, W] on the store's device, stats)."""
    dev = store.device
    seen = torch.empty(0, dtype=torch.int64, device=dev)
    front = torch.unique(root_keys.to(dev))
    parts, st = [], {"levels": 0, "objects": 0, "tuples": 0}
    for _ in range(levels):
        if len(seen) and len(front):
            front = front[~torch.isin(front, seen)]
        if not comm.any_rank(len(front)):
            break
        st["levels"] += 1
        st["objects"] += len(front)
        seen = torch.sort(torch.cat([seen, front]))[0]
        dest = _owner(front, comm.world)
        order = torch.argsort(dest, stable=True)
        asked, asked_counts = comm.a2a(front[order], torch.bincount(dest, minlength=comm.world))
        rows, cnt = store.rows_of(asked)  # this rank's tuples for the objects asked of it
        src = torch.repeat_interleave(torch.arange(comm.world, device=dev), asked_counts)
        back = torch.zeros(comm.world, dtype=torch.int64, device=dev).index_add_(0, src, cnt)
        got, _ = comm.a2a(rows, back)
        parts.append(got)
        ss = got[got[:, F_KIND] == 1]
        front = torch.unique(_keys(ss[:, F_SNS], ss[:, F_SOBJ]))
    out = torch.cat(parts) if parts else store.tuples[:0]
    st["tuples"] = int(out.shape[0])
    return out, st


class PartitionedEngine:
    """check.Engine / expand.Engine over a graph partitioned by object across the ranks of a
    job: one rank per GPU, `part_tuples` = this rank's partition (keto_object_owner == rank).
    Collective: every rank calls check_batch / expand_batch for each batch together."""

    def __init__(self, namespaces, ns_names, rel_names, n_uuids: int, part_tuples, *, strict: bool = False,
                 device: int = 0, max_read_depth: int = 5, max_read_width: int = 100, group=None,
                 store_device: str | None = None):
        self.namespaces, self.ns_names, self.rel_names = namespaces, list(ns_names), list(rel_names)
        self.n_uuids, self.strict, self.device = n_uuids, strict, device
        self.max_read_depth, self.max_read_width = max_read_depth, max_read_width
        self.comm = _Comm(group)
        # the exchange runs where the process group's tensors live: on the GPU under RCCL, on
        # the host under gloo (and for a single rank), where the closure is uploaded through
        # the library's own allocator
        if store_device is None:
            store_device = f"cuda:{device}" if self.comm.dev == "cuda" else "cpu"
        self.store = ObjectStore(part_tuples, store_device)
        self.stream = None
        self.last = {}

    def levels(self) -> int:
        # rows are read at rest depth >= 1 (max_read_depth - 1 hops); the found-lookahead
        # probes one level beyond a row it expands
        return self.max_read_depth + 1

    def closure_tuples(self, ns: np.ndarray, obj: np.ndarray):
        keys = _keys(torch.from_numpy(np.ascontiguousarray(ns, np.uint32).view(np.int32)),
                     torch.from_numpy(np.ascontiguousarray(obj, np.uint32).view(np.int32)))
        return closure(self.store, self.comm, keys, self.levels())

    def _snapshot(self, rows: torch.Tensor) -> Snapshot:
        n = int(rows.shape[0])
        if rows.is_cuda:
            rows = rows.contiguous()
            torch.cuda.synchronize(rows.device)  # the builder reads them from its own stream
            return Snapshot(self.namespaces, None, self.ns_names, self.rel_names, self.n_uuids, strict=self.strict,
                            device=self.device, device_tuples=(rows.data_ptr(), n))
        host = np.ascontiguousarray(rows.numpy()).view(_abi.TUPLE_DT).reshape(-1)
        buf = DeviceBuffer(self.device, max(1, host.nbytes))
        try:
            if n:
                buf.upload(self._stream(), host)
            return Snapshot(self.namespaces, None, self.ns_names, self.rel_names, self.n_uuids, strict=self.strict,
                            device=self.device, device_tuples=(buf.ptr, n))
        finally:
            buf.free()  # the build has finished reading the records

    def _stream(self) -> Stream:
        if self.stream is None:
            self.stream = Stream(self.device)
        return self.stream

    def check_batch(self, queries: np.ndarray):
        """queries: QUERY_DT (this rank's) -> (allowed u8[n], err i32[n])"""
        q = np.ascontiguousarray(queries, dtype=_abi.QUERY_DT)
        t0 = time.perf_counter()
        rows, st = self.closure_tuples(q["ns"], q["obj"])
        t1 = time.perf_counter()
        snap = self._snapshot(rows)
        t2 = time.perf_counter()
        try:
            eng = CheckEngine(snap, self._stream(), self.max_read_depth, self.max_read_width)
            allowed, err = eng.check_batch(q)
        finally:
            snap.close()
        t3 = time.perf_counter()
        self.last = dict(st, closure_s=t1 - t0, build_s=t2 - t1, check_s=t3 - t2)
        return allowed, err

    def expand_batch(self, roots: np.ndarray):
        """roots: SUBJSET_DT (this rank's) -> (nodes TREE_DT, offsets u64[n+1], err i32[n])"""
        r = np.ascontiguousarray(roots, dtype=_abi.SUBJSET_DT)
        rows, st = self.closure_tuples(r["ns"], r["obj"])
        snap = self._snapshot(rows)
        try:
            out = ExpandEngine(snap, self._stream(), self.max_read_depth).build_trees(r)
        finally:
            snap.close()
        self.last = st
        return out

    def close(self):
        if self.stream is not None:
            self.stream.close()
            self.stream = None
