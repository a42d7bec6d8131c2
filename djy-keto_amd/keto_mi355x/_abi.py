"""ctypes declarations of include/keto_mi355x.h (the C ABI of libketo_mi355x.so)."""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref

import numpy as np

LIB_NAME = "libketo_mi355x.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# A/B experiments and the CPU kernel-debug harness only (tools/): load another build of
# the same ABI when explicitly unlocked.  Nothing in the product, tests' GPU runs or the
# bench sets these variables.
if os.environ.get("KETO_MI355X_ALLOW_OVERRIDE") == "tools" and os.environ.get("KETO_MI355X_LIB_OVERRIDE"):
    LIB_PATH = os.environ["KETO_MI355X_LIB_OVERRIDE"]

KETO_OK = 0
KETO_E_INVALID, KETO_E_DEVICE, KETO_E_CAPACITY, KETO_E_LIMIT = -1, -2, -3, -4
F_DEVICE_PTRS, F_ASYNC, F_COUNT_WORK, F_ERR_DETAIL, F_PART_DIST = 0x1, 0x2, 0x4, 0x8, 0x10
QERR_NONE, QERR_NO_RELATION, QERR_INTERNAL, QERR_NOT_IMPLEMENTED = 0, 1, 2, 3

TUPLE_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("subj_kind", "<u4"), ("s_obj", "<u4"),
                     ("s_ns", "<u4"), ("s_rel", "<u4"), ("reserved", "<u4"), ("shard_id", "u1", (16,))])
QUERY_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("subj_kind", "<u4"), ("s_obj", "<u4"),
                     ("s_ns", "<u4"), ("s_rel", "<u4"), ("max_depth", "<i4")])
SUBJSET_DT = np.dtype([("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"), ("max_depth", "<i4")])
TREE_DT = np.dtype([("type", "<u4"), ("subj_kind", "<u4"), ("s_obj", "<u4"), ("s_ns", "<u4"), ("s_rel", "<u4"),
                    ("n_children", "<u4")])
assert TUPLE_DT.itemsize == 48 and QUERY_DT.itemsize == 32 and TREE_DT.itemsize == 24
# keto_query16 (ABI 7): {obj, s_obj, ns | rel << 12 | s_rel << 22, s_ns | subj_kind << 12 | depth << 16}
QUERY16_DT = np.dtype([("obj", "<u4"), ("s_obj", "<u4"), ("ns_rel", "<u4"), ("s_ns_depth", "<u4")])
assert QUERY16_DT.itemsize == 16


class SnapshotConfig(ctypes.Structure):
    _fields_ = [("n_namespaces", ctypes.c_uint32), ("namespace_names", ctypes.POINTER(ctypes.c_char_p)),
                ("n_relations", ctypes.c_uint32), ("relation_names", ctypes.POINTER(ctypes.c_char_p)),
                ("n_uuids", ctypes.c_uint32), ("namespaces_json", ctypes.c_char_p),
                ("strict_mode", ctypes.c_int32), ("device", ctypes.c_int32)]


class SnapshotInfo(ctypes.Structure):
    _fields_ = [("n_tuples", ctypes.c_uint64), ("n_nodes", ctypes.c_uint64), ("n_entities", ctypes.c_uint64),
                ("n_set_edges", ctypes.c_uint64), ("n_rev_entries", ctypes.c_uint64),
                ("device_bytes", ctypes.c_uint64), ("build_seconds", ctypes.c_double), ("version", ctypes.c_uint64),
                ("n_reach", ctypes.c_uint64)]


class Placement(ctypes.Structure):
    """keto_placement (ABI 7): block[ns] > 0 puts object obj of namespace ns on rank (obj / block[ns]) % world"""
    _fields_ = [("block", ctypes.c_uint32 * 16)]


class Limits(ctypes.Structure):
    _fields_ = [("max_read_depth", ctypes.c_int32), ("max_read_width", ctypes.c_int32)]


class WorkCounters(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_uint64 * 3), ("edges", ctypes.c_uint64 * 3), ("probes", ctypes.c_uint64 * 3),
                ("out_nodes", ctypes.c_uint64 * 3), ("queries", ctypes.c_uint64 * 3),
                ("wave_steps", ctypes.c_uint64 * 3), ("lane_steps", ctypes.c_uint64 * 3)]


class FrontierStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("batches", "queries", "routed", "goals", "generations",
                                               "max_generations", "async_batches")]


class BatchEvent(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("requests", ctypes.c_uint32), ("queries", ctypes.c_uint64),
                ("wall_ms", ctypes.c_double), ("device_ms", ctypes.c_double), ("rc", ctypes.c_int32)]


BATCH_HOOK_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(BatchEvent))


class DispatcherConfig(ctypes.Structure):
    _fields_ = [("limits", Limits), ("max_batch", ctypes.c_uint32), ("max_wait_us", ctypes.c_uint32),
                ("inflight", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("on_batch", BATCH_HOOK_FN),
                ("hook_ctx", ctypes.c_void_p)]


class DispatcherStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("requests", ctypes.c_uint64), ("queries", ctypes.c_uint64),
                ("max_batch_seen", ctypes.c_uint64), ("wall_ms_sum", ctypes.c_double),
                ("device_ms_sum", ctypes.c_double)]


class PartitionStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("levels", ctypes.c_uint64), ("objects", ctypes.c_uint64),
                ("tuples", ctypes.c_uint64), ("bytes_sent", ctypes.c_uint64), ("closure_s", ctypes.c_double),
                ("build_s", ctypes.c_double), ("run_s", ctypes.c_double), ("rows", ctypes.c_uint64),
                ("edges", ctypes.c_uint64), ("probes", ctypes.c_uint64), ("queries", ctypes.c_uint64),
                ("generations", ctypes.c_uint64), ("goals", ctypes.c_uint64), ("routed", ctypes.c_uint64),
                ("exchange_bytes", ctypes.c_uint64), ("device_s", ctypes.c_double), ("exchange_s", ctypes.c_double)]


class PartitionLevel(ctypes.Structure):
    _fields_ = [("objects", ctypes.c_uint64), ("request_bytes", ctypes.c_uint64), ("tuples", ctypes.c_uint64),
                ("tuple_bytes_sent", ctypes.c_uint64), ("ms", ctypes.c_double)]


class PartitionGeneration(ctypes.Structure):
    _fields_ = [("goals", ctypes.c_uint64), ("record_bytes_out", ctypes.c_uint64), ("records_in", ctypes.c_uint64),
                ("value_bytes_back", ctypes.c_uint64), ("ms", ctypes.c_double)]


# keto_collective callbacks
ABI_VERSION = 7  # include/keto_mi355x.h KETO_ABI_VERSION

ALLTOALL_U64_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64))
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))
ALLREDUCE_MAX_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))
ALLTOALLV_DEV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)


class NameTables(ctypes.Structure):
    _fields_ = [("n_namespaces", ctypes.c_uint32), ("namespace_names", ctypes.POINTER(ctypes.c_char_p)),
                ("n_relations", ctypes.c_uint32), ("relation_names", ctypes.POINTER(ctypes.c_char_p)),
                ("n_uuids", ctypes.c_uint64), ("uuid_strings", ctypes.POINTER(ctypes.c_char_p))]


# symbol -> (restype, argtypes); the header's complete export list
_VP, _U32, _I32, _U64, _SZ = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
SIGNATURES = {
    "keto_abi_version": (ctypes.c_int, []),
    "keto_shutdown": (ctypes.c_int, []),
    "keto_last_error": (_SZ, [ctypes.c_char_p, _SZ]),
    "keto_snapshot_build": (ctypes.c_int, [ctypes.POINTER(SnapshotConfig), _VP, _U64, ctypes.POINTER(_VP)]),
    "keto_snapshot_build_device": (ctypes.c_int, [ctypes.POINTER(SnapshotConfig), _VP, _U64, ctypes.POINTER(_VP)]),
    "keto_snapshot_free": (ctypes.c_int, [_VP]),
    "keto_snapshot_save": (ctypes.c_int, [_VP, ctypes.c_char_p]),
    "keto_snapshot_load": (ctypes.c_int, [ctypes.c_char_p, _I32, ctypes.POINTER(_VP)]),
    "keto_snapshot_info_get": (ctypes.c_int, [_VP, ctypes.POINTER(SnapshotInfo)]),
    "keto_stream_create": (ctypes.c_int, [_I32, ctypes.POINTER(_VP)]),
    "keto_stream_destroy": (ctypes.c_int, [_VP]),
    "keto_stream_sync": (ctypes.c_int, [_VP]),
    "keto_stream_counters": (ctypes.c_int, [_VP, ctypes.POINTER(WorkCounters), _I32]),
    "keto_stream_last_kernel_ms": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double)]),
    "keto_stream_frontier_stats": (ctypes.c_int, [_VP, ctypes.POINTER(FrontierStats), _I32]),
    "keto_host_alloc": (ctypes.c_int, [_U64, ctypes.POINTER(ctypes.c_void_p)]),
    "keto_stream_expand_time": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64), _I32]),
    "keto_host_free": (ctypes.c_int, [_VP]),
    "keto_stream_kernel_time": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64), _I32]),
    "keto_check_batch": (ctypes.c_int, [_VP, _VP, _VP, _U64, ctypes.POINTER(Limits), _VP, _VP, _U32]),
    "keto_check_batch16": (ctypes.c_int, [_VP, _VP, _VP, _U64, ctypes.POINTER(Limits), _VP, _VP, _U32]),
    "keto_pack_query16": (ctypes.c_int, [_VP, _U64, _VP]),
    "keto_expand_batch": (ctypes.c_int, [_VP, _VP, _VP, _U64, ctypes.POINTER(Limits), _VP, _U64, _VP, _VP]),
    "keto_expand_batch_spans": (ctypes.c_int, [_VP, _VP, _VP, _U64, ctypes.POINTER(Limits), _VP, _U64, _VP, _VP, _VP,
                                               ctypes.POINTER(ctypes.c_uint64)]),
    "keto_device_alloc": (ctypes.c_int, [_I32, _U64, ctypes.POINTER(_VP)]),
    "keto_device_free": (ctypes.c_int, [_VP]),
    "keto_memcpy_h2d": (ctypes.c_int, [_VP, _VP, _VP, _U64]),
    "keto_memcpy_d2h": (ctypes.c_int, [_VP, _VP, _VP, _U64]),
    "keto_device_count": (ctypes.c_int, [ctypes.POINTER(_I32)]),
    "keto_store_create": (ctypes.c_int, [_I32, _VP, _U64, _U32, ctypes.POINTER(_VP)]),
    "keto_store_transact": (ctypes.c_int, [_VP, _VP, _U64, _VP, _U64, _U32]),
    "keto_store_snapshot": (ctypes.c_int, [_VP, ctypes.POINTER(SnapshotConfig), ctypes.POINTER(_VP)]),
    "keto_store_snapshot_patch": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(SnapshotConfig), ctypes.POINTER(_VP),
                                                 ctypes.POINTER(_I32)]),
    "keto_store_snapshot_advance": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(_I32)]),
    "keto_store_info": (ctypes.c_int, [_VP, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "keto_store_free": (ctypes.c_int, [_VP]),
    "keto_dispatcher_create": (ctypes.c_int, [_VP, ctypes.POINTER(DispatcherConfig), ctypes.POINTER(_VP)]),
    "keto_dispatcher_destroy": (ctypes.c_int, [_VP]),
    "keto_dispatcher_check": (ctypes.c_int, [_VP, _VP, _U64, _VP, _VP]),
    "keto_dispatcher_expand": (ctypes.c_int, [_VP, _VP, _U64, _VP, _U64, _VP, _VP]),
    "keto_dispatcher_set_snapshot": (ctypes.c_int, [_VP, _VP]),
    "keto_dispatcher_stats_get": (ctypes.c_int, [_VP, ctypes.POINTER(DispatcherStats)]),
    "keto_partition_create": (ctypes.c_int, [ctypes.POINTER(SnapshotConfig), _VP, _U64, _U32, _VP,
                                             ctypes.POINTER(Limits), ctypes.POINTER(_VP)]),
    "keto_partition_create_placed": (ctypes.c_int, [ctypes.POINTER(SnapshotConfig), _VP, _U64, _U32, _VP,
                                                    ctypes.POINTER(Limits), ctypes.POINTER(Placement), ctypes.POINTER(_VP)]),
    "keto_partition_check": (ctypes.c_int, [_VP, _VP, _U64, _VP, _VP, _U32]),
    "keto_partition_check_many": (ctypes.c_int, [_VP, _U32, _VP, _VP, _VP, _VP, _U32]),
    "keto_partition_expand": (ctypes.c_int, [_VP, _VP, _U64, ctypes.POINTER(_U64)]),
    "keto_partition_expand_result": (ctypes.c_int, [_VP, _VP, _U64, _VP, _VP]),
    "keto_partition_stats_get": (ctypes.c_int, [_VP, ctypes.POINTER(PartitionStats)]),
    "keto_partition_levels_get": (ctypes.c_int, [_VP, ctypes.POINTER(PartitionLevel), _U32, ctypes.POINTER(_U32)]),
    "keto_partition_generations_get": (ctypes.c_int, [_VP, ctypes.POINTER(PartitionGeneration), _U32, ctypes.POINTER(_U32)]),
    "keto_partition_free": (ctypes.c_int, [_VP]),
    "keto_trees_to_json": (ctypes.c_int, [_VP, _VP, _U64, ctypes.POINTER(NameTables), _VP, _U64, _VP]),
    "keto_trees_to_proto": (ctypes.c_int, [_VP, _VP, _U64, ctypes.POINTER(NameTables), _VP, _U64, _VP]),
}


class KetoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"keto error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load the HIP engine.  There is no fallback: a missing library is an error."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C djy-keto_amd` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.keto_abi_version() != ABI_VERSION:
            raise RuntimeError("libketo_mi355x ABI version mismatch")
        _lib = L
        if not os.environ.get("KETO_MI355X_NO_TEARDOWN"):  # (tools/exit_probe.py "leak": diagnostics only)
            atexit.register(_shutdown)
    return _lib


# Objects owning library handles (streams, snapshots, ...).  At interpreter exit they are closed
# -- dispatchers before the snapshots they serve, streams before snapshots -- and keto_shutdown
# hands the library's cached device blocks and events back, all while the HIP runtime is still
# fully alive: nothing of the library is left to the runtime's own teardown inside exit().
_live = weakref.WeakSet()
_CLOSE_ORDER = ("Dispatcher", "PartitionedEngine", "Stream", "Snapshot", "TupleStore", "DeviceBuffer", "PinnedArray")


def track(obj):
    _live.add(obj)
    return obj


def _close_rank(obj) -> int:
    name = type(obj).__name__
    return _CLOSE_ORDER.index(name) if name in _CLOSE_ORDER else len(_CLOSE_ORDER)


def _shutdown():
    if _lib is None:
        return
    for obj in sorted(list(_live), key=_close_rank):
        fn = getattr(obj, "close", None) or getattr(obj, "free", None)
        try:
            if fn is not None:
                fn()
        except Exception:  # (exit path: keep closing the rest)
            pass
    _lib.keto_shutdown()


def last_error() -> str:
    buf = ctypes.create_string_buffer(4096)
    lib().keto_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int):
    if rc != KETO_OK:
        raise KetoError(rc, last_error())
    return rc
