"""keto_mi355x -- MI355X (gfx950) batched permission Check / Expand for Ory Keto's hot path.

The product is libketo_mi355x.so (C ABI: include/keto_mi355x.h).  This package is
its Python host binding (ctypes), used by the tests and bench.py.
"""
from ._abi import (F_ASYNC, F_COUNT_WORK, F_DEVICE_PTRS, QERR_INTERNAL, QERR_NO_RELATION, QERR_NONE,
                   QERR_NOT_IMPLEMENTED, QUERY16_DT, QUERY_DT, SIGNATURES, SUBJSET_DT, TREE_DT, TUPLE_DT, KetoError,
                   LIB_PATH, lib)
from .engine import (CheckEngine, DeviceBuffer, Dispatcher, PinnedArray, ExpandEngine, TupleStore, Interner, Mapper, Snapshot,
                     Stream, pack_queries16, shard_bytes)

__all__ = ["CheckEngine", "ExpandEngine", "Dispatcher", "PinnedArray", "TupleStore", "Snapshot", "Stream", "DeviceBuffer", "Mapper", "Interner",
           "shard_bytes", "pack_queries16", "lib", "KetoError", "TUPLE_DT", "QUERY_DT", "QUERY16_DT", "SUBJSET_DT", "TREE_DT", "SIGNATURES",
           "LIB_PATH", "F_DEVICE_PTRS", "F_ASYNC", "F_COUNT_WORK", "QERR_NONE", "QERR_NO_RELATION",
           "QERR_INTERNAL", "QERR_NOT_IMPLEMENTED"]
