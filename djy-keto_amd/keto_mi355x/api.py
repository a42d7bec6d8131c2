"""Expand trees -> API form, host side of the shim.

`keto_expand_batch` returns trees of interned ids.  The reference turns each tree into the
API form in two steps:
- `Mapper.ToTree` (internal/relationtuple/uuid_mapping.go:347-399) maps ids to strings;
- then one of two encodings:
  - REST: encoding/json of `ketoapi.Tree` (ketoapi/public_api_definitions.go:217-229);
  - gRPC: `Tree.ToProto` (ketoapi/enc_proto.go:119-133) into `SubjectTree`.

Both run natively in the library (csrc/treefmt.cpp: keto_trees_to_json /
keto_trees_to_proto), one call per batch of trees.  This module binds them.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from ._abi import check, lib


class NameTables:
    """id -> string tables: the Mapper's view of namespaces, relations and keto_uuid_mappings
    (str, or bytes taken as they are)."""

    def __init__(self, namespaces: list, relations: list, uuids: list):
        enc = lambda xs: (ctypes.c_char_p * max(1, len(xs)))(  # noqa: E731
            *[x if isinstance(x, bytes) else x.encode() for x in xs])
        self._ns, self._rel, self._uuid = enc(namespaces), enc(relations), enc(uuids)
        self.c = _abi.NameTables(len(namespaces), self._ns, len(relations), self._rel, len(uuids), self._uuid)


def _format(fn, nodes: np.ndarray, offsets: np.ndarray, names: NameTables):
    nodes = np.ascontiguousarray(nodes, dtype=_abi.TREE_DT)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    outo = np.zeros(n + 1, dtype=np.uint64)
    cap = max(256, 64 * len(nodes))
    while True:
        buf = ctypes.create_string_buffer(cap)
        rc = fn(nodes.ctypes.data, offsets.ctypes.data, n, ctypes.byref(names.c), buf, cap, outo.ctypes.data)
        if rc == _abi.KETO_E_CAPACITY:
            cap = int(outo[n])
            continue
        check(rc)
        raw = buf.raw
        return [raw[int(outo[i]):int(outo[i + 1])] if outo[i + 1] > outo[i] else None for i in range(n)]


def trees_to_json(nodes: np.ndarray, offsets: np.ndarray, names: NameTables) -> list:
    """REST expand bodies: one JSON text per tree (None for a nil tree)."""
    return [None if b is None else b.decode() for b in _format(lib().keto_trees_to_json, nodes, offsets, names)]


def trees_to_proto(nodes: np.ndarray, offsets: np.ndarray, names: NameTables) -> list:
    """gRPC ExpandResponse.tree: serialized SubjectTree per tree (None for a nil tree)."""
    return _format(lib().keto_trees_to_proto, nodes, offsets, names)
