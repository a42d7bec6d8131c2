"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports exactly the
entry points include/keto_mi355x.h declares, its record layouts match the header, and it
fails loudly (no CPU fallback) where no GPU is present."""
import ctypes
import os
import re

import numpy as np
import pytest

import keto_mi355x as km
from keto_mi355x import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "keto_mi355x.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t)\s+(keto_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    fns = header_functions()
    assert "keto_check_batch" in fns and "keto_expand_batch" in fns and "keto_snapshot_build" in fns
    assert sorted(_abi.SIGNATURES) == fns


def test_library_exports_every_declared_symbol():
    lib = km.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.keto_abi_version() == 7


def test_record_layouts_match_header():
    src = open(HEADER).read()
    assert "uint8_t shard_id[16];" in src
    assert km.TUPLE_DT.itemsize == 48 and km.QUERY_DT.itemsize == 32
    assert km.SUBJSET_DT.itemsize == 16 and km.TREE_DT.itemsize == 24
    assert ctypes.sizeof(_abi.Limits) == 8 and ctypes.sizeof(_abi.WorkCounters) == 168


def test_invalid_arguments_are_rejected():
    lib = km.lib()
    assert lib.keto_snapshot_build(None, None, 0, None) == _abi.KETO_E_INVALID
    assert "null" in _abi.last_error()
    assert lib.keto_check_batch(None, None, None, 0, None, None, None, 0) == _abi.KETO_E_INVALID


def _gpu_present():
    n = ctypes.c_int32(0)
    return km.lib().keto_device_count(ctypes.byref(n)) == 0 and n.value > 0


@pytest.mark.skipif(_gpu_present(), reason="GPU present: the failure path is exercised on GPU-less hosts only")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(km.KetoError) as ei:
        km.Stream(0)
    assert ei.value.code == _abi.KETO_E_DEVICE
    cfg = {"g": []}
    t = np.zeros(1, dtype=km.TUPLE_DT)
    with pytest.raises(km.KetoError):
        km.Snapshot(cfg, t, ["g"], ["m"], 2)


def test_exit_teardown_order():
    """At interpreter exit (_abi._shutdown, registered with atexit when the library loads) the
    live handle owners are closed dispatchers first, then partitions, streams, snapshots, stores
    and raw buffers, and keto_shutdown returns the library's cached device blocks -- while the
    HIP runtime is still alive (the round-3 exit SIGSEGV)."""
    km.lib()
    closed = []
    objs = []
    for name in ("PinnedArray", "Snapshot", "Dispatcher", "TupleStore", "Stream", "PartitionedEngine",
                 "DeviceBuffer"):
        meth = "free" if name in ("PinnedArray", "DeviceBuffer") else "close"
        cls = type(name, (), {meth: (lambda self, n=name: closed.append(n))})
        objs.append(_abi.track(cls()))
    _abi._shutdown()
    assert closed == ["Dispatcher", "PartitionedEngine", "Stream", "Snapshot", "TupleStore", "DeviceBuffer",
                      "PinnedArray"]
    assert km.lib().keto_shutdown() == 0  # idempotent, and harmless without a device


def test_process_exit_is_clean():
    """a process that loaded the library exits 0 through the atexit path"""
    import subprocess
    import sys
    code = "import keto_mi355x as km; km.lib(); print('ok')"
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "djy-keto_amd"),
                                                       os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
