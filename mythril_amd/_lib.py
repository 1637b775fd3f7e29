"""ctypes binding of libpathfeas.so (include/pathfeas.h).

The library is built in-tree by ``mythril_amd.build.build_library()`` (or
``__graft_entry__.build()``).  There is no CPU fallback: if the shared object or a GPU is
missing, every call raises :class:`PathFeasError` — the product path never silently
answers on the host.
"""

from __future__ import annotations

import ctypes
import os
import sys
import threading
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpathfeas.so")


class PathFeasError(RuntimeError):
    pass


class pf_stats(ctypes.Structure):
    _fields_ = [
        ("evals_full", ctypes.c_uint64),
        ("cands_decided", ctypes.c_uint64),
        ("ops", ctypes.c_uint64),
        ("n_sat", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_float),
        ("timed_out", ctypes.c_uint32),
    ]


_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t

# name -> (restype, argtypes); kept in sync with include/pathfeas.h (tests/test_abi.py)
SIGNATURES = {
    "pf_init": (ctypes.c_int, [ctypes.c_uint64]),
    "pf_init_contexts": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32), _sz, ctypes.POINTER(ctypes.c_int32)]),
    "pf_shutdown": (ctypes.c_int, []),
    "pf_last_error": (ctypes.c_char_p, []),
    "pf_version": (ctypes.c_int, []),
    "pf_device_count": (ctypes.c_int, []),
    "pf_batch_create": (ctypes.c_int, [_u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p,
                                       _sz, _u64p]),
    "pf_batch_create_on": (ctypes.c_int, [ctypes.c_int, _u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p,
                                          _sz, _u32p, _sz, _u64p]),
    "pf_batch_free": (ctypes.c_int, [ctypes.c_uint64]),
    "pf_check_batch": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, _u32p, _u8p,
                                      ctypes.POINTER(pf_stats)]),
    "pf_check_batches": (ctypes.c_int, [_u64p, _sz, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_uint32, _u32p,
                                        ctypes.POINTER(pf_stats)]),
    "pf_check_batch_dev": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.POINTER(pf_stats), ctypes.c_void_p]),
    "pf_materialize": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, _u32p, _u32p, _sz,
                                      _u32p]),
    "pf_eval_assignments": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, _u32p,
                                           ctypes.c_uint32, _u8p]),
    "pf_eval_program": (ctypes.c_int, [ctypes.c_int, _u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p,
                                       ctypes.c_uint32, _u8p]),
    "pf_eval_programs": (ctypes.c_int, [ctypes.c_int, _u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p,
                                        ctypes.c_uint32, _u8p]),
    "pf_eval_assignments_dev": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "pf_device_program": (ctypes.c_int, [_u32p, _sz, _u32p, _sz, _u32p, _sz, _u32p, ctypes.POINTER(_sz), _u32p]),
    "pf_keccak256_batch": (ctypes.c_int, [_u8p, _u64p, _sz, _u8p]),
    "pf_keccak256_fixed_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, _sz,
                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                              ctypes.c_void_p]),
}

_lib = None
_lib_lock = threading.Lock()
_initialised: set = set()
# context ids per device tuple handed to pf_init_contexts: an engine built again over the same
# tuple reuses them instead of adding streams, events and a device pool per build
_contexts: dict = {}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libpathfeas.so and bind every C-ABI symbol (no device work)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 /
        # libhsa-runtime64.so.1 (same SONAMEs as /opt/rocm's).  Importing torch first makes
        # the dynamic loader bind this library to the already-loaded copies, so torch
        # (device memory, streams, RCCL) and the engine share one runtime and one device
        # context.  Loading ours first would map a second runtime and torch's device init
        # then fails ("No HIP GPUs are available").  A process that never uses torch — a
        # Mythril analysis through integration.install(), which sets PF_TORCH=0 — loads the
        # engine on /opt/rocm's runtime alone and pays neither torch's import (~1.5 s) nor
        # its memory.
        if os.environ.get("PF_TORCH", "1") != "0" or "torch" in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(path):
            raise PathFeasError(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def lib() -> ctypes.CDLL:
    return load_library()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().pf_last_error().decode(errors="replace")
        raise PathFeasError(f"{what} failed ({rc}): {msg}")


def init(devices=0) -> None:
    """Initialise the engine's GPUs: one index (one process per GPU) or several (one process
    driving a node: pf_init's device mask)."""
    devs = [devices] if isinstance(devices, int) else list(devices)
    L = lib()
    if set(devs) <= _initialised:
        return
    n = L.pf_device_count()
    if n <= 0:
        raise PathFeasError("no HIP device visible: the MI355X path-feasibility engine has no CPU fallback")
    mask = 0
    for d in devs:
        if not 0 <= d < min(n, 64):
            raise PathFeasError(f"device {d} out of range ({n} visible)")
        mask |= 1 << d
    check(L.pf_init(mask), f"pf_init({devs})")
    _initialised.update(devs)


def init_contexts(devices) -> list:
    """One execution context per entry of ``devices`` (repeats allowed: two contexts on one
    GPU, each with its own stream — pf_init_contexts); returns their ids, which stand in for
    device indices wherever the engine names a device."""
    devs = [int(d) for d in devices]
    L = lib()
    key = tuple(devs)
    if key in _contexts:
        return list(_contexts[key])
    n = L.pf_device_count()
    if n <= 0:
        raise PathFeasError("no HIP device visible: the MI355X path-feasibility engine has no CPU fallback")
    arr = (ctypes.c_int32 * len(devs))(*devs)
    out = (ctypes.c_int32 * len(devs))()
    check(L.pf_init_contexts(arr, len(devs), out), f"pf_init_contexts({devs})")
    _contexts[key] = tuple(out)
    return list(out)


# A one-element ctypes array over the numpy buffer (from_buffer: C-contiguous and writable, or
# it raises) passes the buffer's address as T* for about a third of ndarray.ctypes.data_as's
# cost (numpy builds its _ctypes helper per call); read-only and empty arrays take data_as.
_U32_1, _U8_1, _U64_1 = ctypes.c_uint32 * 1, ctypes.c_uint8 * 1, ctypes.c_uint64 * 1


def _ptr(a: np.ndarray, one, ptype):
    try:
        return one.from_buffer(a)
    except (TypeError, ValueError):
        assert a.flags.c_contiguous
        return a.ctypes.data_as(ptype)


def ptr_u32(a: np.ndarray):
    assert a.dtype == np.uint32
    return _ptr(a, _U32_1, _u32p)


def ptr_u8(a: np.ndarray):
    assert a.dtype == np.uint8
    return _ptr(a, _U8_1, _u8p)


def ptr_u64(a: np.ndarray):
    assert a.dtype == np.uint64
    return _ptr(a, _U64_1, _u64p)
