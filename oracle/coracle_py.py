"""ORACLE (test infrastructure): ctypes wrapper of oracle/libcoracle.so (the C restatement).

Used by tests/ as a fast checker and by bench.py's cpu_baseline leg.  Never imported by
mythril_amd/.
"""

import ctypes
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libcoracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(SO)
        u32p, u8p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint8)
        L.co_eval_generated.argtypes = [u32p] * 5 + [ctypes.c_uint32, ctypes.c_uint64,
                                                     ctypes.c_uint32, ctypes.c_uint32, u8p]
        L.co_eval_generated.restype = ctypes.c_int
        L.co_eval_explicit.argtypes = [u32p] * 5 + [ctypes.c_uint32, u32p, ctypes.c_uint32, u8p]
        L.co_eval_explicit.restype = ctypes.c_int
        L.co_gen_values.argtypes = [u32p] * 5 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint32, u32p]
        L.co_gen_values.restype = None
        L.co_keccak256_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p]
        L.co_keccak256_fixed.restype = None
        _lib = L
    return _lib


class Packed:
    """Flat arrays of a mythril_amd.ir.Batch, kept alive for the C calls."""

    def __init__(self, batch):
        def arr(a, cols):
            a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1)
            return a if a.size else np.zeros(cols, dtype=np.uint32)

        self.code = arr(batch.code, 4)
        self.consts = arr(batch.consts, 8)
        self.schema = arr(batch.schema, 4)
        self.parents = arr(batch.parents, 8)
        self.descs = arr(batch.descs, 8)
        self.n = len(batch)

    def ptrs(self):
        p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        return p(self.code), p(self.consts), p(self.schema), p(self.parents), p(self.descs)

    def eval_generated(self, s, gseed, cand0, n):
        out = np.zeros(n, dtype=np.uint8)
        rc = lib().co_eval_generated(*self.ptrs(), s, gseed, cand0, n,
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        assert rc == 0, "coracle: unknown opcode"
        return out.astype(bool)

    def first_sat(self, s, gseed, budget):
        sat = self.eval_generated(s, gseed, 0, budget)
        idx = np.nonzero(sat)[0]
        return int(idx[0]) if idx.size else None


def baseline(programs, budget, seed, target_s):
    """CPU evals/s of the C restatement on all host cores over a bounded sample."""
    from mythril_amd import ir

    P = Packed(ir.Batch(programs))
    cores = os.cpu_count() or 1
    env_threads = os.environ.get("OMP_NUM_THREADS")
    if env_threads:
        cores = int(env_threads)
    chunk = 4096
    t0 = time.perf_counter()
    evals, s = 0, 0
    while time.perf_counter() - t0 < target_s:
        P.eval_generated(s % P.n, seed, (s // P.n) * chunk, chunk)
        evals += chunk
        s += 1
    dt = time.perf_counter() - t0
    return {"value": evals / dt, "unit": "evals/s", "cores": cores, "kind": "port",
            "sample": f"C restatement (oracle/coracle.c, OpenMP) over {s} sets x {chunk} "
                      f"candidates of the same workload, {dt:.1f} s"}


def keccak256_fixed(data: np.ndarray, length: int, n: int) -> np.ndarray:
    """Keccak-256 of n fixed-length messages (uint8 array, row-major) -> (n, 32) uint8."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert data.size >= length * n
    out = np.zeros((n, 32), dtype=np.uint8)
    lib().co_keccak256_fixed(data.ctypes.data, length, n, out.ctypes.data)
    return out


def keccak_baseline(length, target_s):
    """CPU hashes/s of the C Keccak restatement on all host cores (bounded sample)."""
    cores = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    chunk = 1 << 16
    data = np.random.default_rng(1).integers(0, 256, size=chunk * length, dtype=np.uint8)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < target_s:
        keccak256_fixed(data, length, chunk)
        done += chunk
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "hashes/s", "cores": cores, "kind": "port",
            "sample": f"C Keccak-256 restatement (oracle/coracle.c, OpenMP), {done} x {length}-byte "
                      f"messages, {dt:.1f} s"}
