"""pfl_hints (the native hint solver, csrc/pf_seed.cpp) timed alone on dumped DAGs
(tools/dump_hint_dags.py -> tools/data/hint_dags_r06.npz: the largest buckets of the
single-query sample's slowest queries): min over repetitions per DAG, and a digest of the hint
values so two builds can be checked for identical decisions.  Host-only tool.

usage: python tools/hint_bench.py [libpflower.so] [reps]"""
import ctypes
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "mythril_amd", "libpflower.so")
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
L = ctypes.CDLL(lib)
P, Z = ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t
L.pfl_hints.argtypes = [P, Z, P, Z, P, Z, P, Z, P, P, ctypes.POINTER(ctypes.c_int)]
d = np.load(os.path.join(ROOT, "tools", "data", "hint_dags_r06.npz"))
qs = sorted({k.split("_")[0] for k in d.files})
total = 0.0
for q in qs:
    nn, npool, nr, nv = (int(x) for x in d[q + "_meta"])
    a = [np.ascontiguousarray(d[q + s]) for s in ("_nodes", "_pool", "_roots", "_widths", "_soft")]
    out = np.zeros((max(nv, 1), 8), dtype=np.uint32)
    ns = ctypes.c_int()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        rc = L.pfl_hints(*(x.ctypes.data_as(P) if isinstance(x, np.ndarray) else x for x in
                           (a[0], nn, a[1], npool, a[2], nr, a[3], nv, a[4], out)), ctypes.byref(ns))
        best = min(best, time.perf_counter() - t)
    assert rc == 0
    total += best
    print(f"{q}: {nn:5d} nodes {nv:4d} vars  {best * 1e6:8.1f} us  n_sat {ns.value}  "
          f"digest {hashlib.sha256(out.tobytes()).hexdigest()[:12]}")
print(f"total {total * 1e6:.1f} us")
