"""Fixed cost of one small bucket job through native_terms.lower_many (the single-query
path's ~3.5 jobs per query): the Python wrapper's parts and the native call, min over
repetitions, and the registry blob's size (pflt_lower parses it per job).  GPU-box tool (the
corpus build hashes on the engine).

usage: python tools/lower_overhead_probe.py [reps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import native_terms as NT, terms as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
c = corpus.build(48, 2, seed=2024)
sample = [q for q in c.queries if q.label == "sat"][:96]
st = NT.batch_api()
reg = c.kfm.registry
blob = NT._registry_blob(reg)
print("registry blob words", len(blob), "actors", len(reg.actors), "keccak specs", len(reg.keccak),
      "concrete", sum(len(s.concrete) for s in reg.keccak.values()))
small = min((b for q in sample for b in NT.buckets([x for x in q.constraints if x is not T.TRUE])), key=len)
job = [(list(small), None)]


def best(f):
    m = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        f()
        m = min(m, time.perf_counter() - t)
    return round(m * 1e6, 2)


print("lower_many, one small job:", best(lambda: NT.lower_many(job, reg, True, [0], 1, st)), "us")
# the native call alone, with the wrapper's arrays prepared once
n = 1
roots = np.array([st.export(t) for t in small], dtype=np.uint32)
arr = np.zeros(n, dtype=NT._JOB)
arr["roots"] = roots.ctypes.data
arr["n"] = len(small)
arr["parents"] = 0
arr["flags"] = NT.PROGRAM | NT.HINTS
arr["seed"] = 0
res = (ctypes.c_void_p * n)()


def native():
    st.L.pflt_lower_many(st.h, arr.ctypes.data, n, NT._p32(blob), len(blob), 1, res)
    st.L.pflt_result_free(res[0])


print("pflt_lower_many alone (+ free):", best(native), "us")
empty = np.array([0], dtype=np.uint32)


def native_noreg():
    st.L.pflt_lower_many(st.h, arr.ctypes.data, n, NT._p32(empty), 1, 1, res)
    st.L.pflt_result_free(res[0])


print("... with an empty registry:", best(native_noreg), "us")
print("_registry_blob lookup:", best(lambda: NT._registry_blob(reg)), "us")
