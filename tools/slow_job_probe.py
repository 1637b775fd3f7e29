"""Where the cold pass's one slow bucket (tools/job_time_probe.py: job 7 of the corpus, three
conjuncts over an actor, a call value and a balance read, ~80 ms the first time, ~1 ms after)
spends its first lowering: the native pflt_lower_many call alone vs lower_many's Python
wrapping, lowered first in a fresh process.  GPU-box tool.

usage: python tools/slow_job_probe.py [job index]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import native_terms as NT, terms as T  # noqa: E402

idx = int(sys.argv[1]) if len(sys.argv) > 1 else 7
c = corpus.build(48, 2, seed=2024)
st = NT.batch_api()
jobs, seen = [], set()
for q in c.queries:
    for b in NT.buckets([x for x in q.constraints if x is not T.TRUE]) or []:
        k = tuple(b)
        if k not in seen:
            seen.add(k)
            jobs.append(list(b))
bucket = jobs[idx]
for rep in range(3):
    roots = np.array(st.export_many(bucket), dtype=np.uint32)
    arr = np.zeros(1, dtype=NT._JOB)
    arr["roots"] = roots.ctypes.data
    arr["n"] = len(bucket)
    arr["flags"] = NT.PROGRAM | NT.HINTS
    blob = NT._registry_blob(c.kfm.registry)
    res = (ctypes.c_void_p * 1)()
    t = time.perf_counter()
    st.L.pflt_lower_many(st.h, arr.ctypes.data, 1, NT._p32(blob), len(blob), 1, res)
    tn = time.perf_counter() - t
    t = time.perf_counter()
    r = NT._Result(st, res[0])
    lo, prog = NT.NativeLowered(r), NT.NativeProgram(r, 0)
    tp = time.perf_counter() - t
    print(f"rep {rep}: native {tn * 1e3:.2f} ms, wrap {tp * 1e3:.3f} ms, status {st.L.pflt_result_status(res[0])}, "
          f"ins {r.info[6]} vars {r.info[0]}", flush=True)
    del lo, prog, r
