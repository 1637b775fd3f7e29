"""Cold vs warm native lowering in one fresh process: the corpus's bucket jobs lowered by
native_terms.lower_many on one thread, three times; with PF_LOWER_SO at a -DPFLT_PROFILE build
the phase totals print at exit (summed over the three calls; PFLT_PROFILE_RESET between calls
is not available, so compare against a run with one call: argv[1] = calls).  GPU-box tool.

usage: python tools/cold_lower_probe.py [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check, native_terms as NT, terms as T  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
c = corpus.build(48, 2, seed=2024)
st = NT.batch_api()
jobs, seen = [], set()
for q in c.queries:
    for b in NT.buckets([x for x in q.constraints if x is not T.TRUE]) or []:
        k = tuple(b)
        if k not in seen:
            seen.add(k)
            jobs.append((list(b), None))
seeds = [gpu_check._set_seed(b) for b, _ in jobs]
for i in range(calls):
    t = time.perf_counter()
    out = NT.lower_many(jobs, c.kfm.registry, True, seeds, 1, st)
    dt = time.perf_counter() - t
    print(f"call {i}: {len(jobs)} jobs {dt * 1e3:.1f} ms ({dt * 1e6 / len(jobs):.1f} us/job)", flush=True)
    del out
