"""What a native lowering result's release costs (pflt_result_shrink after upload, then
pflt_result_free at eviction) over the bench's 1,006-query corpus buckets: total ms per pass
for each, and the largest single results.  GPU-box tool (the corpus build hashes on the
engine).

usage: python tools/shrink_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check, native_terms as NT, terms as T  # noqa: E402

c = corpus.build(48, 2, seed=2024)
st = NT.batch_api()
jobs = []
for q in c.queries:
    for b in NT.buckets([x for x in q.constraints if x is not T.TRUE]) or []:
        jobs.append((list(b), None))
seeds = [gpu_check._set_seed(b) for b, _ in jobs]
for rep in range(3):
    out = NT.lower_many(jobs, c.kfm.registry, True, seeds, 1, st)
    los = [lo for lo, _, err in out if err is None]
    t = time.perf_counter()
    per = []
    for lo in los:
        t1 = time.perf_counter()
        NT.shrink(lo)
        per.append((time.perf_counter() - t1, int(lo.res.info[8])))
    ts = time.perf_counter() - t
    t = time.perf_counter()
    del out, los, lo
    tf = time.perf_counter() - t
    per.sort(reverse=True)
    print(f"{len(per)} results: shrink {ts * 1e3:.2f} ms, free {tf * 1e3:.2f} ms; "
          f"slowest shrinks (us, dag nodes): {[(round(a * 1e6, 1), n) for a, n in per[:5]]}; "
          f"median {per[len(per) // 2][0] * 1e6:.2f} us")
