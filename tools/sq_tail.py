"""The single-query sample's tail (bench.py discharge: 96 planted-SAT corpus queries, one
check_sets call each, answer caches cleared): per-query latency and phases of the slowest
queries, with their bucket count and program sizes.  GPU-box tool.

usage: [SQ_ONLY=i,j,..] [SQ_NO_HINTS=1] python tools/sq_tail.py [n_slowest]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check, native_terms, terms as T  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 12
gpu_check.warm_pool()
c = corpus.build(48, 2, seed=2024)
gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
sample = [q for q in c.queries if q.label == "sat"][:96]
cfg = gpu_check.CONFIG
if os.environ.get("SQ_NO_HINTS") == "1":
    from dataclasses import replace
    cfg = replace(cfg, hints=False)
only = [int(i) for i in os.environ["SQ_ONLY"].split(",")] if os.environ.get("SQ_ONLY") else None
rows = []
for rep in range(3):
    for i, q in enumerate(sample):
        if only is not None and i not in only:
            continue
        gpu_check.reset_cache()
        before = dict(gpu_check.STATS.phase_s)
        t = time.perf_counter()
        got = gpu_check.check_sets([q.constraints], registry=c.kfm.registry, config=cfg)[0]
        ms = 1e3 * (time.perf_counter() - t)
        ph = {k: round(1e3 * (v - before.get(k, 0.0)), 3) for k, v in gpu_check.STATS.phase_s.items()
              if v - before.get(k, 0.0) > 0}
        if rep == 2:
            rows.append((ms, i, dict(ph, sat=got is not None)))
lat = np.array([r[0] for r in rows])
print("median", round(float(np.median(lat)), 3), "p90", round(float(np.percentile(lat, 90)), 3),
      "p95", round(float(np.percentile(lat, 95)), 3), "max", round(float(lat.max()), 3))
for ms, i, ph in sorted(rows, reverse=True)[:top]:
    q = sample[i]
    cs = [x for x in q.constraints if x is not T.TRUE]
    bks = native_terms.buckets(cs) or []
    print(f"q{i:3d} {ms:7.3f} ms  conj {len(cs):3d} buckets {len(bks):2d} sizes {[len(b) for b in bks]}  {ph}")
