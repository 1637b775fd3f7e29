"""Probe of the cold single-query latency (bench.py discharge.single_query_ms): the same
96-query sample, one check_sets call per query, with each call's searches recorded — bucket
count, program lengths, kernel time and the witness index per bucket — so the slow tail can
be attributed.  GPU tool (tools/, not product).

usage: python tools/single_query_probe.py [n_scenarios] [top]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus, engine  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    gpu_check.warm_pool()
    c = corpus.build(n, 2, seed=2024)
    corpus.validate(c)
    eng = engine.get_engine()
    calls = []
    orig = eng.check

    def rec(db, *a, **k):
        r = orig(db, *a, **k)
        lens = [int(d[1]) for d in np.asarray(db.batch.descs).reshape(-1, 8)]
        calls.append({"sets": len(db), "kernel_ms": round(r.kernel_ms, 3),
                      "found": [int(x) if x != 0xFFFFFFFF else -1 for x in r.found], "lens": lens})
        return r

    eng.check = rec
    # warm: the corpus in one call, as the bench runs it before the sample
    gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
    sample = [q for q in c.queries if q.label == "sat"][:96]
    gpu_check.STATS.probe_split = gpu_check.STATS.probe_split_sat = 0
    rows = []
    for i, q in enumerate(sample):
        gpu_check.reset_cache()
        calls.clear()
        before = dict(gpu_check.STATS.phase_s)
        ts = time.perf_counter()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
        ms = 1e3 * (time.perf_counter() - ts)
        ph = {k: round(1e3 * (v - before.get(k, 0.0)), 3) for k, v in gpu_check.STATS.phase_s.items()}
        rows.append((ms, i, q.origin, ph, list(calls)))
    lat = np.array([r[0] for r in rows])
    print(f"median {np.median(lat):.3f} mean {lat.mean():.3f} p95 {np.percentile(lat, 95):.3f} "
          f"max {lat.max():.3f} ms  split probe {gpu_check.STATS.probe_split} buckets, "
          f"{gpu_check.STATS.probe_split_sat} answered")
    for ms, i, origin, ph, cl in sorted(rows, key=lambda r: -r[0])[:top]:
        print(f"{ms:8.3f} ms  query {i} {origin}  phases {ph}")
        for cc in cl:
            print(f"          search: {cc['sets']} buckets, kernel {cc['kernel_ms']} ms, "
                  f"found {cc['found'][:12]}, program lengths {cc['lens'][:12]}")


if __name__ == "__main__":
    main()
