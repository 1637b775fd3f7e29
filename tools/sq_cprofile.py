"""cProfile of the bench's single-query sample (bench.py discharge: 96 planted-SAT corpus
queries, one check_sets call each with the answer caches cleared) on the GPU box: where the
host part of a single query's latency goes.  Tool.

usage: [SQ_ONLY=i,j,..] python tools/sq_cprofile.py [top] [reps]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 40
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
gpu_check.warm_pool()
c = corpus.build(48, 2, seed=2024)
gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
sample = [q for q in c.queries if q.label == "sat"][:96]
if os.environ.get("SQ_ONLY"):   # comma-separated sample indices (tools/sq_tail.py numbering)
    sample = [sample[int(i)] for i in os.environ["SQ_ONLY"].split(",")]


def one_pass():
    lat = []
    for q in sample:
        gpu_check.reset_cache()
        t = time.perf_counter()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
        lat.append(1e3 * (time.perf_counter() - t))
    return lat


one_pass()
gpu_check.STATS.phase_s.clear()
lat = one_pass()
print("mean ms (no profiler)", round(sum(lat) / len(lat), 3),
      {k: round(1e3 * v / len(lat), 3) for k, v in gpu_check.STATS.phase_s.items()})
pr = cProfile.Profile()
pr.enable()
for _ in range(reps):
    one_pass()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(top)
