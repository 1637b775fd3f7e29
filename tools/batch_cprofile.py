"""cProfile of the bench's batched discharge pass (bench.py discharge: the 1,006-query corpus
in one check_sets call, answer caches cleared, terms already stored) on the GPU box: where the
host part of the batched rate goes.  Tool.

usage: python tools/batch_cprofile.py [top] [reps]"""
import cProfile
import gc
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 40
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gpu_check.warm_pool()
c = corpus.build(48, 2, seed=2024)
sets = [q.constraints for q in c.queries]
gpu_check.check_sets(sets, registry=c.kfm.registry)
for _ in range(2):
    gpu_check.reset_cache()
    gpu_check.STATS.phase_s.clear()
    gc.collect()
    t = time.perf_counter()
    gpu_check.check_sets(sets, registry=c.kfm.registry)
    dt = time.perf_counter() - t
    print(f"{len(sets)} queries {dt * 1e3:.1f} ms ({len(sets) / dt:.0f} q/s)",
          {k: round(1e3 * v, 2) for k, v in gpu_check.STATS.phase_s.items()})
pr = cProfile.Profile()
for _ in range(reps):
    gpu_check.reset_cache()
    gc.collect()
    pr.enable()
    gpu_check.check_sets(sets, registry=c.kfm.registry)
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(top)
