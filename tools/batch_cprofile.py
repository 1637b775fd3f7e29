"""cProfile of the bench's batched discharge pass (bench.py discharge: the 1,006-query corpus
in one check_sets call, answer caches cleared, terms already stored) on the GPU box: where the
host part of the batched rate goes.  Tool.

usage: [COLD=1] python tools/batch_cprofile.py [top] [reps]
COLD=1 profiles the first pass instead (the terms enter the native store: bench's cold rate)."""
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
if os.environ.get("COLD") == "1":
    import resource

    gc.collect()
    pr = cProfile.Profile()
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    t = time.perf_counter()
    pr.enable()
    gpu_check.check_sets(sets, registry=c.kfm.registry)
    pr.disable()
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    print(f"cold pass (profiled) {1e3 * (time.perf_counter() - t):.1f} ms",
          {k: round(1e3 * v, 2) for k, v in gpu_check.STATS.phase_s.items()},
          f"minor faults {r1.ru_minflt - r0.ru_minflt}, user {r1.ru_utime - r0.ru_utime:.3f} s, "
          f"sys {r1.ru_stime - r0.ru_stime:.3f} s")
    pstats.Stats(pr).sort_stats("tottime").print_stats(top)
    sys.exit(0)
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
