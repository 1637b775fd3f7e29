#!/usr/bin/env python3
"""Host-thread scaling of the native lowering (pflt_lower_many) on the bench corpus's 1,023
buckets (diagnostic, tools/).  Times each thread count several times after a warm call, so
the term export and lazy initialisation are outside the clock.

usage: python tools/lower_threads_probe.py [reps] [--check-sets]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
    from mythril_amd import corpus
    from mythril_amd.smt import gpu_check
    from mythril_amd.smt import native_terms as NT
    from mythril_amd.smt.independence import buckets

    c = corpus.build(48, 2, seed=2024)
    seen, bks = set(), []
    for q in c.queries:
        for b in buckets(q.constraints):
            if tuple(b) not in seen:
                seen.add(tuple(b))
                bks.append(b)
    jobs = [(b, None) for b in bks]
    seeds = [gpu_check._set_seed(b) for b in bks]
    NT.lower_many(jobs, c.kfm.registry, True, seeds, 16)
    print(f"{len(bks)} buckets, os.cpu_count {os.cpu_count()}, sched_getaffinity "
          f"{len(os.sched_getaffinity(0))}", flush=True)
    for th in (1, 2, 4, 8, 16, 32):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            NT.lower_many(jobs, c.kfm.registry, True, seeds, th)
            ts.append(time.perf_counter() - t0)
        print(f"threads {th:2d}: min {1e3 * min(ts):7.1f} ms, median {1e3 * sorted(ts)[len(ts) // 2]:7.1f} ms",
              flush=True)
    if "--check-sets" in sys.argv:  # the bench's batched call, phases per repeat (GPU)
        for rep in range(3):
            gpu_check.reset_cache()
            before = dict(gpu_check.STATS.phase_s)
            t0 = time.perf_counter()
            gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
            dt = time.perf_counter() - t0
            ph = {k: round(1e3 * (v - before.get(k, 0.0)), 1) for k, v in gpu_check.STATS.phase_s.items()}
            print(f"check_sets {1e3 * dt:.1f} ms, phases (ms) {ph}", flush=True)


if __name__ == "__main__":
    main()
