"""Fixed cost of one small search (the fork-prune call site: one query, a few buckets):
wall time of Engine.check on 1..16 planted config-3 sets (candidate 0 is the witness, so the
kernel stops in its first group) against the kernel's own event time.  The difference is the
host/runtime part of the search phase: the queue/verdict resets, the launch, the copies of
the counters and verdicts and the stream synchronisation.  GPU tool (tools/, not product).

usage: python tools/search_overhead_probe.py [reps] [library]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import _lib, ir, synth  # noqa: E402
from mythril_amd.engine import get_engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    if len(sys.argv) > 2:  # an alternative build (tools/build_variants.sh)
        _lib.load_library(sys.argv[2])
    eng = get_engine()
    flags = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT
    for plant, n in ((True, 1), (True, 4), (True, 16), (False, 1), (False, 4), (False, 16)):
        db = eng.upload([synth.random_dag_set(i, plant=plant)[0] for i in range(n)])
        for _ in range(20):
            eng.check(db, budget=65536, seed=0, flags=flags)
        wall, kern = [], []
        for _ in range(reps):
            t = time.perf_counter()
            r = eng.check(db, budget=65536, seed=0, flags=flags)
            wall.append(1e3 * (time.perf_counter() - t))
            kern.append(r.kernel_ms)
        assert not plant or int(r.sat.sum()) == n, "planted witnesses must be found"
        w, k = np.array(wall), np.array(kern)
        print(f"{'planted' if plant else 'search '} sets {n:3d} ({int(r.sat.sum())} sat): wall median {np.median(w):.4f} ms mean {w.mean():.4f} | kernel (events) "
              f"median {np.median(k):.4f} ms | host+runtime {np.median(w) - np.median(k):.4f} ms | witnesses {[int(x) for x in r.found[:16]]}", flush=True)
        db.free()
    # upload (pf_batch_create: validation, device program, one copy) of one prepared batch
    from mythril_amd.ir import Batch
    for n in (1, 4, 16):
        b = Batch([synth.random_dag_set(i, plant=True)[0] for i in range(n)])
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            db = eng.upload(b)
            ts.append(1e3 * (time.perf_counter() - t))
            db.free()
        print(f"upload sets {n:3d}: median {np.median(ts):.4f} ms mean {np.mean(ts):.4f}", flush=True)


if __name__ == "__main__":
    main()
