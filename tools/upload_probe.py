"""Where a single query's upload phase goes (bench discharge single_query_ms phase
``upload``): the 96-query sample's searched programs captured from check_sets, then per
query the batch packing (ir.Batch) and pf_batch_create + pf_batch_free timed apart, min of
20 repetitions.  GPU-box tool.

usage: python tools/upload_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus, engine, ir  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402


def main():
    eng = engine.get_engine()
    c = corpus.build(48, 2, seed=2024)
    pack, create, free = [], [], []
    orig = eng.upload_sharded

    def rec(progs):
        # timed here, while the programs' native lowering results are alive (check_sets
        # releases them once uploaded)
        progs = list(progs)
        bp = bc = bf = 1e9
        for _ in range(20):
            t0 = time.perf_counter()
            b = ir.Batch(progs)
            t1 = time.perf_counter()
            db = engine.DeviceBatch(b, eng.device)
            t2 = time.perf_counter()
            db.free()
            t3 = time.perf_counter()
            bp, bc, bf = min(bp, t1 - t0), min(bc, t2 - t1), min(bf, t3 - t2)
        pack.append(bp)
        create.append(bc)
        free.append(bf)
        return orig(progs)

    eng.upload_sharded = rec
    for q in [q for q in c.queries if q.label == "sat"][:96]:
        gpu_check.reset_cache()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
    eng.upload_sharded = orig
    calls = pack
    us = lambda xs: f"median {1e6 * np.median(xs):.1f} mean {1e6 * np.mean(xs):.1f} us"  # noqa: E731
    print(f"{len(calls)} upload calls")
    print("pack (ir.Batch):          ", us(pack))
    print("pf_batch_create:          ", us(create))
    print("pf_batch_free:            ", us(free))


if __name__ == "__main__":
    main()
