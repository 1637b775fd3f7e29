"""Where does the candidate search (host hints off) miss on the LASER-shaped corpus?

CPU probe: runs gpu_check.check_sets over mythril_amd/corpus.py on the C oracle engine
(tests/oracle_engine.py) with hints off, in one batch (no parents) and in live order (fork
pairs one call at a time, parents from the previous witnesses), and prints the origins of
the queries neither answers plus the bucket conjuncts that failed.  Measurement scaffolding.
"""

import os
import sys
import time
from collections import Counter
from dataclasses import replace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import oracle_engine  # noqa: E402

import mythril_amd.engine as E  # noqa: E402
from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402
from mythril_amd.smt.independence import buckets  # noqa: E402


def main():
    n_sc = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    eng = oracle_engine.OracleEngine()
    E.get_engine = lambda device=None: eng
    gpu_check.CONFIG.workers = 1
    c = corpus.build(n_sc, 2, seed=2024)
    qs = c.queries
    reg = c.kfm.registry
    cfg = replace(gpu_check.CONFIG, hints=False, budget=budget)
    gpu_check.reset_cache()
    t0 = time.time()
    ms = gpu_check.check_sets([q.constraints for q in qs], registry=reg, config=replace(cfg, parents=False))
    t1 = time.time()
    print(f"batch, no hints, no parents: {sum(m is not None for m in ms)}/{len(qs)} ({t1 - t0:.1f}s)")
    gpu_check.reset_cache()
    live = [None] * len(qs)
    idx = {id(q): i for i, q in enumerate(qs)}
    for g in corpus.live_order_groups(qs):
        r = gpu_check.check_sets([q.constraints for q in g], registry=reg, config=cfg)
        for q, m in zip(g, r):
            live[idx[id(q)]] = m
    t2 = time.time()
    origins = Counter(m.origin for m in live if m is not None)
    print(f"live order, no hints, parents: {sum(m is not None for m in live)}/{len(qs)} "
          f"({t2 - t1:.1f}s) origins {dict(origins)}")
    sat_lab = [i for i, q in enumerate(qs) if q.label == "sat"]
    print(f"planted-SAT queries: {len(sat_lab)}; live answered {sum(live[i] is not None for i in sat_lab)}")
    miss = Counter()
    shown = 0
    gpu_check.reset_cache()
    for i in sat_lab:
        if live[i] is not None:
            continue
        q = qs[i]
        site = q.origin.split("#")[0] + ":" + q.origin.split(":", 2)[-1]
        miss[site] += 1
        if shown < int(os.environ.get("SHOW", "6")):
            shown += 1
            print("----", q.origin)
            for b in buckets(q.constraints):
                r = gpu_check.check_sets([b], registry=reg, config=replace(cfg, parents=False))[0]
                if r is None:
                    print("  failing bucket:")
                    for cc in b:
                        print("   ", T.to_sexpr(cc)[:300])
    print("misses by site:", miss.most_common(30))


if __name__ == "__main__":
    main()
