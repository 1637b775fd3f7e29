#!/usr/bin/env python3
"""Diagnostic: config-3 DAGs whose planted witness (attached as the parent model, so it is
candidate 0) the GPU search does NOT report at candidate 0.  Every such set is a kernel
error: the oracle evaluates the same candidate as SAT.  Prints the DAG ids, the oracle's
verdict on candidate 0, and the GPU's verdict on the same explicit assignment
(pf_eval_assignments), then writes the failing programs to --out (JSON) for host replay.

    python tools/planted_miss.py --first 0 --n 65536 [--workers 16]
"""
import argparse
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _planted(args):
    import copy

    from mythril_amd import synth

    first, n = args
    out = []
    for i in range(first, first + n):
        p, wit = synth.random_dag_set(i, plant=False)
        q = copy.copy(p)
        q.vars = [copy.copy(v) for v in p.vars]
        for v, x in zip(q.vars, wit):
            v.parent = x
        out.append(q)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/planted_miss.json")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        from mythril_amd import _lib

        _lib.load_library(a.lib)
    import numpy as np

    pool = ProcessPoolExecutor(a.workers)
    piece = 1024
    progs = []
    for ps in pool.map(_planted, [(f, min(piece, a.first + a.n - f)) for f in range(a.first, a.first + a.n, piece)]):
        progs += ps
    pool.shutdown()
    from mythril_amd import ir
    from mythril_amd.engine import Engine
    import pyoracle as O

    eng = Engine(0)
    db = eng.upload(progs)
    r = eng.check(db, budget=64, seed=0, flags=ir.FLAG_EARLY_EXIT)
    miss = [int(s) for s in np.nonzero(r.found != 0)[0]]
    print(json.dumps({"dags": a.n, "first": a.first, "missed_at_candidate_0": len(miss)}), flush=True)
    b = ir.Batch(progs)
    rows = []
    for s in miss[:32]:
        sv = O.SetView.from_batch(b, s)
        vals = sv.gen_assignments(np.array([0], dtype=np.uint64), 0)[0]
        ok = sv.evaluate(vals)
        one = eng.upload([progs[s]])
        soa = ir.pack_assignments(progs[s], [vals])
        gpu = eng.eval_assignments(one, 0, soa)
        one.free()
        print(json.dumps({"dag": a.first + s, "found": int(r.found[s]), "oracle_cand0": bool(ok),
                          "gpu_eval_cand0": int(gpu[0])}), flush=True)
        rows.append({"dag": a.first + s, "values": [hex(v) for v in vals],
                     "code": [repr(i) for i in progs[s].code]})
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
