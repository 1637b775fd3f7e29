"""Test tooling: the discharge pipeline of mythril_amd/smt/gpu_check.py (independence buckets
-> lowering -> hint models -> candidate search) with the C oracle (oracle/coracle.c) standing
in for the GPU, so the corpus hit rate can be checked and iterated on without a GPU.

``python tests/discharge_oracle.py [n_scenarios] [budget]`` prints the rates.
"""

from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import coracle_py  # noqa: E402
import pyoracle as O  # noqa: E402

from mythril_amd import ir  # noqa: E402
from mythril_amd import keccak_manager as KM  # noqa: E402
from mythril_amd.lower import LoweringError  # noqa: E402
from mythril_amd.smt import symbol_factory  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402
from mythril_amd.smt.gpu_check import _lower_bucket  # noqa: E402
from mythril_amd.smt.independence import buckets  # noqa: E402


def host_keccak():
    """Concrete hashes from the oracle's Keccak-256 (the product uses the GPU kernel)."""
    KM.KeccakFunctionManager.find_concrete_keccak = staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256))


def discharge(queries, registry, budget=4096, seed=0x4D595448, hints=True, split=True):
    """Per query: True (every bucket has a witness among `budget` candidates), False, or
    None (a bucket did not lower)."""
    progs, index, per_query = [], {}, []
    for q in queries:
        cs = [c for c in q.constraints if c is not T.TRUE]
        keys = []
        ok = True
        for b in (buckets(cs) if split else [cs]):
            key = tuple(b)
            if key not in index:
                try:
                    _, prog = _lower_bucket(b, registry, None, hints)
                    index[key] = len(progs)
                    progs.append(prog)
                except LoweringError:
                    index[key] = None
            if index[key] is None:
                ok = False
            keys.append(key)
        per_query.append(keys if ok else None)
    found = {}
    if progs:
        P = coracle_py.Packed(ir.Batch(progs))
        for i in range(len(progs)):
            found[i] = P.first_sat(i, seed, budget) is not None
    out = []
    for keys in per_query:
        out.append(None if keys is None else all(found[index[k]] for k in keys))
    return out, len(progs)


def main():
    from mythril_amd import corpus

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    host_keccak()
    t0 = time.time()
    c = corpus.build(n, 2)
    n_sat = corpus.validate(c)
    t1 = time.time()
    res, nb = discharge(c.queries, c.kfm.registry, budget)
    t2 = time.time()
    sat_lab = [r for r, q in zip(res, c.queries) if q.label == "sat"]
    print(f"{len(c.queries)} queries ({n_sat} planted-SAT), {nb} distinct buckets; "
          f"build {t1 - t0:.1f}s, pipeline {t2 - t1:.1f}s")
    print(f"discharged: {sum(1 for r in res if r)}/{len(res)} all, "
          f"{sum(1 for r in sat_lab if r)}/{len(sat_lab)} planted-SAT, "
          f"lowering failures {sum(1 for r in res if r is None)}")
    for r, q in zip(res, c.queries):
        if q.label == "sat" and not r:
            print("  missed:", q.origin, "(not lowered)" if r is None else "")


if __name__ == "__main__":
    main()
