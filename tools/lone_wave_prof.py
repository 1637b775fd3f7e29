#!/usr/bin/env python3
"""Where a lone wave's time goes on the single-query tail's longest program (diagnostic).

The slowest single queries of the bench sample (BECToken#1 tx1, storage / calldata-heavy
buckets of 5-9k instructions) are one set each: one wave walks the whole program, so its
time is the per-instruction latency, not throughput.  This runs that program alone on the
unit-profiling library (tools/unitprof.py --build: every bytecode instruction's s_memtime
delta accumulated per datapath unit, FETCH = the wait for the instruction's scalar load)
with one candidate group, and prints the cycle shares next to the program's opcode mix.

usage (GPU): python tools/lone_wave_prof.py [sample_index ...]
"""
import ctypes
import json
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from unitprof import BUCKETS, PROF_SO  # noqa: E402


def main():
    from mythril_amd import _lib, corpus, ir
    from mythril_amd.smt import gpu_check

    L = _lib.load_library(PROF_SO)
    L.pf_prof_read.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.pf_prof_read.restype = ctypes.c_int
    from mythril_amd import engine

    eng = engine.get_engine()
    got = []
    orig = eng.upload

    def rec(progs, *a, **k):
        for p in progs:
            if hasattr(p, "decode"):
                p.decode()
        got.append(list(progs))
        return orig(progs, *a, **k)

    eng.upload = rec
    c = corpus.build(48, 2, seed=2024)
    sample = [q for q in c.queries if q.label == "sat"][:96]
    idxs = [int(x) for x in sys.argv[1:]] or [16, 18]
    nb = len(BUCKETS)
    for qi in idxs:
        q = sample[qi]
        gpu_check.reset_cache()
        got.clear()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
        big = max(got[-1], key=len)  # decoded at upload; re-packed as a plain program
        prog = ir.PackedProgram(big.words, big.consts, big.vars, seed=big.seed)
        mix = Counter(ir.OPNAMES[i.op] for i in prog.code)
        eng.upload = orig
        db = eng.upload([prog])
        rows = {}
        for budget in (64, 64, 4096):
            r = eng.check(db, budget=budget, seed=gpu_check.CONFIG.seed, flags=gpu_check.CONFIG.flags)
            out = (ctypes.c_uint64 * (nb + 1))()
            _lib.check(L.pf_prof_read(db.handle, out), "pf_prof_read")
            tot = sum(out[:15])
            rows[budget] = {"kernel_ms": round(r.kernel_ms, 3), "found": int(r.found[0]),
                            "wave_cycles": int(out[nb]), "instr_cycles": int(tot),
                            "cycles_per_instr": round(tot / max(len(prog), 1), 1),
                            "share": {BUCKETS[i]: round(out[i] / max(tot, 1), 4)
                                      for i in range(len(BUCKETS)) if out[i]}}
        db.free()
        eng.upload = rec
        print(json.dumps({"query": q.origin, "instructions": len(prog),
                          "mix": dict(mix.most_common(12)), "runs": rows}, indent=1), flush=True)


if __name__ == "__main__":
    main()
