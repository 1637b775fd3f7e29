"""Opcode x width census of the lowered programs the single-query sample searches (bench
discharge: the 96 planted-SAT queries of the 48-scenario corpus, one check_sets call each),
as lowered (before pf_batch_create's device peepholes).  What a narrow-width interpreter path
could cover: W instructions by result width class, B instructions, per opcode.  GPU-box tool
(the corpus build and the searches use the engine).

usage: python tools/bucket_census.py [out.md]"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus, engine, ir  # noqa: E402
from mythril_amd.smt import gpu_check  # noqa: E402


def cls(op, w):
    if op >= ir.B_CONST or op == ir.ASSERT:
        return "B"
    return "<=32" if w <= 32 else "<=64" if w <= 64 else "<=160" if w <= 160 else "<=256"


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    eng = engine.get_engine()
    sets = []
    orig = eng.upload

    def up(programs, *a, **k):
        b = programs if isinstance(programs, ir.Batch) else ir.Batch(programs)
        code = np.asarray(b.code, dtype=np.uint32).reshape(-1, 4)
        for d in np.asarray(b.descs, dtype=np.uint32).reshape(-1, 8):
            sets.append(code[d[0]:d[0] + d[1]])
        return orig(programs, *a, **k)

    c = corpus.build(48, 2, seed=2024)
    eng.upload = up
    for q in [q for q in c.queries if q.label == "sat"][:96]:
        gpu_check.reset_cache()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
    names = {}
    for k, v in vars(ir).items():
        if isinstance(v, int) and (k.startswith("W_") or k.startswith("B_") or k in ("ASSERT", "END")):
            names.setdefault(v, k)
    by = collections.Counter()
    width = collections.Counter()
    for s in sets:
        for ins in s:
            op, w = int(ins[0]) & 0xFF, (int(ins[0]) >> 8) & 0x3FF
            by[(names.get(op, str(op)), cls(op, w))] += 1
            width[cls(op, w)] += 1
    tot = sum(width.values())
    lines = [f"# Opcode x width census: {len(sets)} searched programs, {tot} lowered instructions", "",
             "| class | instructions | share |", "|---|---|---|"]
    lines += [f"| {k} | {v} | {100 * v / tot:.1f} % |" for k, v in sorted(width.items())]
    lines += ["", "| opcode | class | instructions | share |", "|---|---|---|---|"]
    lines += [f"| {o} | {k} | {v} | {100 * v / tot:.1f} % |" for (o, k), v in by.most_common(30)]
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
