"""Native lowering time per bucket job of chosen single-query sample queries (bench.py
discharge numbering, tools/sq_tail.py): min over repetitions, with the program size, the
variable count and the hint solver's satisfied roots.  With PF_LOWER_SO pointing at a
-DPFLT_PROFILE build, the phase totals print at exit.  GPU-box tool (the corpus build hashes
on the engine).

usage: python tools/lower_query_probe.py i,j,... [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import native_terms, terms as T  # noqa: E402

idx = [int(i) for i in sys.argv[1].split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = corpus.build(48, 2, seed=2024)
sample = [q for q in c.queries if q.label == "sat"][:96]
st = native_terms.batch_api()
for i in idx:
    cs = [x for x in sample[i].constraints if x is not T.TRUE]
    for bk in native_terms.buckets(cs):
        job = [(list(bk), None)]
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            out = native_terms.lower_many(job, c.kfm.registry, True, [0], 1, st)
            best = min(best, time.perf_counter() - t0)
        lo, prog, err = out[0]
        if err:
            print(f"q{i} bucket {len(bk)}: {err}")
            continue
        info = prog.native_result.info
        ops = {}
        for t in bk:
            stack, seen = [t], set()
            while stack:
                u = stack.pop()
                if u in seen:
                    continue
                seen.add(u)
                ops[u.op] = ops.get(u.op, 0) + 1
                stack.extend(u.args)
        top = sorted(ops.items(), key=lambda kv: -kv[1])[:8]
        print(f"q{i} bucket {len(bk):2d} conj: {best * 1e6:7.1f} us  vars {info[0]} ins {info[6]} "
              f"roots {info[10]} hint_sat {info[13]}  terms {sum(ops.values())} {top}")
