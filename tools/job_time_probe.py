"""Per-bucket native lowering time over the corpus's 1,023 distinct bucket jobs, each lowered
alone (one thread), twice in one fresh process: the slowest jobs cold and warm, and the sum —
whether one long job sets the batched cold pass's critical path.  GPU-box tool.

usage: python tools/job_time_probe.py [top]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import corpus  # noqa: E402
from mythril_amd.smt import gpu_check, native_terms as NT, terms as T  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 8
c = corpus.build(48, 2, seed=2024)
st = NT.batch_api()
jobs, seen = [], set()
for q in c.queries:
    for b in NT.buckets([x for x in q.constraints if x is not T.TRUE]) or []:
        k = tuple(b)
        if k not in seen:
            seen.add(k)
            jobs.append((list(b), None))
times = []
for rep in range(2):
    tj = []
    for j, job in enumerate(jobs):
        t = time.perf_counter()
        out = NT.lower_many([job], c.kfm.registry, True, [gpu_check._set_seed(job[0])], 1, st)
        tj.append(time.perf_counter() - t)
        del out
    times.append(tj)
    order = sorted(range(len(jobs)), key=lambda i: -tj[i])[:top]
    print(f"pass {rep}: sum {sum(tj) * 1e3:.1f} ms; slowest (ms, conjuncts, job index): "
          f"{[(round(tj[i] * 1e3, 2), len(jobs[i][0]), i) for i in order]}", flush=True)
    if rep == 0:
        i = order[0]
        ops = {}
        for t0 in jobs[i][0]:
            stack, seen_t = [t0], set()
            while stack:
                u = stack.pop()
                if u in seen_t:
                    continue
                seen_t.add(u)
                ops[u.op] = ops.get(u.op, 0) + 1
                stack.extend(u.args)
        print("slowest job ops:", sorted(ops.items(), key=lambda kv: -kv[1])[:12])
        print("slowest job:", str(jobs[i][0])[:600])
