"""Native lowering time per bucket job (min over repetitions) of the 96-query single-query
sample (bench discharge), one thread: compare libpflower.so builds with PF_LOWER_SO.
GPU-box tool (the corpus build hashes on the engine)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd import corpus
from mythril_amd.smt import native_terms, terms as T
c = corpus.build(48, 2, seed=2024)
sample = [q for q in c.queries if q.label == "sat"][:96]
st = native_terms.batch_api()
jobs = []
for q in sample:
    for bk in native_terms.buckets([x for x in q.constraints if x is not T.TRUE]): jobs.append((list(bk), None))
best = 1e9
for rep in range(25):
    t0=time.perf_counter()
    out = native_terms.lower_many(jobs, c.kfm.registry, True, [0]*len(jobs), 1, st)
    best = min(best, time.perf_counter()-t0)
    del out
print(sys.argv[1], 'min us per job', round(best*1e6/len(jobs),1))
