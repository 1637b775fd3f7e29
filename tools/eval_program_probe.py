"""GPU box: wall time of pf_eval_program (one call: validate, upload, launch, read back) on
the explicit programs of corpus queries, 100 candidates each, vs program length."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402

from mythril_amd import corpus as C  # noqa: E402
from mythril_amd import model_cache as MC  # noqa: E402
from mythril_amd.engine import get_engine  # noqa: E402
from mythril_amd.smt import terms as T  # noqa: E402

eng = get_engine()
corp = C.build(n_scenarios=8, txs=2, seed=7)
rows_out = []
for q in corp.queries[:60:3]:
    leaves, prog = MC._lower_explicit([c for c in q.constraints if c is not T.TRUE])
    ev = C._PlantedEval(q.planted, corp.kfm.registry) if q.planted is not None else None
    vals = [int(ev.ev(t)) & ((1 << max(t.width, 1)) - 1) if ev else 0 for t in leaves]
    for n_cand in (4, 100):
        soa = MC.soa_of(MC.rows_of_ints([vals] * n_cand), MC.n_vars(prog))
        eng.eval_program(prog, soa)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            eng.eval_program(prog, soa)
            ts.append(1e3 * (time.perf_counter() - t0))
        rows_out.append({"n_ins": int(prog.native_result.info[6]) if hasattr(prog, "native_result") else len(prog.code),
                         "n_vars": MC.n_vars(prog), "n_cand": n_cand, "ms_median": float(np.median(ts))})
print(json.dumps(rows_out))
