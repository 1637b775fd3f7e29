"""bench.py's full-pass leg (tools/full_pass.py: config 3 over a range of DAG ids, the host
workers building chunks while the device sweeps) on the C oracle: the chunked, offset-
patched batches give every DAG the verdict it gets on its own."""

import os
import sys

import numpy as np

import oracle_engine
from mythril_amd import ir, synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import full_pass  # noqa: E402


def test_full_pass_chunks_match_per_dag_search(monkeypatch):
    eng = oracle_engine.OracleEngine()
    res = full_pass.run_full_pass(eng, dags=40, chunk=16, piece=6, workers=2, budget=256, seed=0,
                                  mp_context="spawn")
    fs = res["full_sweep"]
    # chunks ramp up from chunk / 8 (at least one piece): 6 + 12 + 18 + 4 DAGs
    assert fs["evals_full"] == 40 * 256 and fs["chunks"] == 4
    want = 0
    for i in range(40):
        p = synth.random_dag_set(i, plant=False)[0]
        r = eng.check(eng.upload([p]), budget=256, seed=0)
        want += int(r.sat.sum())
    assert fs["sets_with_witness"] == want
    # the planted pass: every DAG's witness is candidate 0
    assert res["planted_early_exit"]["sets_with_witness"] == 40
    assert res["full_sweep"]["evals_per_s_wall"] > 0
