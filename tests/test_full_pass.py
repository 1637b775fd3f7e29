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
    # chunks ramp up from chunk / 32 (at least one piece): 6 + 12 + 18 + 4 DAGs
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


def test_full_pass_reports_a_device_error_without_hanging():
    """An engine that fails mid-pass: the error comes back from run_full_pass (the uploader
    and device threads drain and stop) instead of a hang on the bounded queues."""
    import pytest

    class Failing(oracle_engine.OracleEngine):
        def check(self, db, budget=65536, seed=0, flags=0, timeout_ms=0):
            if self.launches >= 3:
                raise RuntimeError("device lost")
            return super().check(db, budget, seed, flags, timeout_ms)

    with pytest.raises(RuntimeError, match="device lost"):
        full_pass.run_full_pass(Failing(), dags=60, chunk=8, piece=4, workers=2, budget=64, seed=0,
                                mp_context="spawn")


def test_full_pass_reports_an_upload_error_without_hanging():
    import pytest

    class Failing(oracle_engine.OracleEngine):
        def __init__(self):
            super().__init__()
            self.uploads = 0

        def upload(self, programs):
            self.uploads += 1
            if self.uploads >= 4:
                raise ValueError("bad batch")
            return super().upload(programs)

    with pytest.raises(ValueError, match="bad batch"):
        full_pass.run_full_pass(Failing(), dags=60, chunk=8, piece=4, workers=2, budget=64, seed=0,
                                mp_context="spawn")
