"""Test tooling: an engine with the interface of mythril_amd.engine.Engine whose "device" is
the C oracle (oracle/coracle.c) — so the host pipeline above the C ABI (gpu_check.check_sets,
the drop-in Optimize, the tx-boundary batch) runs end to end in CPU tests.  The GPU tests
run the same pipeline on the real engine.  Never imported by mythril_amd/.
"""

from __future__ import annotations

import numpy as np

import coracle_py
import pyoracle as O

from mythril_amd import ir
from mythril_amd.engine import NOT_FOUND, CheckResult


class _DB:
    def __init__(self, batch):
        self.batch = batch
        self.packed = coracle_py.Packed(batch)

    def __len__(self):
        return len(self.batch)

    def free(self):
        pass


class OracleEngine:
    """upload / check / materialize with the kernel's contract (smallest witness index)."""

    def __init__(self):
        self.launches = 0
        self.last_budget = None

    def upload(self, programs):
        return _DB(programs if isinstance(programs, ir.Batch) else ir.Batch(programs))

    def check(self, db, budget=65536, seed=0, flags=0, timeout_ms=0):
        self.launches += 1
        self.last_budget = budget
        found = np.full(len(db), NOT_FOUND, dtype=np.uint32)
        for s in range(len(db)):
            f = db.packed.first_sat(s, seed, budget)
            if f is not None:
                found[s] = f
        return CheckResult(found, budget * len(db), budget * len(db), 0, 0.0)

    def eval_assignments(self, db, set_id, soa):
        """Engine.eval_assignments: the SAT flag of each explicit candidate ([var][limb][cand])."""
        self.evals = getattr(self, "evals", 0) + 1
        sv = O.SetView.from_batch(db.batch, int(set_id))
        nv = len(db.batch.programs[set_id].vars)
        out = []
        for c in range(soa.shape[-1]):
            vals = [O.limbs_to_int(soa[v, :, c]) for v in range(nv)]
            out.append(bool(sv.evaluate(vals)))
        return np.array(out, dtype=bool)

    def eval_programs(self, pack, soa):
        """Engine.eval_programs: flags [program][cand] of the packed programs, program s
        reading SoA rows descs[s].var_off .. + n_vars (mythril_amd/model_cache.py groups)."""
        self.evals = getattr(self, "evals", 0) + 1
        code, consts, schema, descs = pack
        b = ir.Batch.__new__(ir.Batch)
        b.code, b.consts = code.reshape(-1, 4), consts.reshape(-1, 8)
        b.schema, b.descs = schema.reshape(-1, 4), descs.reshape(-1, 8)
        b.parents = np.zeros((0, 8), dtype=np.uint32)
        out = np.zeros((len(b.descs), soa.shape[-1]), dtype=bool)
        for s in range(len(b.descs)):
            sv = O.SetView.from_batch(b, s)
            off, nv = int(b.descs[s][4]), int(b.descs[s][5])
            for c in range(soa.shape[-1]):
                out[s, c] = bool(sv.evaluate([O.limbs_to_int(soa[off + v, :, c]) for v in range(nv)]))
        return out

    def keccak256(self, messages):
        return [O.keccak256(bytes(m)) for m in messages]

    def materialize_limbs(self, db, set_ids, cand_ids, seed=0):
        """Engine.materialize_limbs: the (set, candidate) pairs' variables as limb rows."""
        self.materialized = getattr(self, "materialized", 0) + len(set_ids)
        vals = [x for vs in self.materialize(db, set_ids, cand_ids, seed) for x in vs]
        return ir.limbs_array(vals) if vals else np.zeros((0, 8), dtype=np.uint32)

    def materialize(self, db, set_ids, cand_ids, seed=0):
        out = []
        for s, c in zip(set_ids, cand_ids):
            sv = O.SetView.from_batch(db.batch, int(s))
            out.append([int(v) for v in sv.gen_assignments(np.array([c], dtype=np.uint64), seed)[0]])
        return out


def install(monkeypatch):
    """Make gpu_check.check_sets run on the oracle engine."""
    import mythril_amd.engine as E

    eng = OracleEngine()
    monkeypatch.setattr(E, "get_engine", lambda device=None: eng)
    from mythril_amd.smt import gpu_check

    monkeypatch.setattr(gpu_check.CONFIG, "workers", 1)
    gpu_check.reset_cache()
    return eng
