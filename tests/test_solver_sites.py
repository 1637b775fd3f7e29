"""Seam #1's ``Solver()`` half: the modules that build ``mythril.laser.smt.Solver`` directly,
outside the query funnel — the symbolic calldata slice loop (ref
laser/ethereum/state/calldata.py:64-93, ``s = Solver()`` at :78) and the summary plugin
(plugins/summary/summary.py:114, summary/core.py:223).  ``integration.install()`` rebinds
their ``Solver`` to ``GpuSolver``, which shares ``GpuOptimize``'s objective-free GPU path and
its single ``@stat_smt_query`` count.

The slice loop's queries are ``current_index != stop``: SAT on every iteration but the
last, which is UNSAT and ends the slice.  With a real z3 the last one returns ``unsat``; the
stand-in z3 answers ``unknown`` (it decides nothing), which ends the loop the same way — so
``parts`` is what the reference loop returns with libz3: one element per index in
[start, stop).  The CPU tests run the engine's host pipeline on the C oracle; the ``gpu``
test runs the same loop on the MI355X engine.
"""

import pytest

import fake_z3 as z3
import mythril_standin
import oracle_engine
from mythril_amd import integration
from mythril_amd.smt import gpu_check
from mythril_amd.smt.solver import SolverStatistics


def _stats():
    import sys

    return sys.modules["mythril.laser.smt.solver.solver_statistics"].SolverStatistics()


def _fresh(monkeypatch, cpu):
    ns = mythril_standin.install(monkeypatch, z3)
    eng = oracle_engine.install(monkeypatch) if cpu else None
    if cpu:
        monkeypatch.setattr(gpu_check.CONFIG, "budget", 4096)
    gpu_check.reset_cache()
    integration._BATCH_CACHE.clear()
    st = SolverStatistics()
    st.gpu_sat = st.gpu_attempts = 0
    ms = _stats()
    ms.enabled, ms.query_count = True, 0
    return ns, eng


def _slice_loop(ns, start, stop, values):
    cd = ns.calldata.Calldata("1", values)
    return cd[start:stop]


def _run_slice_case(ns, start, stop, values):
    """The loop before and after install(): same parts, same query count; after install every
    SAT iteration is a GPU answer."""
    ms = _stats()
    ms.query_count = 0
    want = _slice_loop(ns, start, stop, values)       # stand-in z3: the first query is unknown
    assert ms.query_count == 1 and want == []
    integration.install()
    assert ns.calldata.Solver is integration.gpu_solver_class()
    ms.query_count = 0
    parts = _slice_loop(ns, start, stop, values)
    n = max(0, stop - start)
    assert [p.value for p in parts] == [values[i] if i < len(values) else None for i in range(start, stop)]
    assert len(parts) == n
    # one query per iteration plus the final UNSAT one, each counted once
    assert ms.query_count == n + 1
    assert SolverStatistics().gpu_sat == n
    assert SolverStatistics().gpu_attempts == n + 1
    return parts


@pytest.mark.parametrize("start,stop", [(4, 36), (0, 1), (7, 7), (60, 68)])
def test_calldata_slice_loop_through_gpu_solver(monkeypatch, start, stop):
    ns, _ = _fresh(monkeypatch, cpu=True)
    values = [(i * 37 + 5) & 0xFF for i in range(64)]
    parts = _run_slice_case(ns, start, stop, values)
    # bytes beyond the concrete calldata are symbolic reads of the calldata array
    if stop > len(values):
        assert all(p.symbolic for p in parts[len(values) - start:])


def test_install_rebinds_every_solver_site(monkeypatch):
    ns, _ = _fresh(monkeypatch, cpu=True)
    integration.install()
    gs = integration.gpu_solver_class()
    assert ns.calldata.Solver is gs and ns.summary.Solver is gs and ns.summary_core.Solver is gs
    import sys

    assert sys.modules["mythril.support.model"].Optimize is integration.gpu_optimize_class()
    assert issubclass(gs, ns.Solver) and not issubclass(gs, ns.Optimize)
    # Solver's own surface still reaches z3
    s = gs()
    s.add(ns.Bool(z3.BitVec("x", 256) == z3.BitVecVal(3, 256)))
    s.reset()
    assert s.raw.assertions() == []


def test_summary_checks_through_gpu_solver(monkeypatch):
    """summary.py:114-117 (state constraints under the summary's conditions) and
    core.py:222-227 (two storage keys alias, with the keccak conditions): SAT sets are GPU
    answers, each counted once; a contradiction falls back to z3."""
    ns, _ = _fresh(monkeypatch, cpu=True)
    integration.install()
    B = ns.Bool
    x = z3.BitVec("storage_key_1", 256)
    ms = _stats()
    ms.query_count = 0
    assert ns.summary.summary_applies([B(z3.ULT(x, z3.BitVecVal(100, 256))), B(x != z3.BitVecVal(0, 256))], 2000)
    k1 = ns.BitVec(x)
    k2 = ns.BitVec(z3.BitVec("storage_key_2", 256))
    assert ns.summary_core.keys_may_alias(k1, k2)
    assert SolverStatistics().gpu_sat == 2
    assert not ns.summary.summary_applies([B(z3.ULT(x, z3.BitVecVal(5, 256))),
                                           B(z3.ULT(z3.BitVecVal(9, 256), x))], 2000)
    assert ms.query_count == 3 and SolverStatistics().gpu_sat == 2


@pytest.mark.gpu
def test_gpu_calldata_slice_loop_through_gpu_solver(monkeypatch, engine):
    ns, _ = _fresh(monkeypatch, cpu=False)
    values = [(i * 91 + 3) & 0xFF for i in range(40)]
    _run_slice_case(ns, 4, 36, values)
    ns2, _ = _fresh(monkeypatch, cpu=False)
    _run_slice_case(ns2, 30, 44, values)
