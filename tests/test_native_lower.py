"""The native lowering (libpflower.so, include/pf_lower.h) emits exactly the program of the
Python reference (mythril_amd/lower.py:lower_py): same instructions, registers, spill slots
and constant pool, or the same LoweringError — on config-3 DAGs, LASER-shaped corpus buckets
(with hint models), register-pressure DAGs that spill, and wide (chunked) sets."""

import numpy as np
import pytest

import pyoracle as O
from mythril_amd import ir, lower as LW, synth
from mythril_amd import keccak_manager as KM
from mythril_amd.lower import Dag, LoweringError
from mythril_amd.smt import symbol_factory

pytestmark = pytest.mark.skipif(not LW._native(), reason="libpflower.so not built")


def _words(prog):
    if isinstance(prog, ir.PackedProgram):
        w = prog.words.copy()
    else:
        w = np.array([ins.words() for ins in prog.code], dtype=np.uint32).reshape(-1, 4)
    w[:, 3] = 0
    return w


def _same1(dag, seed, nw):
    try:
        want = LW.lower_py(dag, seed=seed, nw=nw)
    except LoweringError as e:
        with pytest.raises(LoweringError):
            LW.lower(dag, seed=seed, nw=nw)
        return str(e)
    got = LW.lower(dag, seed=seed, nw=nw)
    assert isinstance(got, ir.PackedProgram)
    assert np.array_equal(_words(got), _words(want))
    assert got.consts == want.consts
    assert [v.name for v in got.vars] == [v.name for v in want.vars]
    return None


def _same(dag, seed=0):
    """Native == Python at both register counts the engine uses, and the default policy:
    the narrow program unless it does not fit, or is spill-heavy and the 15-register one at
    least halves its spill code."""
    e_narrow = _same1(dag, seed, ir.NW_NARROW)
    e_wide = _same1(dag, seed, ir.NW)
    if e_wide is not None:
        return e_wide
    got = LW.lower(dag, seed=seed)
    narrow = None if e_narrow is not None else LW.lower_py(dag, seed=seed, nw=ir.NW_NARROW)
    wide = LW.lower_py(dag, seed=seed, nw=ir.NW)
    if narrow is not None and (not LW._spill_heavy(narrow)
                               or 2 * LW._spill_code(wide)[1] > LW._spill_code(narrow)[1]):
        assert np.array_equal(_words(got), _words(narrow))
    else:
        assert np.array_equal(_words(got), _words(wide))
    return None


def _synth_dag(dag_id, **kw):
    got = {}
    orig = synth.lower

    def cap(dag, **k):
        got["dag"] = dag
        return orig(dag, **k)

    synth.lower = cap
    try:
        synth.random_dag_set(dag_id, **kw)
    finally:
        synth.lower = orig
    return got["dag"]


@pytest.mark.parametrize("dag_id", range(40))
def test_config3_dags_identical(dag_id):
    assert _same(_synth_dag(dag_id)) is None


def test_corpus_buckets_identical(monkeypatch):
    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))
    from mythril_amd import corpus, seed
    from mythril_amd.smt.independence import buckets
    from mythril_amd.smt.to_dag import TermLowering

    c = corpus.build(8, 2, seed=3)
    n = 0
    for q in c.queries[::3]:
        for b in buckets(q.constraints):
            try:
                lo = TermLowering(c.kfm.registry).lower(b)
            except LoweringError:
                continue
            seed.apply_hints(lo.dag)
            _same(lo.dag, seed=n)
            n += 1
    assert n > 50


def _pressure(n_live):
    dag = Dag()
    x, y = dag.var("x", 256), dag.var("y", 256)
    prods = [dag.op(ir.W_MUL, 256, x, dag.op(ir.W_ADD, 256, y, dag.const(k + 1, 256))) for k in range(n_live)]
    acc = prods[0]
    for p in prods[1:]:
        acc = dag.op(ir.W_XOR, 256, acc, p)
    for p in prods:
        dag.assert_(dag.op(ir.B_ULT, 256, p, acc))
    return dag


@pytest.mark.parametrize("n_live", [4, 14, 15, 16, 24, 40, 90])
def test_pressure_and_spills_identical(n_live):
    _same(_pressure(n_live))


def test_native_program_runs_like_python_on_the_oracle():
    dag = _synth_dag(7, plant=True)
    prog = LW.lower(dag, seed=5)
    ref = LW.lower_py(dag, seed=5, nw=ir.NW_NARROW)
    a = O.SetView.from_batch(ir.Batch([prog]), 0).check(512, 9)
    b = O.SetView.from_batch(ir.Batch([ref]), 0).check(512, 9)
    assert a == b
    assert np.array_equal(ir.Batch([prog]).code, ir.Batch([ref]).code)


@pytest.mark.parametrize("n_vars,n_pairs", [(30, 36), (40, 36), (40, 30)])
def test_slot_steal_edge_identical(n_vars, n_pairs):
    """The fill-at-last-use slot steal: native and Python agree — the same
    program, or the same LoweringError — at both register counts."""
    from test_lowering import _slot_steal_dag

    _same(_slot_steal_dag(n_vars, n_pairs))
