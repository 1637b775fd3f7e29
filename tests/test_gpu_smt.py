"""GPU: the drop-in SMT facade, mirroring the reference's own SMT tests.

* tests/laser/smt/model_test.py:1-57 (decls / __getitem__ / eval().as_long());
* tests/laser/keccak_tests.py:8-146 — SAT/UNSAT labels.  Soundness bar: the GPU never says
  sat on an UNSAT-labelled set (every witness is re-checked on the host anyway).  On
  SAT-labelled sets the GPU answers sat where a witness is reachable by the generator;
  otherwise it reports unknown (z3 is absent here; with z3 the query would fall back).
* tests/laser/state/calldata_test.py:27-90 term shapes (calldata size bounds).
"""

import pytest

from mythril_amd.exceptions import SolverTimeOutException, UnsatError
from mythril_amd.keccak_manager import keccak_function_manager as kfm
from mythril_amd.smt import (ULT, And, Array, If, Not, Optimize, Solver, SolverStatistics,
                             symbol_factory, sat, unknown, unsat)
from mythril_amd.support.model import get_model, get_models

pytestmark = pytest.mark.gpu

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


def _solver_x_eq_2(engine):
    solver = Solver()
    x = BV("x", 256)
    solver.add(x == BVV(2, 256))
    return solver, x


def test_model_decls(engine):
    solver, x = _solver_x_eq_2(engine)
    assert solver.check() == sat
    assert x.raw.decl() in solver.model().decls()


def test_model_get_item(engine):
    solver, x = _solver_x_eq_2(engine)
    assert solver.check() == sat
    assert 2 == solver.model()[x.raw.decl()]


def test_model_as_long(engine):
    solver, x = _solver_x_eq_2(engine)
    assert solver.check() == sat
    assert solver.model().eval(x.raw).as_long() == 2


@pytest.mark.parametrize("i1,i2,expected", [
    (("v", 100, 8), ("v", 101, 8), "unsat"),
    (("v", 100, 8), ("v", 100, 16), "unsat"),
    (("v", 100, 8), ("v", 100, 8), "sat"),
    (("s", "N1", 256), ("s", "N2", 256), "sat"),
    (("v", 100, 256), ("s", "N1", 256), "sat"),
    (("v", 100, 8), ("s", "N1", 256), "unsat"),
])
def test_keccak_basic(engine, i1, i2, expected):
    mk = lambda t: BVV(t[1], t[2]) if t[0] == "v" else BV(t[1], t[2])
    s = Solver()
    kfm.reset()
    o1 = kfm.create_keccak(mk(i1))
    o2 = kfm.create_keccak(mk(i2))
    s.add(kfm.create_conditions())
    s.add(o1 == o2)
    r = s.check()
    if expected == "unsat":
        assert r != sat
    else:
        assert r == sat  # reachable by the generator (equal small/boundary values, seeds)


def test_keccak_symbol_and_val(engine):
    s = Solver()
    kfm.reset()
    n = BV("n", 256)
    o1 = kfm.create_keccak(BVV(100, 256))
    o2 = kfm.create_keccak(n)
    s.add(kfm.create_conditions())
    s.add(o1 == o2)
    s.add(n == BVV(10, 256))
    assert s.check() != sat  # unsat in the reference


def test_keccak_complex_eq(engine):
    kfm.reset()
    s = Solver()
    a, b = BV("a", 160), BV("b", 160)
    o1 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(a))
    o2 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(b))
    s.add(kfm.create_conditions())
    s.add(o1 == o2)
    s.add(a != b)
    assert s.check() != sat  # unsat in the reference


def test_keccak_complex_eq2(engine):
    kfm.reset()
    s = Solver()
    a, b = BV("a", 160), BV("b", 160)
    o1 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(a))
    o2 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(b))
    s.add(kfm.create_conditions())
    s.add(o1 == o2)
    assert s.check() == sat
    m = s.model()
    assert m.eval(a.raw).as_long() == m.eval(b.raw).as_long()


def test_keccak_simple_number(engine):
    kfm.reset()
    s = Solver()
    o = kfm.create_keccak(BV("a", 160))
    s.add(kfm.create_conditions())
    s.add(BVV(10, 256) == o)
    assert s.check() != sat  # unsat in the reference


def test_keccak_other_num(engine):
    kfm.reset()
    s = Solver()
    a, b = BV("a", 160), BV("b", 256)
    o = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(a))
    s.add(kfm.create_conditions())
    s.add(b == o)
    r = s.check()
    assert r != unsat  # sat in the reference; b must equal a computed hash -> may be unknown


def test_mapping_slot_witness_evaluates(engine):
    """balances[keccak(caller || slot)] style query: model.eval reproduces the kernel."""
    kfm.reset()
    s = Solver()
    caller = BV("sender_1", 256)
    slot = kfm.create_keccak(symbol_factory.BitVecVal(0, 256) + caller)  # 256-bit input
    storage = Array("Storage0", 256, 256)
    s.add(kfm.create_conditions())
    s.add(storage[slot] == BVV(5, 256))
    s.add(ULT(BVV(3, 256), storage[slot]))
    assert s.check() == sat
    m = s.model()
    assert m.eval(storage[slot].raw).as_long() == 5


def test_calldata_size_bounds(engine):
    # calldata_test.py:27-90 shapes: symbolic calldata[51] == 1 with size == 50 is unsat;
    # the same read with size 60 is sat (If(i <s size, select, 0), calldata.py:233-246)
    cd = Array("1_calldata", 256, 8)
    size = BV("1_calldatasize", 256)
    read = If(BVV(51, 256) < size, cd[BVV(51, 256)], BVV(0, 8))
    s = Solver()
    s.add(read == BVV(1, 8), size == BVV(50, 256))
    assert s.check() != sat
    s = Solver()
    s.add(read == BVV(1, 8), size == BVV(60, 256))
    assert s.check() == sat
    assert s.model().eval(cd[BVV(51, 256)].raw).as_long() == 1


def test_get_model_funnel(engine):
    x = BV("x", 256)
    m = get_model((x == BVV(7, 256),))
    assert m.eval(x.raw).as_long() == 7
    with pytest.raises(UnsatError):
        get_model((False,))
    with pytest.raises(SolverTimeOutException):  # no witness, no z3 -> timeout semantics
        get_model((x == BVV(7, 256), x == BVV(8, 256)))


def test_get_models_batch_and_stats(engine):
    st = SolverStatistics()
    before = st.gpu_sat
    xs = [BV(f"v{i}", 256) for i in range(64)]
    sets = [(ULT(x, BVV(1000, 256)), Not(x == BVV(0, 256))) for x in xs]
    sets.append((xs[0] == BVV(1, 256), xs[0] == BVV(2, 256)))
    models = get_models(sets)
    assert all(m is not None for m in models[:64]) and models[64] is None
    for x, m in zip(xs, models):
        v = m.eval(x.raw).as_long()
        assert 0 < v < 1000
    assert st.gpu_sat - before == 64


def test_optimize_with_objectives_is_not_discharged(engine):
    o = Optimize()
    x = BV("x", 256)
    o.add(ULT(x, BVV(10, 256)))
    o.minimize(x)
    assert o.check() in (unknown, sat)  # objectives always go to z3 (absent here -> unknown)


def test_device_deadline_cuts_a_long_search(engine):
    """Solver timeout as a device deadline (SURVEY §8b threading: the engine bounds its own
    runtime by the passed timeout): a long witness-free search with a 2 ms deadline returns
    within a few ms and reports the cut, so its NOT_FOUND verdicts are not cached; the same
    search without a deadline reports no cut.  Any witness a cut search did report is real."""
    import numpy as np

    import pyoracle as O
    from mythril_amd import ir, synth

    progs = [synth.random_dag_set(9000 + i, plant=False)[0] for i in range(256)]
    db = engine.upload(progs)
    r = engine.check(db, budget=1 << 22, seed=0, flags=ir.FLAG_SHORTCIRCUIT, timeout_ms=2)
    assert r.timed_out
    assert r.kernel_ms < 100.0, r.kernel_ms
    b = ir.Batch(progs)
    for s in np.nonzero(r.found != 0xFFFFFFFF)[0][:8]:
        vals = O.SetView.from_batch(b, int(s)).gen_assignments(np.array([r.found[s]], dtype=np.uint64), 0)[0]
        assert O.SetView.from_batch(b, int(s)).evaluate(vals)
    r2 = engine.check(db, budget=4096, seed=0, flags=ir.FLAG_SHORTCIRCUIT, timeout_ms=60000)
    assert not r2.timed_out
    db.free()
