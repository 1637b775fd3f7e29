"""CPU: the SMT-LIB2 reader (--solver-log dumps, mythril/support/model.py:46-57)."""

import random

import pyoracle as O

from mythril_amd import ir
from mythril_amd.lower import lower
from mythril_amd.smt import ULT, Array, Concat, Function, If, Optimize, symbol_factory
from mythril_amd.smt import terms as T
from mythril_amd.smt.interp import Witness
from mythril_amd.smt.to_dag import TermLowering, UFRegistry
from mythril_amd.smtlib import read_query

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym

Z3_STYLE = """
(declare-fun |1_calldatasize| () (_ BitVec 256))
(declare-fun |1_calldata| () (Array (_ BitVec 256) (_ BitVec 8)))
(declare-fun sender_1 () (_ BitVec 256))
(declare-fun |keccak256_512| ((_ BitVec 512)) (_ BitVec 256))
(declare-fun |keccak256_512-1| ((_ BitVec 256)) (_ BitVec 512))
(declare-fun flag () Bool)
(assert (let ((a!1 (concat (ite (bvslt #x0000000000000000000000000000000000000000000000000000000000000000
                                       |1_calldatasize|)
                                (select |1_calldata| #x0000000000000000000000000000000000000000000000000000000000000000)
                                #x00)
                           (ite (bvslt (_ bv1 256) |1_calldatasize|)
                                (select |1_calldata| (_ bv1 256))
                                #x00))))
  (= ((_ extract 15 8) a!1) #xa9)))
(assert (or (= sender_1 #x000000000000000000000000deadbeefdeadbeefdeadbeefdeadbeefdeadbeef) flag))
(assert (bvuge |1_calldatasize| (_ bv4 256)))
(assert (= (|keccak256_512-1| (|keccak256_512| (concat sender_1 (_ bv0 256)))) (concat sender_1 (_ bv0 256))))
(assert (not (= ((_ zero_extend 248) ((_ extract 7 0) sender_1)) (_ bv7 256))))
(assert (distinct ((_ sign_extend 8) #xff) #x00ff))
(minimize |1_calldatasize|)
(check-sat)
"""


def test_reads_z3_printer_forms():
    q = read_query(Z3_STYLE)
    assert len(q.assertions) == 6 and len(q.minimize) == 1 and not q.objective_free
    assert q.assertions[5] is T.TRUE  # folded: sign_extend(#xff) = #xffff != #x00ff
    lo = TermLowering(UFRegistry()).lower(q.assertions)
    prog = lower(lo.dag)
    assert prog.code[-1].op == ir.END


def test_roundtrip_through_sexpr_preserves_semantics():
    """Facade terms -> Optimize.sexpr() -> reader -> lowered programs agree on random models."""
    rng = random.Random(5)
    x, y, s = BV("x", 256), BV("y", 256), BV("1_calldatasize", 256)
    cd = Array("1_calldata", 256, 8)
    f = Function("keccak256_256", [256], 256)
    o = Optimize()
    o.add(ULT(x + y * BVV(3, 256), BVV(1 << 200, 256)))
    o.add(If(x > y, x - y, y - x) != BVV(0, 256))
    o.add(Concat(cd[BVV(0, 256)], cd[BVV(1, 256)]) == BVV(0xA9B0, 16))
    o.add(ULT(s, BVV(100, 256)))
    o.add(f(x) != f(y))
    text = o.sexpr()
    q = read_query(text)
    assert len(q.assertions) == 5
    reg = UFRegistry()
    lo_a = TermLowering(reg).lower(list(o.constraints))
    lo_b = TermLowering(reg).lower(q.assertions)
    pa, pb = lower(lo_a.dag), lower(lo_b.dag)
    sva = O.SetView.from_batch(ir.Batch([pa]), 0)
    svb = O.SetView.from_batch(ir.Batch([pb]), 0)
    names_a = [v.name for v in pa.vars]
    names_b = [v.name for v in pb.vars]
    assert sorted(names_a) == sorted(names_b)
    for _ in range(50):
        vals = {n: rng.getrandbits(w.width) for n, w in zip(names_a, pa.vars)}
        if rng.random() < 0.3:
            vals["1_calldata[0]"] = 0xA9
            vals["1_calldata[1]"] = 0xB0
        va = [vals[n] for n in names_a]
        vb = [vals[n] for n in names_b]
        assert sva.evaluate(va) == svb.evaluate(vb)
        wa = Witness(lo_a, va, reg)
        assert all(wa.ev(c) for c in o.constraints) == sva.evaluate(va)
