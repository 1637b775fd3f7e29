"""The ``Power`` UF (symbolic EXP): interpretation by construction that satisfies the
conditions of mythril/laser/ethereum/function_managers/exponent_function_manager.py:40-68 —
``Power(b, e) >s 0`` per symbolic EXP, the 32 table entries ``Power(256, i) = 256^i``,
``Power(256, e %u 32) == Power(256, e)`` for base 256, ``Power(c1, c2) = c1^c2`` for a
concrete EXP — so symbolic-EXP queries (e >= 32 included) can be discharged.

The queries are built with the facade exactly as the manager builds them; a GPU witness must
re-check under those very conditions (host evaluator, mythril_amd/smt/interp.py).  CPU: the
host pipeline on the C oracle (tests/oracle_engine.py); GPU: the same on the MI355X.
"""

import pytest

import oracle_engine
from mythril_amd.smt import (ULT, UGE, And, Function, K, URem, UDiv, symbol_factory)
from mythril_amd.smt import gpu_check
from mythril_amd.smt import terms as T

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


class ExponentManager:
    """Restatement of ExponentFunctionManager.create_condition (exponent_function_manager.py:
    40-68) over the facade: the conditions a symbolic EXP appends to the path."""

    def __init__(self):
        self.power = Function("Power", [256, 256], 256)
        n256 = BVV(256, 256)
        self.concrete_constraints = And(*[self.power(n256, BVV(i, 256)) == BVV(256 ** i, 256)
                                          for i in range(32)])

    def create_condition(self, base, exponent):
        exp = self.power(base, exponent)
        if not base.symbolic and not exponent.symbolic:
            c = BVV(pow(base.value, exponent.value, 2 ** 256), 256)
            return c, c == exp
        cond = And(exp > BVV(0, 256), self.concrete_constraints)   # signed >, bitvec.py:165
        if base.value == 256:
            cond = And(cond, self.power(base, URem(exponent, BVV(32, 256))) == exp)
        return exp, cond


def _queries():
    em = ExponentManager()
    e = BV("e", 256)
    p, cond = em.create_condition(BVV(256, 256), e)
    # base 256, exponent >= 32: real modexp would make Power 0 here (unsat under >s 0)
    q_e32 = [cond, UGE(e, BVV(32, 256)), ULT(e, BVV(100, 256)), p == BVV(1 << 16, 256)]
    # symbolic base: Power is a free positive value, consistent by argument value
    b = BV("b", 256)
    pb, condb = em.create_condition(b, e)
    pb2, condb2 = em.create_condition(b, e)
    q_base = [condb, condb2, ULT(BVV(10, 256), b), pb == pb2, ULT(pb, BVV(1 << 200, 256))]
    # a concrete EXP next to a symbolic one (functional consistency with the concrete fact)
    c, condc = em.create_condition(BVV(3, 256), BVV(5, 256))
    q_mix = [cond, condc, c == BVV(243, 256), ULT(e, BVV(40, 256)), p == BVV(256 ** 7, 256)]
    return {"base256_e_ge_32": q_e32, "symbolic_base": q_base, "mixed_concrete": q_mix}


def _flag_array_query():
    """flag_array.sol (tests/testdata/input_contracts/flag_array.sol): ``bool[4096] _flags``
    packed 32 per slot, ``_flags[1234] = true`` in the constructor, ``extractMoney(idx)``
    requires ``idx < 4096`` and ``_flags[idx]``.  The read is Solidity's packed-bool load:
    ``(sload(idx / 32) / 256^(idx % 32)) & 0xff != 0`` with EXP -> Power
    (instructions.py:625-639).  Storage after construction: slot 38 = 1 << (8 * 18).
    Expected witness (tests/integration_tests/analysis_tests.py:19): idx = 1234."""
    em = ExponentManager()
    idx = BV("idx", 256)
    storage = K(256, 256, 0)
    storage[BVV(1234 // 32, 256)] = BVV(1 << (8 * (1234 % 32)), 256)
    exp, cond = em.create_condition(BVV(256, 256), URem(idx, BVV(32, 256)))
    word = UDiv(storage[UDiv(idx, BVV(32, 256))], exp)
    return [ULT(idx, BVV(4096, 256)), cond, (word & BVV(0xFF, 256)) != BVV(0, 256)], idx


def _check(sets):
    return gpu_check.check_sets([[c.raw for c in cs] for cs in sets])


def _assert_witnesses(models, queries):
    for (name, q), m in zip(queries.items(), models):
        assert m is not None, name
        # the witness re-checks under the manager's own conditions
        assert all(bool(m.eval(c.raw)) for c in q), name


def test_power_interpretation_cpu(monkeypatch):
    oracle_engine.install(monkeypatch)
    qs = _queries()
    models = _check(list(qs.values()))
    _assert_witnesses(models, qs)
    e = models[0].eval(BV("e", 256).raw).as_long()
    assert 32 <= e < 100 and e % 32 == 2
    assert models[2].eval(BV("e", 256).raw).as_long() % 32 == 7


def test_power_bucket_couples_table_constraints():
    """All constraints applying Power share one independence bucket (the concrete table
    entries included), so the interpretation sees every concrete fact."""
    from mythril_amd.smt.independence import buckets

    q = _queries()["mixed_concrete"]
    bks = buckets([c.raw for c in q])
    power_buckets = [b for b in bks if any("Power" in repr(c) for c in b)]
    assert len(power_buckets) == 1


def test_flag_array_witness_cpu(monkeypatch):
    oracle_engine.install(monkeypatch)
    q, idx = _flag_array_query()
    m = _check([q])[0]
    assert m is not None
    assert m.eval(idx.raw).as_long() == 1234
    assert all(bool(m.eval(c.raw)) for c in q)


@pytest.mark.gpu
def test_power_interpretation_gpu(engine):
    gpu_check.reset_cache()
    qs = _queries()
    _assert_witnesses(_check(list(qs.values())), qs)
    q, idx = _flag_array_query()
    m = _check([q])[0]
    assert m is not None and m.eval(idx.raw).as_long() == 1234
    assert all(bool(m.eval(c.raw)) for c in q)
