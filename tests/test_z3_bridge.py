"""mythril_amd/smt/z3_bridge.py — the z3 back end of the z3-free facade — driven through the
z3 stand-in (tests/fake_z3.py; z3-solver is not installed here).  The
converter's output read back by the live-analysis walker (mythril_amd/z3_terms.py) must be
the same hash-consed term (a round trip through z3's AST), for every operator the lowering
takes; ``check`` builds an Optimize with the objectives and maps the stand-in's ``unknown``.
Parity with real z3 is unpinned (no z3 here)."""

import pytest

import fake_z3
from mythril_amd.smt import terms as T
from mythril_amd.smt import z3_bridge
from mythril_amd.z3_terms import Z3Converter


@pytest.fixture
def bridge(monkeypatch):
    monkeypatch.setattr(z3_bridge, "z3", fake_z3)
    monkeypatch.setattr(z3_bridge, "HAVE_Z3", True)
    return z3_bridge


def _terms():
    x, y = T.var("x", 256), T.var("y", 256)
    b = T.boolvar("flag")
    arr = T.array("Storage", 256, 256)
    st = T.store(T.const_array(256, T.const(0, 256)), x, y)
    f = T.apply("keccak256_512", 256, T.concat(x, T.const(1, 256)))
    out = [T.binop(op, x, y) for op in ("bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem",
                                        "bvsmod", "bvand", "bvor", "bvxor", "bvshl", "bvlshr", "bvashr")]
    out += [T.bvnot(x), T.bvneg(y), T.extract(159, 0, x), T.zero_extend(8, T.extract(7, 0, y)),
            T.concat(T.extract(7, 0, x), T.extract(7, 0, y)), T.ite(b, x, y),
            T.select(arr, x), T.select(st, T.const(3, 256)), f]
    bools = [T.cmp(op, x, y) for op in ("bvult", "bvule", "bvslt", "bvsle", "bvumul_noovfl")]
    bools += [T.eq(x, y), T.and_(b, T.cmp("bvult", x, y)), T.or_(b, T.not_(b)), T.xor(b, T.eq(x, y)),
              T.Term("iff", T.BOOL, (b, T.eq(x, y)))]
    return out, bools


def test_converter_round_trips_through_the_walker(bridge):
    conv = bridge.Converter()
    back = Z3Converter(fake_z3)
    bvs, bools = _terms()
    for t in bvs + bools:
        z = conv(t)
        assert back.term(z) is t, T.to_sexpr(t)[:200]


def test_converter_rejects_what_z3_lacks(bridge):
    with pytest.raises(ValueError):
        bridge.Converter()(T.binop("bvexp", T.var("a", 256), T.var("b", 256)))


def test_check_builds_the_optimize_and_maps_unknown(bridge):
    x = T.var("call_value1", 256)
    r, model, s = bridge.check([T.cmp("bvult", x, T.const(9, 256))], minimize=[x], timeout_ms=250)
    assert r == fake_z3.unknown and model is None
    assert len(s.assertions()) == 1 and s._objectives[0][0] == "minimize" and s.timeout == 250
