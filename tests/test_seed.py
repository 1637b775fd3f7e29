"""Host logic of the discharge pipeline: hint models (mythril_amd/seed.py), independence
buckets (mythril_amd/smt/independence.py, after mythril/laser/smt/solver/independence_solver.py),
the LASER-shaped corpus (mythril_amd/corpus.py) and — with the C oracle standing in for the
GPU — the end-to-end hit rate on that corpus."""

import pytest

import discharge_oracle as D
from mythril_amd import corpus, seed
from mythril_amd.keccak_manager import KeccakFunctionManager
from mythril_amd.smt import (UGE, ULT, Array, Concat, If, Not, Or, UDiv, symbol_factory)
from mythril_amd.smt import terms as T
from mythril_amd.smt.expr import LShR
from mythril_amd.smt.independence import buckets
from mythril_amd.smt.to_dag import ACTORS, TermLowering, UFRegistry

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


@pytest.fixture(scope="module", autouse=True)
def _host_keccak():
    D.host_keccak()


def _hint_satisfies(cs):
    lo = TermLowering(UFRegistry()).lower([c.raw for c in cs])
    n_ok = seed.apply_hints(lo.dag)
    return n_ok == len(set(lo.dag.roots)), {v.name: v.parent for v in lo.dag.vars}


def _word(cd, size, off):
    return Concat([If(BVV(off + i, 256) < size, cd[BVV(off + i, 256)], BVV(0, 8)) for i in range(32)])


@pytest.mark.parametrize("div_style", [False, True])
def test_dispatcher_path_hint(div_style):
    cd, size = Array("1_calldata", 256, 8), BV("1_calldatasize", 256)
    w0 = _word(cd, size, 0)
    sel = (UDiv(w0, BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)) if div_style else LShR(w0, BVV(224, 256))
    caller, val = BV("sender_1", 256), BV("call_value1", 256)
    cs = [Or(*[caller == BVV(a, 256) for a in ACTORS]),
          UGE(Array("balance", 256, 256)[caller], val),
          Not(ULT(size, BVV(4, 256))),
          Not(sel == BVV(0x12345678, 256)),
          sel == BVV(0xA9059CBB, 256),
          If(val == BVV(0, 256), BVV(1, 256), BVV(0, 256)) != BVV(0, 256),
          ULT(_word(cd, size, 4), BVV(1000, 256)),
          Not(_word(cd, size, 36) == BVV(0, 256)),
          caller == BVV(ACTORS[1], 256)]
    ok, vals = _hint_satisfies(cs)
    assert ok
    assert vals["sender_1"] == ACTORS[1]
    assert [vals[f"1_calldata[{i}]"] for i in range(4)] == [0xA9, 0x05, 0x9C, 0xBB]


def test_signed_and_unsigned_ranges_hint():
    x, y = BV("x", 256), BV("y", 256)
    ok, vals = _hint_satisfies([x > BVV(5, 256), x < BVV(9, 256), ULT(BVV(100, 256), y),
                                ULT(y, BVV(200, 256))])
    assert ok and 5 < vals["x"] < 9 and 100 < vals["y"] < 200


def test_mapping_slot_equality_by_congruence():
    # approved[keccak(caller . 1)] written for an address argument, read for the caller
    kfm = KeccakFunctionManager(UFRegistry())
    cd, size = Array("1_calldata", 256, 8), BV("1_calldatasize", 256)
    arg = _word(cd, size, 4) & BVV((1 << 160) - 1, 256)
    caller = BV("sender_2", 256)
    k1 = kfm.create_keccak(Concat(arg, BVV(1, 256)))
    k2 = kfm.create_keccak(Concat(caller & BVV((1 << 160) - 1, 256), BVV(1, 256)))
    st = T.store(T.const_array(256, T.const(0, 256)), k1.raw, T.const(1, 256))
    read = T.select(st, k2.raw)
    cs = [Or(*[caller == BVV(a, 256) for a in ACTORS]).raw, T.eq(read, T.const(1, 256)),
          kfm.create_conditions().raw]
    lo = TermLowering(kfm.registry).lower(cs)
    assert seed.apply_hints(lo.dag) == len(set(lo.dag.roots))


def test_buckets_partition():
    a, b, c = BV("a", 256), BV("b", 256), BV("c", 256)
    arr = Array("Storage", 256, 256)
    cs = [(a == BVV(1, 256)).raw, ULT(b, c).raw, (arr[a] == BVV(2, 256)).raw,
          (arr[BVV(7, 256)] == BVV(3, 256)).raw, ULT(c, BVV(9, 256)).raw]
    bk = buckets(cs)
    as_sets = sorted(sorted(T.to_sexpr(x) for x in g) for g in bk)
    assert len(bk) == 2                       # {a, Storage} and {b, c}
    assert sum(len(g) for g in bk) == len(cs)
    assert any(len(g) == 3 for g in as_sets) and any(len(g) == 2 for g in as_sets)


def test_corpus_labels_hold():
    c = corpus.build(12, 2, seed=7)
    n_sat = corpus.validate(c)                # every planted label re-evaluated
    assert n_sat > 50 and len(c.queries) > n_sat
    origins = {q.origin.split("#")[0] for q in c.queries}
    assert {"token", "BECToken", "EtherStore", "Rubixi", "KillBilly", "WalletLibrary"} <= origins


def test_corpus_discharge_with_oracle_search():
    """The whole pipeline (buckets -> lowering -> hints -> generated candidates) with the
    C oracle doing the search: most planted-SAT queries are discharged."""
    c = corpus.build(6, 2, seed=11)
    res, _ = D.discharge(c.queries, c.kfm.registry, budget=256)
    planted = [r for r, q in zip(res, c.queries) if q.label == "sat"]
    assert sum(1 for r in planted if r) >= 0.8 * len(planted)
