"""The native hint derivation (libpflower.so pfl_hints, include/pf_lower.h) computes exactly
the hint model of the Python reference (mythril_amd/seed.py:Seeder): the same value for
every variable and the same satisfied-root count, on config-3 DAGs, LASER-shaped corpus
buckets (with caller parents), and random DAGs over every opcode the seeder propagates
through or evaluates (division family, shifts, hash, exp, signed compares, overflow
predicates, ite / or / xor choices)."""

import random

import pytest

import pyoracle as O
from mythril_amd import ir, lower as LW, seed as SD, synth
from mythril_amd import keccak_manager as KM
from mythril_amd.lower import Dag, LoweringError
from mythril_amd.smt import symbol_factory

pytestmark = pytest.mark.skipif(not LW._native(), reason="libpflower.so not built")


def _same(dag):
    want = SD.hints_py(dag)
    got = SD.hints(dag)
    assert got[0] == want[0]
    assert got[1] == want[1]
    return want


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


@pytest.mark.parametrize("dag_id", range(24))
def test_config3_dags_identical(dag_id):
    _same(_synth_dag(dag_id, plant=bool(dag_id & 1)))


def test_corpus_buckets_identical(monkeypatch):
    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))
    from mythril_amd import corpus
    from mythril_amd.smt.independence import buckets
    from mythril_amd.smt.to_dag import TermLowering

    monkeypatch.setattr(SD, "apply_hints", lambda dag: 0)  # compare on the raw lowered DAGs
    c = corpus.build(8, 2, seed=5)
    n = sat = 0
    for q in c.queries[::2]:
        for b in buckets(q.constraints):
            try:
                lo = TermLowering(c.kfm.registry).lower(b)
            except LoweringError:
                continue
            vals, k = _same(lo.dag)
            sat += k == len(set(lo.dag.roots))
            n += 1
    assert n > 50
    assert sat > n // 2  # the hint model itself satisfies most LASER buckets


_W2 = [ir.W_ADD, ir.W_SUB, ir.W_MUL, ir.W_UDIV, ir.W_UREM, ir.W_SDIV, ir.W_SREM, ir.W_SMOD,
       ir.W_AND, ir.W_OR, ir.W_XOR, ir.W_SHL, ir.W_LSHR, ir.W_ASHR, ir.W_EXP]
_CMP = [ir.B_EQ, ir.B_ULT, ir.B_ULE, ir.B_SLT, ir.B_SLE]


def _interesting(rng, w):
    m = ir.mask(w)
    return rng.choice([0, 1, 2, 3, 7, 8, 32, w - 1, w, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1,
                       rng.getrandbits(w), rng.getrandbits(min(w, 16)), 0xDEADBEEF & m]) & m


def _random_dag(seed):
    rng = random.Random(seed)
    dag = Dag()
    widths = [8, 64, 256]
    ws = {w: [] for w in widths}
    for i in range(rng.randint(2, 6)):
        w = rng.choice(widths)
        ws[w].append(dag.var(f"v{i}", w, parent=rng.choice([None, rng.getrandbits(w)])))
    bv = dag.var("flag", 1, kind=ir.VK_BOOL)
    for w in widths:
        if not ws[w]:
            ws[w].append(dag.op(ir.W_MOV, w, ws[256][0]) if ws[256] and w == 256 else
                         dag.var(f"f{w}", w))
    bools = [bv]

    def pick(w):
        return rng.choice(ws[w]) if rng.random() < 0.7 else dag.const(_interesting(rng, w), w)

    for _ in range(rng.randint(4, 24)):
        w = rng.choice(widths)
        r = rng.random()
        if r < 0.45:
            op = rng.choice(_W2)
            b = pick(w)
            if op in (ir.W_SHL, ir.W_LSHR, ir.W_ASHR) and rng.random() < 0.7:
                b = dag.const(rng.randrange(0, w + 3), w)
            ws[w].append(dag.op(op, w, rng.choice(ws[w]), b))
        elif r < 0.55:
            ws[w].append(dag.op(rng.choice([ir.W_NOT, ir.W_NEG]), w, rng.choice(ws[w])))
        elif r < 0.65 and w > 8:
            lo = rng.randrange(0, w - 8)
            ws[8].append(dag.op(ir.W_EXTRACT, 8, rng.choice(ws[w]), aux=lo))
        elif r < 0.72 and w == 64:
            ws[256].append(dag.op(rng.choice([ir.W_MOV, ir.W_SEXT]), 256, rng.choice(ws[64]),
                                  aux=64))
        elif r < 0.8 and w == 64:
            hi, lo = rng.choice(ws[8]), rng.choice(ws[8])
            c = dag.op(ir.W_CONCAT, 16, hi, lo, aux=8)
            ws[64].append(dag.op(ir.W_MOV, 64, c))
        elif r < 0.9:
            ws[w].append(dag.op(ir.W_ITE, w, rng.choice(bools), rng.choice(ws[w]), pick(w)))
        else:
            ws[256].append(dag.op(ir.W_HASH, 256, rng.choice(ws[256]), aux=rng.getrandbits(32)))
        # one Bool fact per step
        r = rng.random()
        w = rng.choice(widths)
        if r < 0.6:
            x = rng.choice(ws[w])
            y = dag.const(_interesting(rng, w), w) if rng.random() < 0.6 else rng.choice(ws[w])
            if rng.random() < 0.5:
                x, y = y, x
            bools.append(dag.op(rng.choice(_CMP), w, x, y))
        elif r < 0.7:
            bools.append(dag.op(rng.choice([ir.B_UADD_NOOVF, ir.B_UMUL_NOOVF]), w,
                                rng.choice(ws[w]), pick(w)))
        elif len(bools) >= 2:
            op = rng.choice([ir.B_AND, ir.B_OR, ir.B_XOR, ir.B_NOT, ir.B_ITE])
            if op == ir.B_NOT:
                bools.append(dag.op(op, 1, rng.choice(bools)))
            elif op == ir.B_ITE:
                bools.append(dag.op(op, 1, rng.choice(bools), rng.choice(bools), rng.choice(bools)))
            else:
                bools.append(dag.op(op, 1, rng.choice(bools), rng.choice(bools)))
    for b in rng.sample(bools[1:] or bools, k=min(len(bools) - 1 or 1, rng.randint(1, 6))):
        dag.assert_(b)
    if rng.random() < 0.3:
        dag.assert_(dag.op(ir.B_NOT, 1, rng.choice(bools)))
    return dag


@pytest.mark.parametrize("chunk", range(8))
def test_random_dags_identical(chunk):
    n = 0
    for s in range(chunk * 60, chunk * 60 + 60):
        dag = _random_dag(s)
        if not dag.roots or not dag.vars:
            continue
        _same(dag)
        n += 1
    assert n > 40


def test_ite_chain_and_actor_choice():
    """The LASER shapes the seeder exists for: a calldata byte ite-chain read, an actor
    disjunction, and a keccak congruence (ite / or / hash)."""
    dag = Dag()
    size = dag.var("calldatasize", 256)
    cd = [dag.var(f"cd{i}", 8) for i in range(4)]
    bytes_ = [dag.op(ir.W_ITE, 8, dag.op(ir.B_ULT, 256, dag.const(i, 256), size), cd[i], dag.const(0, 8))
              for i in range(4)]
    word = bytes_[0]
    for i in range(1, 4):
        word = dag.op(ir.W_CONCAT, 8 * (i + 1), word, bytes_[i], aux=8)
    dag.assert_(dag.op(ir.B_EQ, 32, word, dag.const(0xA9059CBB, 32)))
    caller = dag.var("caller", 256)
    eqs = [dag.op(ir.B_EQ, 256, caller, dag.const(a, 256)) for a in (0xAFFE, 0xDEADBEEF, 0xCAFE)]
    dag.assert_(dag.op(ir.B_OR, 1, dag.op(ir.B_OR, 1, eqs[0], eqs[1]), eqs[2]))
    k1 = dag.var("k1", 256)
    dag.assert_(dag.op(ir.B_EQ, 256, dag.op(ir.W_HASH, 256, caller, aux=3),
                       dag.op(ir.W_HASH, 256, k1, aux=3)))
    vals, n_sat = _same(dag)
    assert n_sat == 3
    assert vals[dag.vars.index(next(v for v in dag.vars if v.name == "k1"))] == 0xAFFE
