"""CPU: the mythril.laser.smt mirror — operator semantics, constant folding, lowering, and the
host model evaluator agreeing with the bytecode (oracle) on random assignments."""

import random

import numpy as np
import pyoracle as O
import pytest

from mythril_amd import ir
from mythril_amd.lower import lower
from mythril_amd.smt import (UGE, UGT, ULE, ULT, And, Array, BVAddNoOverflow, BVMulNoOverflow,
                             BVSubNoUnderflow, Concat, Extract, Function, If, K, LShR, Not, Or,
                             SRem, UDiv, URem, symbol_factory)
from mythril_amd.smt import terms as T
from mythril_amd.smt.interp import Witness, uf_hash
from mythril_amd.smt.to_dag import KeccakSpec, TermLowering, UFRegistry

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


def test_signed_operators_match_reference_semantics():
    # bitvec.py:138-180: < > <= >= are signed; / is sdiv; >> is ashr
    a, b = BVV(-1, 256), BVV(1, 256)
    assert (a < b).is_true and (b > a).is_true and (a <= b).is_true and (b >= a).is_true
    assert ULT(b, a).is_true and UGT(a, b).is_true
    assert (BVV(-7, 256) / BVV(2, 256)).value == (-3) % (1 << 256)
    assert (BVV(-8, 256) >> BVV(1, 256)).value == (-4) % (1 << 256)
    assert LShR(BVV(-8, 256), BVV(1, 256)).value == ((1 << 256) - 8) >> 1
    assert UDiv(BVV(7, 256), BVV(0, 256)).value == (1 << 256) - 1
    assert URem(BVV(7, 256), BVV(0, 256)).value == 7
    assert SRem(BVV(-7, 256), BVV(2, 256)).value == (-1) % (1 << 256)


def test_ule_uge_are_or_forms():
    x, y = BV("x", 256), BV("y", 256)
    assert ULE(x, y).raw.op == "or" and UGE(x, y).raw.op == "or"


def test_padded_equality():
    # bitvec.py:16-22: == between different widths zero-pads the narrower operand
    a = Concat(BV("k", 256), BV("s", 256))
    e = (a == BV("z", 256))
    assert e.raw.args[1].op == "zero_extend" and e.raw.args[1].width == 512
    assert (BVV(100, 8) == BVV(100, 16)).is_true


def test_noovf_predicates_fold():
    m = (1 << 256) - 1
    assert BVAddNoOverflow(BVV(m, 256), BVV(1, 256), False).is_false
    assert BVAddNoOverflow(BVV(m - 1, 256), BVV(1, 256), False).is_true
    assert BVMulNoOverflow(BVV(1 << 128, 256), BVV(1 << 128, 256), False).is_false
    assert BVSubNoUnderflow(BVV(3, 256), BVV(4, 256), False).is_false


@pytest.mark.parametrize("seed", range(6))
def test_constant_folding_matches_oracle(seed):
    rng = random.Random(seed)
    ops = [("bvadd", O.bvadd), ("bvsub", O.bvsub), ("bvmul", O.bvmul), ("bvudiv", O.bvudiv),
           ("bvurem", O.bvurem), ("bvsdiv", O.bvsdiv), ("bvsrem", O.bvsrem), ("bvsmod", O.bvsmod),
           ("bvshl", O.bvshl), ("bvlshr", O.bvlshr), ("bvashr", O.bvashr)]
    for w in (8, 160, 256):
        for _ in range(50):
            a = rng.choice([0, 1, (1 << w) - 1, 1 << (w - 1), rng.getrandbits(w)])
            b = rng.choice([0, 1, 3, w, (1 << w) - 1, rng.getrandbits(w)])
            for name, fn in ops:
                assert T.binop(name, T.const(a, w), T.const(b, w)).val == fn(a, b, w), (name, a, b, w)


def _random_constraints(rng, registry):
    x, y = BV("x", 256), BV("y", 256)
    s = BV("sender_1", 256)
    size = BV("1_calldatasize", 256)
    b = symbol_factory.BoolSym("flag")
    cd = Array("1_calldata", 256, 8)
    st = K(256, 256, 0)
    st[BVV(5, 256)] = x
    st[y] = BVV(9, 256)
    keccak = Function("keccak256_512", [512], 256)
    inv = Function("keccak256_512-1", [256], 512)
    power = Function("Power", [256, 256], 256)
    other = Function("blockhash_x", [256], 256)
    word = Concat([If(BVV(i, 256) < size, cd[BVV(i, 256)], BVV(0, 8)) for i in range(4, 8)])
    key = Concat(x, y)
    h = keccak(key)
    cs = [
        ULT(x, BVV(rng.getrandbits(256), 256)) if rng.random() < 0.5 else (x > y),
        Or(s == BVV(0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 256), b),
        UGE(st[y], BVV(rng.getrandbits(4), 256)),
        Not(word == BVV(rng.getrandbits(32), 32)),
        inv(h) == key,
        ULE(BVV(registry.keccak[512].lo, 256), h),
        URem(h, BVV(64, 256)) == 0,
        cd[x] == cd[BVV(4, 256)],
        Extract(7, 0, other(y)) != BVV(3, 8),
        power(BVV(256, 256), y) > 0,
        BVAddNoOverflow(x, y, False),
        If(b, x, y) != BVV(0, 256),
    ]
    rng.shuffle(cs)
    return [c.raw for c in cs[: rng.randint(4, len(cs))]]


@pytest.mark.parametrize("seed", range(8))
def test_host_model_eval_matches_bytecode(seed):
    """Witness.ev (host Model.eval) == oracle evaluation of the lowered program."""
    rng = random.Random(seed)
    reg = UFRegistry()
    reg.keccak[512] = KeccakSpec(lo=(10 ** 40 - 34534) * ((2 ** 256 - 1) // 10 ** 40))
    reg.keccak[512].concrete[(7 << 256) | 9] = rng.getrandbits(256)
    cs = _random_constraints(rng, reg)
    lo = TermLowering(reg).lower(cs)
    prog = lower(lo.dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    agree = 0
    for trial in range(40):
        vals = []
        for v in prog.vars:
            choice = rng.random()
            if v.name in ("x", "y") and choice < 0.3:
                vals.append(rng.choice([0, 1, 5, 7, 9]))
            else:
                vals.append(rng.getrandbits(v.width))
        w = Witness(lo, vals, reg)
        host = all(w.ev(c) for c in cs)
        dev = sv.evaluate(vals)
        assert host == dev, (seed, trial)
        agree += 1
    assert agree == 40


def test_uf_hash_matches_oracle():
    rng = random.Random(1)
    for _ in range(20):
        x, salt = rng.getrandbits(256), rng.getrandbits(32)
        assert uf_hash(x, salt) == O.uf_hash(x, salt)


def test_keccak_interpretation_satisfies_conditions_by_construction():
    """Any candidate: inv(f(k)) == k, interval and %64 hold (keccak_function_manager.py:150-179)."""
    reg = UFRegistry()
    lo_idx = 10 ** 40 - 34534
    part = (2 ** 256 - 1) // 10 ** 40
    reg.keccak[256] = KeccakSpec(lo=lo_idx * part)
    f = Function("keccak256_256", [256], 256)
    inv = Function("keccak256_256-1", [256], 256)
    n = BV("n", 256)
    cond = And(inv(f(n)) == n, ULE(BVV(lo_idx * part, 256), f(n)),
               ULT(f(n), BVV(lo_idx * part + part, 256)), URem(f(n), BVV(64, 256)) == 0)
    lo = TermLowering(reg).lower([cond.raw])
    prog = lower(lo.dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    rng = np.random.default_rng(0)
    for _ in range(32):
        assert sv.evaluate([int.from_bytes(rng.bytes(32), "little")])


def test_check_sets_caches_witnessless_buckets(monkeypatch):
    """A bucket whose search found no witness is not lowered or searched again under the
    same search configuration (the search is deterministic); a deadline-cut search is not
    cached.  The engine is a stand-in that finds nothing (host logic only)."""
    import mythril_amd.engine as E
    from mythril_amd.smt import gpu_check

    uploads = []

    class _Res:
        def __init__(self, n, cut):
            self.found = np.full(n, 0xFFFFFFFF, dtype=np.uint32)
            self.kernel_ms, self.cands_decided = 0.0, 0
            self.timed_out = cut

    class _DB:
        def __init__(self, n):
            self.n = n

        def __len__(self):
            return self.n

        def free(self):
            pass

    class _Eng:
        cut = False

        def upload(self, progs):
            uploads.append(len(progs))
            return _DB(len(progs))

        def check(self, db, timeout_ms=0, **kw):
            return _Res(db.n, bool(timeout_ms) and self.cut)

    eng = _Eng()
    monkeypatch.setattr(E, "get_engine", lambda *a, **k: eng)
    gpu_check.reset_cache()
    x, y = symbol_factory.BitVecSym("x", 256), symbol_factory.BitVecSym("y", 256)
    sets = [[(x == symbol_factory.BitVecVal(5, 256)).raw, ULT(y, symbol_factory.BitVecVal(3, 256)).raw]]
    assert gpu_check.check_sets(sets) == [None]
    assert uploads == [2]                      # two independence buckets searched
    assert gpu_check.check_sets(sets) == [None]
    assert uploads == [2]                      # both answered from the negative cache
    cfg = gpu_check.GpuConfig(timeout_ms=5)
    gpu_check.check_sets(sets, config=cfg)
    assert uploads == [2]                      # a complete negative holds under a deadline too
    gpu_check.reset_cache()
    eng.cut = True                             # the device deadline cuts every search
    gpu_check.check_sets(sets, config=cfg)
    gpu_check.check_sets(sets, config=cfg)
    assert uploads == [2, 2, 2]                # deadline-cut searches are never cached
    eng.cut = False
    gpu_check.check_sets(sets, config=cfg)
    gpu_check.check_sets(sets, config=cfg)
    assert uploads == [2, 2, 2, 2]             # a deadline search that completed is cached
    gpu_check.reset_cache()


def test_parallel_lowering_matches_sequential(monkeypatch):
    """Lowering in spawned worker processes (terms re-intern on unpickling) yields the same
    programs, in the same order, as lowering in-process."""
    import mythril_amd.engine as E
    from mythril_amd import corpus
    from mythril_amd.smt import gpu_check

    uploaded = []

    class _Res:
        def __init__(self, n):
            self.found = np.full(n, 0xFFFFFFFF, dtype=np.uint32)
            self.kernel_ms, self.cands_decided = 0.0, 0
            self.timed_out = False

    class _DB:
        def __init__(self, n):
            self.n = n

        def __len__(self):
            return self.n

        def free(self):
            pass

    class _Eng:
        def upload(self, progs):
            uploaded.append(ir.Batch(progs))
            return _DB(len(progs))

        def check(self, db, **kw):
            return _Res(db.n)

        def keccak256(self, msgs):
            return [O.keccak256(m) for m in msgs]

    monkeypatch.setattr(E, "get_engine", lambda *a, **k: _Eng())
    c = corpus.build(4, 2, seed=7)
    sets = [q.constraints for q in c.queries]
    for workers in (1, 2):
        gpu_check.reset_cache()
        cfg = gpu_check.GpuConfig(workers=workers, parallel_min=1)
        gpu_check.check_sets(sets, registry=c.kfm.registry, config=cfg)
    seq, par = uploaded
    assert np.array_equal(seq.code, par.code) and np.array_equal(seq.consts, par.consts)
    assert np.array_equal(seq.schema, par.schema) and np.array_equal(seq.descs, par.descs)
    gpu_check.reset_cache()
