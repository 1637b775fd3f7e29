"""GPU parity: the gfx950 kernels against the oracle (oracle/pyoracle.py), bit-exact.

Every check goes through the C ABI (libpathfeas.so via ctypes).  Integer/byte work: the bar
is bit-exact equality, no tolerance.
"""

import numpy as np
import pyoracle as O
import pytest
from conftest import load_golden

import evm_to_ir
from mythril_amd import ir, synth
from mythril_amd.lower import Dag, lower

pytestmark = pytest.mark.gpu

_OPS = {
    "add": ir.W_ADD, "sub": ir.W_SUB, "mul": ir.W_MUL, "udiv": ir.W_UDIV, "urem": ir.W_UREM,
    "sdiv": ir.W_SDIV, "srem": ir.W_SREM, "smod": ir.W_SMOD, "shl": ir.W_SHL,
    "lshr": ir.W_LSHR, "ashr": ir.W_ASHR, "exp": ir.W_EXP,
}
_CMPS = {"ult": ir.B_ULT, "ule": ir.B_ULE, "slt": ir.B_SLT, "sle": ir.B_SLE,
         "uadd_noovf": ir.B_UADD_NOOVF, "umul_noovf": ir.B_UMUL_NOOVF}


def _op_program(name, w):
    """vars a, b, e (width w or 1): assert op(a, b) == e."""
    dag = Dag()
    a, b = dag.var("a", w), dag.var("b", w)
    if name in _OPS:
        e = dag.var("e", w)
        r = dag.op(_OPS[name], w, a, b)
        dag.assert_(dag.op(ir.B_EQ, w, r, e))
    else:
        e = dag.var("e", 1, ir.VK_BOOL)
        r = dag.op(_CMPS[name], w, a, b)
        dag.assert_(dag.op(ir.B_NOT, 1, dag.op(ir.B_XOR, 1, r, e)))
    return lower(dag)


def test_ops_golden_vectors(engine):
    vecs = load_golden("ops.json")
    groups = {}
    for v in vecs:
        groups.setdefault((v["op"], v["w"]), []).append(v)
    progs, keys = [], []
    for (name, w) in sorted(groups):
        progs.append(_op_program(name, w))
        keys.append((name, w))
    db = engine.upload(progs)
    for s, key in enumerate(keys):
        rows = groups[key]
        cands = []
        for v in rows:
            r = v["r"] if isinstance(v["r"], int) else int(v["r"], 16)
            cands.append([int(v["a"], 16), int(v["b"], 16), r])
            # a corrupted expectation must evaluate to false
            cands.append([int(v["a"], 16), int(v["b"], 16), (r ^ 1) & ir.mask(key[1] if key[0] in _OPS else 1)])
        soa = ir.pack_assignments(progs[s], cands)
        got = engine.eval_assignments(db, s, soa)
        want = np.array([i % 2 == 0 for i in range(len(cands))])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (key, [cands[i] for i in bad[:4]])


def test_eip145_shifts(engine):
    progs, cands = [], []
    for case in load_golden("eip145.json"):
        dag = Dag()
        v, s = dag.var("v", 256), dag.var("s", 256)
        op = {"shl": ir.W_SHL, "shr": ir.W_LSHR, "sar": ir.W_ASHR}[case["op"]]
        dag.assert_(dag.op(ir.B_EQ, 256, dag.op(op, 256, v, s), dag.const(int(case["expected"], 16), 256)))
        progs.append(lower(dag))
        cands.append([int(case["value"], 16), int(case["shift"], 16)])
    db = engine.upload(progs)
    for i, p in enumerate(progs):
        assert engine.eval_assignments(db, i, ir.pack_assignments(p, [cands[i]]))[0], i


def test_vmtests_post_storage(engine):
    progs, names = [], []
    for c in load_golden("vmtests.json"):
        try:
            progs.append(lower(evm_to_ir.build(c["code"], c["storage"])))
            names.append(c["name"])
        except evm_to_ir.Unsupported:
            pass
    assert len(progs) >= 200
    db = engine.upload(progs)
    failed = [names[i] for i, p in enumerate(progs)
              if not engine.eval_assignments(db, i, ir.pack_assignments(p, [[]]))[0]]
    assert not failed, failed


def _oracle_first(prog, budget, seed):
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    first, _ = sv.check(budget, seed)
    return first


@pytest.mark.parametrize("flags", [0, ir.FLAG_EARLY_EXIT, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT])
def test_search_matches_oracle(engine, flags):
    """Generated candidates: the smallest witness index equals the oracle's, per set."""
    budget, seed = 512, 0x1234_5678_9ABC
    progs = []
    for i in range(10):
        progs.append(synth.random_dag_set(100 + i, plant=False)[0])
        progs.append(synth.random_dag_set(200 + i, plant=True)[0])
    progs += [synth.mythril_like_set(i) for i in range(2)]
    db = engine.upload(progs)
    res = engine.check(db, budget=budget, seed=seed, flags=flags)
    for i, p in enumerate(progs):
        want = _oracle_first(p, budget, seed)
        got = None if res.found[i] == 0xFFFFFFFF else int(res.found[i])
        assert got == want, (i, p.name, got, want)
    assert res.cands_decided > 0


def _pressure_program(n_live=14):
    dag = Dag()
    x, y = dag.var("x", 256), dag.var("y", 256)
    prods = [dag.op(ir.W_MUL, 256, x, dag.op(ir.W_ADD, 256, y, dag.const(k + 1, 256))) for k in range(n_live)]
    acc = prods[0]
    for p in prods[1:]:
        acc = dag.op(ir.W_XOR, 256, acc, p)
    for p in prods:
        dag.assert_(dag.op(ir.B_ULT, 256, p, acc))
    return lower(dag, nw=ir.NW)


@pytest.mark.parametrize("flags", [0, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT])
def test_narrow_and_wide_register_files_agree(engine, flags):
    """The same sets lowered over 7 registers (8-register, 3-waves/SIMD kernels) and over 15
    (16-register kernels: the batch also holds a program that writes register 14) give the
    oracle's smallest witness in both."""
    budget, seed = 1024, 0xABCD_0123
    ids = [(700 + i, i % 3 == 0) for i in range(12)]
    narrow, wide = [], []
    for d, plant in ids:
        got = {}
        orig = synth.lower
        synth.lower = lambda dag, **k: got.setdefault("dag", dag) and orig(dag, **k)
        try:
            synth.random_dag_set(d, plant=plant)
        finally:
            synth.lower = orig
        narrow.append(lower(got["dag"], nw=ir.NW_NARROW))
        wide.append(lower(got["dag"], nw=ir.NW))
    pw = _pressure_program()
    assert max(int(ins[1] & 0xFF) for ins in ir.Batch([pw]).code.reshape(-1, 4)) >= ir.NW_NARROW
    rn = engine.check(engine.upload(narrow), budget=budget, seed=seed, flags=flags)
    rw = engine.check(engine.upload(wide + [pw]), budget=budget, seed=seed, flags=flags)
    for i, p in enumerate(narrow):
        want = _oracle_first(p, budget, seed)
        gn = None if rn.found[i] == 0xFFFFFFFF else int(rn.found[i])
        gw = None if rw.found[i] == 0xFFFFFFFF else int(rw.found[i])
        assert gn == want and gw == want, (i, gn, gw, want)
    if flags == 0:
        assert rn.evals_full == len(narrow) * budget


def test_planted_witness_found_at_candidate_zero(engine):
    progs = [synth.random_dag_set(300 + i, plant=True)[0] for i in range(16)]
    db = engine.upload(progs)
    res = engine.check(db, budget=4096, seed=99, flags=ir.FLAG_EARLY_EXIT)
    assert (res.found == 0).all()


@pytest.mark.parametrize("n_sets", [1, 2, 20, 64, 65])
def test_parented_small_batches_match_oracle(engine, n_sets):
    """Batches whose every set carries a parent model (2..64 of them take the probe launch,
    pathfeas.hip check_enqueue): candidate 0 is the witness for the untouched planted sets,
    not for the sets whose parent values were shifted by one (the search then continues from
    candidate 64 in the second launch, or finds a neighbourhood candidate among 1..63).  The
    smallest witness equals the oracle's either way, and with 1 or 65 sets (no probe) too."""
    import copy

    budget, seed = 2048, 0x5EED_0042
    progs = []
    for i in range(n_sets):
        p = synth.random_dag_set(500 + i, plant=True)[0]
        if i % 3 == 1:
            p = copy.deepcopy(p)
            for v in p.vars:
                if v.parent is not None:
                    v.parent = (v.parent + 1) & ((1 << v.width) - 1)
        progs.append(p)
    assert all(p.has_parent for p in progs)
    db = engine.upload(progs)
    res = engine.check(db, budget=budget, seed=seed, flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)
    for i, p in enumerate(progs):
        want = _oracle_first(p, budget, seed)
        got = None if res.found[i] == 0xFFFFFFFF else int(res.found[i])
        assert got == want, (n_sets, i, got, want)
        if i % 3 != 1:
            assert got == 0
    # PF_FLAG_NO_PROBE (the caller's "candidate 0 misses") changes no answer
    res2 = engine.check(db, budget=budget, seed=seed,
                        flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT | ir.FLAG_NO_PROBE)
    assert (res2.found == res.found).all()


@pytest.mark.parametrize("truth", [True, False])
def test_varless_set_in_a_parented_batch(engine, truth):
    """A set without variables counts as parented (pathfeas.hip: the batch takes the probe
    launch): a true ground set is answered at candidate 0, a false one never, and the
    parented sets beside it keep their oracle witnesses."""
    budget, seed = 2048, 0x5EED_0043
    progs = [synth.random_dag_set(600 + i, plant=True)[0] for i in range(3)]
    ground = ir.Program(name=f"ground_{truth}")
    ground.emit(ir.W_CONST, 256, dst=0, aux0=ground.const_index(7))
    ground.emit(ir.W_CONST, 256, dst=1, aux0=ground.const_index(7 if truth else 8))
    ground.emit(ir.B_EQ, 256, dst=0, a=0, b=1)
    ground.emit(ir.ASSERT, 1, a=0)
    ground.finish().validate()
    progs.insert(1, ground)
    res = engine.check(engine.upload(progs), budget=budget, seed=seed,
                       flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)
    assert int(res.found[1]) == (0 if truth else 0xFFFFFFFF)
    for i in (0, 2, 3):
        assert int(res.found[i]) == _oracle_first(progs[i], budget, seed) == 0


def test_materialize_matches_generator(engine):
    progs = [synth.random_dag_set(400 + i, plant=(i % 2 == 0))[0] for i in range(6)]
    progs.append(synth.mythril_like_set(5))
    db = engine.upload(progs)
    seed = 0xDEAD_BEEF_0001
    sets, cands = [], []
    for s in range(len(progs)):
        for c in (0, 1, 7, 63, 64, 1000, 65535):
            sets.append(s)
            cands.append(c)
    vals = engine.materialize(db, sets, cands, seed=seed)
    b = ir.Batch(progs)
    for k, (s, c) in enumerate(zip(sets, cands)):
        sv = O.SetView.from_batch(b, s)
        assert vals[k] == sv.gen_assignments(np.array([c], dtype=np.uint64), seed)[0], (s, c)


def test_witness_rechecks_on_oracle(engine):
    """The model handed back for a GPU witness satisfies the set under the oracle."""
    progs = [synth.random_dag_set(500 + i, plant=False)[0] for i in range(12)]
    db = engine.upload(progs)
    seed = 7
    res = engine.check(db, budget=8192, seed=seed, flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)
    sat = [i for i in range(len(progs)) if res.found[i] != 0xFFFFFFFF]
    assert sat, "no generated witness at all"
    vals = engine.materialize(db, sat, [int(res.found[i]) for i in sat], seed=seed)
    b = ir.Batch(progs)
    for k, s in enumerate(sat):
        assert O.SetView.from_batch(b, s).evaluate(vals[k])


def test_keccak_vmsha3_and_random(engine):
    msgs = [bytes(c["size"]) for c in load_golden("vmsha3.json")]
    want = [c["digest"].lower() for c in load_golden("vmsha3.json")]
    got = engine.keccak256(msgs)
    assert ["0x" + g.hex() for g in got] == want
    rng = np.random.default_rng(3)
    msgs = [rng.bytes(n) for n in list(range(0, 300)) + [64] * 50 + [1000, 4096]]
    got = engine.keccak256(msgs)
    for m, g in zip(msgs, got):
        assert g == O.keccak256(m)


@pytest.mark.parametrize("ln,shift", [(64, 0), (32, 0), (128, 0), (16, 0), (0, 0),
                                      (64, 8), (72, 0), (8, 0), (135, 0), (136, 0), (200, 0),
                                      (1, 3)])
def test_keccak_fixed_dev_matches(engine, ln, shift):
    """pf_keccak256_fixed_dev: the unrolled single-block kernel (len % 16 == 0, < 136, 16-B
    aligned) and the LDS-staged general kernel (any other length / alignment), every digest
    against the C Keccak restatement."""
    torch = pytest.importorskip("torch")
    import ctypes

    import coracle_py
    from mythril_amd import _lib
    n = 5000
    host = np.random.default_rng(5 + ln).integers(0, 256, size=n * ln + shift + 1, dtype=np.uint8)
    d_buf = torch.from_numpy(host).to("cuda")
    d_in = d_buf[shift:]
    d_out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ms = ctypes.c_float(0)
    stream = torch.cuda.current_stream().cuda_stream  # same stream as the tensors' producers
    _lib.check(_lib.lib().pf_keccak256_fixed_dev(d_in.data_ptr(), ln, n, d_out.data_ptr(),
                                                 ctypes.byref(ms), stream), "keccak fixed")
    torch.cuda.synchronize()
    out = d_out.cpu().numpy().reshape(n, 32)
    want = coracle_py.keccak256_fixed(host[shift:], ln, n)
    assert np.array_equal(out, want)
    assert out[0].tobytes() == O.keccak256(host[shift:shift + ln].tobytes())


def _rand_operand(rng, w):
    k = int(rng.integers(0, 6))
    M = ir.mask(w)
    if k == 0:
        return [0, 1, 2, M, M - 1, 1 << (w - 1), (1 << (w - 1)) - 1][int(rng.integers(0, 7))] & M
    if k == 1:
        return int.from_bytes(rng.bytes(32), "little") & ((1 << int(rng.integers(1, w + 1))) - 1)
    if k == 2:
        return ((1 << int(rng.integers(0, w))) + int(rng.integers(-1, 2))) & M
    return int.from_bytes(rng.bytes(32), "little") & M


@pytest.mark.parametrize("name", sorted(_OPS))
def test_random_arith_bulk(engine, name):
    """4,096 seeded operand pairs per op (w = 256 and an odd width), GPU vs the oracle."""
    fn = {"add": O.bvadd, "sub": O.bvsub, "mul": O.bvmul, "udiv": O.bvudiv, "urem": O.bvurem,
          "sdiv": O.bvsdiv, "srem": O.bvsrem, "smod": O.bvsmod, "shl": O.bvshl,
          "lshr": O.bvlshr, "ashr": O.bvashr, "exp": O.bvexp}[name]
    rng = np.random.default_rng(0xA11CE + len(name))
    for w in (256, 173):
        prog = _op_program(name, w)
        db = engine.upload([prog])
        cands = []
        for _ in range(2048):
            a, b = _rand_operand(rng, w), _rand_operand(rng, w)
            if name in ("shl", "lshr", "ashr") and rng.random() < 0.7:
                b = int(rng.integers(0, w + 2))
            r = fn(a, b, w)
            cands.append([a, b, r])
            cands.append([a, b, r ^ (1 << int(rng.integers(0, w)))])
        got = engine.eval_assignments(db, 0, ir.pack_assignments(prog, cands))
        want = np.array([i % 2 == 0 for i in range(len(cands))])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, w, [[hex(v) for v in cands[i]] for i in bad[:3]])


def test_exp_split_edges(engine):
    """pf::exp256_split (windowed low 84 bits + 2-adic closed form for bits 84..253) against
    the oracle's pow(b, e, 2^w): exponents at the 84 / 254 / 256 boundaries, odd and even
    bases, and whole waves (64 lanes) that are all-even / all-small-exponent so the
    wave-uniform skips of the closed form are taken too."""
    rng = np.random.default_rng(0xE4F)
    M = (1 << 256) - 1
    exps = [0, 1, 2, 255, 256, 257, (1 << 84) - 1, 1 << 84, (1 << 84) + 1, (1 << 85) + 3,
            (1 << 126) + 5, (1 << 254) - 1, 1 << 254, (1 << 254) + 1, (1 << 255) + 7, M, M - 1]
    bases = [0, 1, 2, 3, 5, 7, M, M - 1, 1 << 255, (1 << 255) + 1, 3 << 100, (1 << 84) + 1]
    for w in (256, 200, 64):
        Mw = ir.mask(w)
        prog = _op_program("exp", w)
        db = engine.upload([prog])
        groups = []
        for b in bases:
            for e in exps:
                groups.append((b, e))
        for _ in range(640):
            groups.append((int.from_bytes(rng.bytes(32), "little"), int.from_bytes(rng.bytes(32), "little")))
        # uniform waves: all-even bases with big exponents, all-odd with small exponents
        even_wave = [(int.from_bytes(rng.bytes(32), "little") & ~1, int.from_bytes(rng.bytes(32), "little"))
                     for _ in range(64)]
        small_wave = [(int.from_bytes(rng.bytes(32), "little") | 1, int(rng.integers(0, 1 << 62)))
                      for _ in range(64)]
        pairs = even_wave + small_wave + groups
        cands = []
        for b, e in pairs:
            b, e = b & Mw, e & Mw
            r = O.bvexp(b, e, w)
            assert r == pow(b, e, 1 << w)
            cands.append([b, e, r])
        got = engine.eval_assignments(db, 0, ir.pack_assignments(prog, cands))
        bad = np.nonzero(~got)[0]
        assert bad.size == 0, (w, [[hex(v) for v in cands[i]] for i in bad[:3]])


@pytest.mark.parametrize("name", ["udiv", "urem", "sdiv", "srem", "smod"])
def test_division_one_limb_divisor_waves(engine, name):
    """Whole waves whose divisors fit one 32-bit limb take the short-division path
    (pf::udivrem256); zero divisors included (z3 conventions), signed forms through the
    magnitudes (a negative 256-bit divisor is wide, so those lanes use positives)."""
    fn = {"udiv": O.bvudiv, "urem": O.bvurem, "sdiv": O.bvsdiv, "srem": O.bvsrem,
          "smod": O.bvsmod}[name]
    rng = np.random.default_rng(0xD1 + len(name))
    w = 256
    prog = _op_program(name, w)
    db = engine.upload([prog])
    cands = []
    for i in range(4096):
        a = _rand_operand(rng, w)
        b = [0, 1, 2, 3, 0xFFFFFFFF, 0x80000000, int(rng.integers(0, 1 << 32))][i % 7]
        r = fn(a, b, w)
        cands.append([a, b, r])
        cands.append([a, b, r ^ (1 << int(rng.integers(0, w)))])
    got = engine.eval_assignments(db, 0, ir.pack_assignments(prog, cands))
    want = np.array([i % 2 == 0 for i in range(len(cands))])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (name, [[hex(v) for v in cands[i]] for i in bad[:3]])


@pytest.mark.parametrize("name", ["udiv", "urem", "sdiv", "smod"])
def test_division_one_digit_quotient_waves(engine, name):
    """Whole waves whose quotients fit one 32-bit digit (bitlen(a) <= bitlen(b) + 31) take
    the f64-estimate path of pf::udivrem256: exact multiples, multiples minus one and
    random operands around the boundary."""
    fn = {"udiv": O.bvudiv, "urem": O.bvurem, "sdiv": O.bvsdiv, "smod": O.bvsmod}[name]
    rng = np.random.default_rng(0x0D16 + len(name))
    w = 256
    prog = _op_program(name, w)
    db = engine.upload([prog])
    cands = []
    for i in range(4096):
        lb = int(rng.integers(33, 255))
        b = int.from_bytes(rng.bytes(32), "little") % (1 << lb) | (1 << (lb - 1))
        k = int(rng.integers(0, 1 << 31))
        a = [b * k, b * k + b - 1, b * k + 1,
             int.from_bytes(rng.bytes(32), "little") % (1 << min(255, lb + 30))][i % 4] % (1 << 255)
        r = fn(a, b, w)
        cands.append([a, b, r])
        cands.append([a, b, r ^ (1 << int(rng.integers(0, w)))])
    got = engine.eval_assignments(db, 0, ir.pack_assignments(prog, cands))
    want = np.array([i % 2 == 0 for i in range(len(cands))])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (name, [[hex(v) for v in cands[i]] for i in bad[:3]])


def test_window_lookup_programs(engine):
    """Array reads through window lookups (smt/to_dag.TermLowering._run: concat, shift by
    8 * (idx - lo), byte): the kernel's verdicts on adversarial index values (partial hits,
    wrap-around at 2^256, overlapping symbolic runs) and its smallest generated witness, with
    and without the host hints, equal the oracle's."""
    import random

    from test_lowering import _WINDOW_X, _window_terms

    from mythril_amd import seed as S
    from mythril_amd.smt.to_dag import TermLowering, UFRegistry

    cs = _window_terms()[0]
    plain = TermLowering(UFRegistry()).lower(cs)
    hinted = TermLowering(UFRegistry()).lower(cs)
    S.apply_hints(hinted.dag)
    progs = [lower(plain.dag), lower(hinted.dag)]
    assert any(ins.op == ir.W_LSHR for ins in progs[0].code)
    db = engine.upload(progs)
    rng = random.Random(29)
    names = [v.name for v in plain.dag.vars]
    cands = []
    for k in range(256):
        vals = [rng.choice(_WINDOW_X + [rng.getrandbits(256)]) if v.width == 256
                else rng.choice((0, 5, 7, 0xA9, rng.getrandbits(8))) for v in plain.dag.vars]
        if k % 4 == 0:
            vals[names.index("y")] = (vals[names.index("x")] + 4 + rng.randrange(-33, 34)) % (1 << 256)
        cands.append(vals)
    sv = O.SetView.from_batch(ir.Batch([progs[0]]), 0)
    got = engine.eval_assignments(db, 0, ir.pack_assignments(progs[0], cands))
    want = np.array([sv.evaluate(c) for c in cands])
    assert np.array_equal(got, want)
    budget, seed = 2048, 0x5EED_0042
    for flags in (0, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT):
        res = engine.check(db, budget=budget, seed=seed, flags=flags)
        for i, p in enumerate(progs):
            w = _oracle_first(p, budget, seed)
            g = None if res.found[i] == 0xFFFFFFFF else int(res.found[i])
            assert g == w, (flags, i, g, w)


def test_candidate0_limbs_match_device_materialize(engine):
    """The host rows gpu_check reads for a witness at candidate 0 of a fully parented program
    (native_terms.candidate0_limbs) are what pf_materialize returns for candidate 0, under
    several seeds (the candidate-0 rule does not depend on the seed)."""
    from test_lowering import _window_terms

    from mythril_amd.smt import native_terms as NT
    from mythril_amd.smt.to_dag import UFRegistry

    if NT.batch_api() is None:
        pytest.skip("libpflower.so without the batch API")
    cs, wx, wy, late = _window_terms()
    buckets_ = [cs, cs[:3], [cs[4]]]
    res = NT.lower_many([(b, None) for b in buckets_], UFRegistry(), True, [1, 2, 3], 1)
    progs = [r[1] for r in res if r[2] is None]
    assert len(progs) == len(buckets_)
    rows = [NT.candidate0_limbs(p) for p in progs]
    assert all(r is not None for r in rows)
    db = engine.upload(progs)
    for seed in (0, 7, 0xDEAD_BEEF):
        got = engine.materialize_limbs(db, list(range(len(progs))), [0] * len(progs), seed=seed)
        assert np.array_equal(got, np.concatenate(rows)), seed


def _spill_heavy_programs(n=24, nw=4):
    """Config-3 DAGs lowered over only ``nw`` W registers (those that fit): spills
    everywhere, many of them across an EXP (scratch) and many not (pf_batch_create's LDS
    slots, PF_SPILL_LDS).  Variables are spilled across EXPs too (PF_VAR_SPILL_USES_EXP=0;
    the default regenerates them there), so both kinds of slot run."""
    import os

    from mythril_amd import lower as L

    real = synth.lower
    env = os.environ.get("PF_VAR_SPILL_USES_EXP")
    out, i = [], 0
    try:
        os.environ["PF_VAR_SPILL_USES_EXP"] = "0"
        synth.lower = lambda dag, seed=0, name="": L.lower(dag, seed, name, nw)
        while len(out) < n and i < 20 * n:
            try:
                out.append(synth.random_dag_set(300 + i, plant=(i % 3 == 0))[0])
            except L.LoweringError:
                pass
            i += 1
    finally:
        synth.lower = real
        if env is None:
            os.environ.pop("PF_VAR_SPILL_USES_EXP", None)
        else:
            os.environ["PF_VAR_SPILL_USES_EXP"] = env
    return out


@pytest.mark.parametrize("flags", [0, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT])
def test_spill_heavy_programs_match_oracle(engine, flags):
    """Programs at three W registers (spill code in most instructions, both kinds of spill
    slot): the smallest witness equals the oracle's, which evaluates the program as lowered."""
    budget, seed = 512, 0x5EED
    progs = _spill_heavy_programs()
    n_spill = sum(int(((p.words[:, 0] & 0xFF) == ir.W_SPILL).sum()) for p in progs if hasattr(p, "words"))
    db = engine.upload(progs)
    res = engine.check(db, budget=budget, seed=seed, flags=flags)
    for i, p in enumerate(progs):
        want = _oracle_first(p, budget, seed)
        got = None if res.found[i] == 0xFFFFFFFF else int(res.found[i])
        assert got == want, (i, p.name, got, want)
    assert n_spill == 0 or n_spill > len(progs)


def _forwarding_programs():
    """Hand-built chains for the device program's forwarding pass (pathfeas.hip pass 5):
    a result read as both operands of the next instruction, a forwarded result also read
    later (its write-back kept), results feeding compares, ITE and B ops in between, a long
    mixed chain (DIV, EXP, shifts, CONCAT / EXTRACT), and the same chains at three W
    registers (spills and fills forwarded)."""
    progs = []
    for nw in (ir.NW_NARROW, 3):
        dag = Dag()
        x, y, z = dag.var("x", 256), dag.var("y", 256), dag.var("z", 256)
        r = dag.op(ir.W_MUL, 256, x, y)
        s = dag.op(ir.W_ADD, 256, r, r)                       # FA + FB
        t = dag.op(ir.W_XOR, 256, s, x)
        dag.assert_(dag.op(ir.B_ULT, 256, t, z))
        progs.append(lower(dag, nw=nw))

        dag = Dag()
        x, y, z = dag.var("x", 256), dag.var("y", 256), dag.var("z", 256)
        r = dag.op(ir.W_MUL, 256, x, y)
        s = dag.op(ir.W_SUB, 256, r, x)                       # r forwarded ...
        u = dag.op(ir.W_ADD, 256, s, r)                       # ... and read again
        b = dag.op(ir.B_ULT, 256, u, z)
        v = dag.op(ir.W_ITE, 256, b, u, s)
        dag.assert_(dag.op(ir.B_ULE, 256, v, dag.op(ir.W_UDIV, 256, z, dag.op(ir.W_OR, 256, y, dag.const(1, 256)))))
        progs.append(lower(dag, nw=nw))

        dag = Dag()
        x, y, z = dag.var("x", 256), dag.var("y", 256), dag.var("z", 256)
        acc, other = x, y
        ops = [ir.W_MUL, ir.W_ADD, ir.W_SDIV, ir.W_XOR, ir.W_UREM, ir.W_SUB, ir.W_SMOD, ir.W_AND,
               ir.W_EXP, ir.W_OR, ir.W_SREM, ir.W_MUL]
        for k in range(30):
            op = ops[k % len(ops)]
            acc = dag.op(op, 256, acc, other if k % 3 else z)
            if k % 5 == 4:
                acc = dag.op(ir.W_SHL, 256, acc, dag.const(k, 256))
            if k % 7 == 6:
                lo = dag.op(ir.W_EXTRACT, 128, acc, aux=0)
                acc = dag.op(ir.W_CONCAT, 256, lo, dag.op(ir.W_EXTRACT, 128, other, aux=128), aux=128)
            other = dag.op(ir.W_ADD, 256, other, acc) if k % 4 == 0 else other
        dag.assert_(dag.op(ir.B_ULT, 256, acc, other))
        progs.append(lower(dag, nw=nw))
    return progs


def test_forwarding_chains_match_oracle(engine):
    """Every explicit candidate's verdict (pf_eval_assignments) and the search's smallest
    witness on the forwarding chains equal the oracle's — with the device program actually
    forwarding (PF_I_FA / PF_I_FB set, some write-backs skipped)."""
    import random

    from test_device_program import I_FA, I_FB, TR_WW, device_program

    progs = _forwarding_programs()
    code, _ = device_program(ir.Batch(progs))
    ops = code[:, 0] & 0xFF
    assert ((code[:, 0] & I_FA) != 0).sum() > 10 and ((code[:, 0] & I_FB) != 0).sum() > 0
    w_res = (ops < ir.B_CONST) & (ops != ir.END) & (ops != ir.W_SPILL)
    assert (w_res & ((code[:, 0] & TR_WW) == 0)).sum() > 5
    rng = random.Random(17)
    db = engine.upload(progs)
    for s, p in enumerate(progs):
        sv = O.SetView.from_batch(ir.Batch([p]), 0)
        cands = []
        for _ in range(192):
            vals = [rng.getrandbits(256) for _ in p.vars]
            if rng.random() < 0.3:
                vals = [v >> rng.randrange(0, 256) for v in vals]
            cands.append(vals)
        got = engine.eval_assignments(db, s, ir.pack_assignments(p, cands))
        want = np.array([bool(sv.evaluate(c)) for c in cands])
        assert (got == want).all(), (s, np.nonzero(got != want)[0][:4])
    budget, seed = 2048, 0xF0D
    res = engine.check(db, budget=budget, seed=seed)
    for i, p in enumerate(progs):
        want = _oracle_first(p, budget, seed)
        got = None if res.found[i] == 0xFFFFFFFF else int(res.found[i])
        assert got == want, (i, got, want)


_WIDTHS = (1, 8, 32, 64, 160, 256)


@pytest.mark.parametrize("w", _WIDTHS)
def test_every_op_at_laser_widths(engine, w):
    """Every arithmetic op and compare at the widths LASER's terms take — a Bool-sized bit
    vector, calldata bytes, 32/64-bit words, 160-bit addresses, full words — 384 seeded
    operand pairs each (boundary values, short random values, powers of two ± 1, uniform),
    GPU against the oracle; each pair also with a corrupted expectation, which must fail."""
    fns = {"add": O.bvadd, "sub": O.bvsub, "mul": O.bvmul, "udiv": O.bvudiv, "urem": O.bvurem,
           "sdiv": O.bvsdiv, "srem": O.bvsrem, "smod": O.bvsmod, "shl": O.bvshl,
           "lshr": O.bvlshr, "ashr": O.bvashr, "exp": O.bvexp}
    M = ir.mask(w)

    def cmp(name, a, b):
        sa = a - (1 << w) if a >> (w - 1) else a
        sb = b - (1 << w) if b >> (w - 1) else b
        return int({"ult": a < b, "ule": a <= b, "slt": sa < sb, "sle": sa <= sb,
                    "uadd_noovf": a + b <= M, "umul_noovf": a * b <= M}[name])

    names = sorted(fns) + sorted(_CMPS)
    progs = [_op_program(n, w) for n in names]
    db = engine.upload(progs)
    rng = np.random.default_rng(0xB175 + w)
    for s, name in enumerate(names):
        cands = []
        for _ in range(384):
            a, b = _rand_operand(rng, w), _rand_operand(rng, w)
            if name in ("shl", "lshr", "ashr") and rng.random() < 0.6:
                b = int(rng.integers(0, w + 2)) & M
            if name in fns:
                r = fns[name](a, b, w)
                cands.append([a, b, r])
                cands.append([a, b, r ^ (1 << int(rng.integers(0, w)))])
            else:
                r = cmp(name, a, b)
                cands.append([a, b, r])
                cands.append([a, b, r ^ 1])
        got = engine.eval_assignments(db, s, ir.pack_assignments(progs[s], cands))
        want = np.array([i % 2 == 0 for i in range(len(cands))])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, w, [[hex(v) for v in cands[i]] for i in bad[:3]])
