"""CPU: lowering preserves the conjunction's value (term-level oracle == bytecode oracle)."""

import random

import coracle_py
import numpy as np
import pyoracle as O
import pytest

from dag_eval import eval_dag
from mythril_amd import ir, synth
from mythril_amd.lower import Dag, LoweringError, lower


def _programs_agree(dag, prog, n=64, seed=7):
    rng = np.random.default_rng(seed)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    for _ in range(n):
        vals = [int.from_bytes(rng.bytes(32), "little") & ir.mask(v.width) for v in dag.vars]
        assert eval_dag(dag, vals) == sv.evaluate(vals)


def _synth_dag(dag_id):
    captured = {}
    orig = synth.lower

    def cap(dag, **kw):
        captured["dag"] = dag
        return orig(dag, **kw)

    synth.lower = cap
    try:
        prog, wit = synth.random_dag_set(dag_id)
    finally:
        synth.lower = orig
    return captured["dag"], prog, wit


# 34783, 38037: config-3 DAGs whose narrow (7-register) lowering once gave a wrong program —
# a node rematerialised inside another node's operand list released an operand register
# the enclosing node had pinned, and its result overwrote it (lower.py emit_node)
@pytest.mark.parametrize("dag_id", list(range(12)) + [34783, 38037])
def test_synth_lowering_agrees(dag_id):
    dag, prog, wit = _synth_dag(dag_id)
    assert eval_dag(dag, wit)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    assert sv.evaluate(wit)
    _programs_agree(dag, prog, n=16)


def test_planted_witness_survives_lowering_scan():
    """Every planted witness of 3,000 config-3 DAGs (ids spread over the 1M range) still
    satisfies the lowered program, at 7 and at 15 W registers."""
    from mythril_amd.lower import lower_py

    bad = []
    for dag_id in range(0, 1_000_000, 333):
        dag, prog, wit = _synth_dag(dag_id)
        for p in (prog, lower_py(dag, nw=15)):
            if not O.SetView.from_batch(ir.Batch([p]), 0).evaluate(wit):
                bad.append(dag_id)
    assert not bad, bad


def test_remat_under_pressure():
    # 20 overlapping calldata-style words force rematerialisation of cheap interior values
    dag = Dag()
    size = dag.var("size", 256)
    words = [synth.calldata_word(dag, 1, off, size) for off in (0, 4, 8, 36)]
    for k, wd in enumerate(words):
        dag.assert_(dag.op(ir.B_ULE, 256, wd, dag.const(1 << (200 + k), 256)))
    prog = lower(dag)
    _programs_agree(dag, prog, n=8)


def _pressure_dag(n):
    """n products, each used twice far apart: more than 15 live W values at once."""
    dag = Dag()
    ys = [dag.var(f"y{i}", 256) for i in range(n)]
    ps = [dag.op(ir.W_MUL, 256, ys[i], ys[i]) for i in range(n)]
    a1 = ps[0]
    for p in ps[1:]:
        a1 = dag.op(ir.W_ADD, 256, a1, p)
    a2 = ps[-1]
    for p in reversed(ps[:-1]):
        a2 = dag.op(ir.W_XOR, 256, a2, p)
    dag.assert_(dag.op(ir.B_EQ, 256, a1, a2))
    return dag


def test_register_pressure_spills_and_evaluates():
    """More live values than registers: the lowering spills (PF_W_SPILL / PF_W_FILL) and
    the bytecode still computes the DAG's value (oracle evaluation of the program)."""
    dag = _pressure_dag(20)
    prog = lower(dag)
    ops = [i.op for i in prog.code]
    assert ir.W_SPILL in ops and ir.W_FILL in ops
    b = ir.Batch([prog])
    sv = O.SetView.from_batch(b, 0)
    rng = random.Random(5)
    for _ in range(20):
        vals = [rng.getrandbits(256) for _ in dag.vars]
        assert sv.evaluate(vals) == bool(eval_dag(dag, vals))
    P = coracle_py.Packed(b)
    cands = sv.gen_assignments(np.arange(64, dtype=np.uint64), 3)
    want = np.array([sv.evaluate(a) for a in cands])
    assert (P.eval_generated(0, 3, 0, 64) == want).all()


def test_beyond_spill_capacity_rejected():
    with pytest.raises(LoweringError):
        lower(_pressure_dag(ir.NW + ir.MAX_SPILL + 4))


def test_too_many_live_values_rejected():
    dag = Dag()
    xs = [dag.var(f"x{i}", 256) for i in range(20)]
    muls = [dag.op(ir.W_MUL, 256, xs[i], xs[(i + 1) % 20]) for i in range(20)]
    acc = muls[0]
    for m in muls[1:]:
        acc = dag.op(ir.W_ADD, 256, acc, m)
    # all products computed first would need 20 live registers; post-order avoids that
    dag.assert_(dag.op(ir.B_EQ, 256, acc, dag.const(0, 256)))
    lower(dag)  # fine in post-order
    # a DAG whose products are each used twice, far apart, cannot stay within 15 registers:
    # it spills (test_register_pressure_spills_and_evaluates)


def test_mythril_like_lowers():
    for i in range(3):
        p = synth.mythril_like_set(i)
        p.validate()
        assert p.code[-1].op == ir.END


def _word_slicing_exprs(dag):
    """Selector / address / low-mask / shift / division patterns over a calldata-like word
    (32 bytes, each If(i <s size, b_i, 0), concatenated)."""
    bs = [dag.var(f"b{i}", 8) for i in range(32)]
    size = dag.var("size", 256)
    parts = [dag.op(ir.W_ITE, 8, dag.op(ir.B_SLT, 256, dag.const(i, 256), size), b, dag.const(0, 8))
             for i, b in enumerate(bs)]
    word, wd = parts[0], 8
    for p in parts[1:]:
        wd += 8
        word = dag.op(ir.W_CONCAT, wd, word, p, aux=8)
    outs = [
        dag.op(ir.W_LSHR, 256, word, dag.const(224, 256)),
        dag.op(ir.W_AND, 256, dag.op(ir.W_UDIV, 256, word, dag.const(1 << 224, 256)), dag.const(0xFFFFFFFF, 256)),
        dag.op(ir.W_AND, 256, word, dag.const((1 << 160) - 1, 256)),
        dag.op(ir.W_AND, 256, dag.const((1 << 160) - 1, 256), word),
        dag.op(ir.W_LSHR, 256, dag.op(ir.W_MOV, 256, dag.op(ir.W_EXTRACT, 100, word, aux=20)), dag.const(30, 256)),
        dag.op(ir.W_EXTRACT, 40, word, aux=100),
        dag.op(ir.W_EXTRACT, 16, dag.op(ir.W_MOV, 256, dag.op(ir.W_EXTRACT, 64, word, aux=8)), aux=60),
        dag.op(ir.W_UDIV, 256, word, dag.const(1, 256)),
        dag.op(ir.W_LSHR, 256, word, dag.const(0, 256)),
        dag.op(ir.W_LSHR, 256, word, dag.const(300, 256)),
    ]
    bools = [dag.op(ir.B_EQ, 256, outs[0], dag.const(0xA9059CBB, 256)),
             dag.op(ir.B_EQ, 256, dag.const(0x1FFFFFFFF, 256), outs[1]),
             dag.op(ir.B_EQ, 256, outs[2], dag.const(7, 256))]
    return outs + bools


def test_word_slicing_rewrites_preserve_values(monkeypatch):
    """Dag.op's z3.simplify-style rewrites (udiv by 2^k, shifts / masks / extracts of
    concats) give the same value as the unrewritten DAG on every input."""
    from dag_eval import eval_dag_values

    monkeypatch.setattr(Dag, "_simplify", lambda self, *a: None)
    plain = Dag()
    e_plain = _word_slicing_exprs(plain)
    monkeypatch.undo()
    simp = Dag()
    e_simp = _word_slicing_exprs(simp)
    rng = random.Random(11)

    def values(dag, raw):
        return [raw[32] if v.name == "size" else raw[int(v.name[1:])] for v in dag.vars]

    for trial in range(200):
        raw = [rng.getrandbits(8) for _ in range(32)]
        raw.append(rng.choice([0, 3, 4, 20, 36, 40, 1 << 255, rng.getrandbits(256)]))
        if trial % 3 == 0:
            raw[:4] = [0xA9, 0x05, 0x9C, 0xBB]
        vp = eval_dag_values(plain, values(plain, raw))
        vs = eval_dag_values(simp, values(simp, raw))
        for a, b in zip(e_plain, e_simp):
            assert vp[a] == vs[b], (trial, a, b)


def test_witness_reads_nested_calldata_offsets_like_the_program():
    """An ABI dynamic argument: a calldata read at an offset itself read from calldata
    (state/calldata.py:233-246 words, BECToken's batchTransfer).  The host Witness must
    interpret the nested reads exactly as the lowered program does (first earlier read with
    an equal index, in lookup order) — a table built before the nested reads were resolved
    rejected GPU witnesses in the host re-check."""
    from mythril_amd.smt import terms as T
    from mythril_amd.smt.interp import Witness
    from mythril_amd.smt.to_dag import TermLowering, UFRegistry

    cd = T.array("1_calldata", 256, 8)
    off = T.concat(*[T.select(cd, T.const(i, 256)) for i in range(4, 8)])   # offset word (32 bits)
    base = T.binop("bvadd", T.zero_extend(224, off), T.const(4, 256))
    n = T.concat(*[T.select(cd, T.binop("bvadd", base, T.const(j, 256))) for j in range(2)])
    cs = [T.cmp("bvult", T.const(0, 16), n), T.cmp("bvult", off, T.const(16, 32))]
    lo = TermLowering(UFRegistry()).lower(cs)
    prog = lower(lo.dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    rng = random.Random(3)
    agree = sat = 0
    for _ in range(400):
        vals = [rng.choice((0, 1, 4, 5, 8, 9, rng.getrandbits(8))) & ir.mask(v.width) for v in lo.dag.vars]
        want = sv.evaluate(vals)
        w = Witness(lo, vals, UFRegistry())
        got = all(bool(w.ev(c)) for c in cs)
        agree += got == want
        sat += want
    assert agree == 400 and sat > 0


def test_reads_at_one_base_and_distinct_offsets_need_no_alias_test():
    """calldata[x + 4 + k] for k = 0..3 (one symbolic base, distinct constant offsets — a
    dynamic-ABI word) can never alias each other, so the lowering emits no index comparison
    between them (TermLowering._offset_form); against a constant index and across bases the
    comparisons stay.  A store at base + c read back at (base + c - 1) + 1 is that store's
    value without a test.  The program, the host Witness and the oracle still agree."""
    from mythril_amd.smt import terms as T
    from mythril_amd.smt.interp import Witness
    from mythril_amd.smt.to_dag import TermLowering, UFRegistry

    cd = T.array("1_calldata", 256, 8)
    x = T.var("x", 256)
    y = T.var("y", 256)
    base = T.binop("bvadd", x, T.const(4, 256))
    word = T.concat(*[T.select(cd, T.binop("bvadd", base, T.const(k, 256))) for k in range(4)])
    lo = TermLowering(UFRegistry()).lower([T.cmp("bvult", T.const(5, 32), word)])
    assert not any(n.kind == ir.B_EQ for n in lo.dag.nodes)
    # a constant index and another base do get compared with the symbolic reads
    cs = [T.cmp("bvult", T.const(5, 32), word),
          T.eq(T.select(cd, T.const(6, 256)), T.const(7, 8)),
          T.eq(T.select(cd, y), T.const(9, 8))]
    lo2 = TermLowering(UFRegistry()).lower(cs)
    # 4 reads x cd[6], 5 earlier reads x cd[y], and the two equalities of the constraints
    assert sum(n.kind == ir.B_EQ for n in lo2.dag.nodes) == 4 + 5 + 2
    st = T.store(T.array("s", 256, 256), T.binop("bvadd", x, T.const(3, 256)), T.const(11, 256))
    idx = T.binop("bvadd", T.binop("bvsub", T.binop("bvadd", x, T.const(3, 256)), T.const(1, 256)),
                  T.const(1, 256))
    rd = TermLowering(UFRegistry())
    assert rd.node(T.select(st, idx)) == rd.dag.const(11, 256)
    prog = lower(lo2.dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    rng = random.Random(5)
    agree = sat = 0
    for _ in range(300):
        vals = [rng.choice((0, 1, 2, 3, 6, 7, 9, rng.getrandbits(8))) & ir.mask(v.width) for v in lo2.dag.vars]
        want = sv.evaluate(vals)
        got = all(bool(Witness(lo2, vals, UFRegistry()).ev(c)) for c in cs)
        agree += got == want
        sat += want
    assert agree == 300 and sat > 0


def _window_terms():
    """A dynamic-ABI shape with long index runs: calldata bytes 0..39 read at constant
    indices (a 40-byte run: a 32-byte window piece and an 8-byte one), a word read at
    x + 4 + k (k = 0..31), a word at another symbolic base y + k compared against both, and a
    constant index read after the symbolic ones (a run of one base: a window too)."""
    from mythril_amd.smt import terms as T

    cd = T.array("1_calldata", 256, 8)
    hdr = [T.select(cd, T.const(i, 256)) for i in range(40)]
    x = T.var("x", 256)
    y = T.var("y", 256)
    wx = T.concat(*[T.select(cd, T.binop("bvadd", T.binop("bvadd", x, T.const(4, 256)), T.const(k, 256)))
                    for k in range(32)])
    wy = T.concat(*[T.select(cd, T.binop("bvadd", y, T.const(k, 256))) for k in range(32)])
    late = T.select(cd, T.const(70, 256))
    cs = [T.cmp("bvult", T.const(3, 256), T.concat(*hdr[4:36])),
          T.eq(hdr[0], T.const(0xA9, 8)),
          T.cmp("bvult", T.const(5, 256), wx),
          T.cmp("bvule", wy, wx),
          T.eq(late, T.const(7, 8))]
    return cs, wx, wy, late


_WINDOW_X = [0, 1, 3, 4, 8, 31, 32, 33, 35, 36, 39, 40, 66, 70, 100, (1 << 256) - 1, (1 << 256) - 4,
             (1 << 256) - 5, (1 << 256) - 31, (1 << 256) - 32, (1 << 256) - 40]


def test_index_runs_become_window_lookups_with_the_same_values(monkeypatch):
    """Runs of >= 8 contiguous indices of a byte array with one base (constants, or one
    symbolic base) are read through a window lookup — concat, shift by 8 * (idx - lo), byte
    — instead of an ite(idx == lo + j) chain: every read and every constraint takes the
    chain's value on every assignment, including indices that hit a run partially, wrap
    around 2^256, or fall between the pieces; the program, the host Witness and the oracle
    agree; and the DAG has a fraction of the chain's comparisons."""
    from dag_eval import eval_dag_values
    from mythril_amd.smt import to_dag
    from mythril_amd.smt.interp import Witness
    from mythril_amd.smt.to_dag import TermLowering, UFRegistry

    cs, wx, wy, late = _window_terms()
    win = TermLowering(UFRegistry())
    lw = win.lower(cs)
    monkeypatch.setattr(to_dag, "_WINDOW_MIN", 1 << 30)
    chain = TermLowering(UFRegistry())
    lc = chain.lower(cs)
    monkeypatch.undo()
    n_eq = [sum(n.kind == ir.B_EQ for n in lo.dag.nodes) for lo in (lw, lc)]
    assert sum(n.kind == ir.W_LSHR for n in lw.dag.nodes) >= 64 + 1
    assert n_eq[0] * 10 < n_eq[1], n_eq
    assert [v.name for v in lw.dag.vars] == [v.name for v in lc.dag.vars]
    reads = [win.memo.get(t) for t in (wx, wy, late)]
    reads_c = [chain.memo.get(t) for t in (wx, wy, late)]
    prog = lower(lw.dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    rng = random.Random(17)
    sat = 0
    for trial in range(400):
        vals = []
        for v in lw.dag.vars:
            if v.width == 256:
                vals.append(rng.choice(_WINDOW_X + [rng.getrandbits(256)]))
            else:
                vals.append(rng.choice((0, 5, 7, 0xA9, rng.getrandbits(8))))
        if trial % 4 == 0:   # y at x + 4 + d: the two symbolic runs overlap
            vals[[v.name for v in lw.dag.vars].index("y")] = (vals[[v.name for v in lw.dag.vars].index("x")]
                                                             + 4 + rng.randrange(-33, 34)) % (1 << 256)
        vw, vc = eval_dag_values(lw.dag, vals), eval_dag_values(lc.dag, vals)
        for a, b in zip(reads, reads_c):
            assert vw[a] == vc[b], trial
        for a, b in zip(lw.dag.roots, lc.dag.roots):
            assert vw[a] == vc[b], trial
        want = sv.evaluate(vals)
        assert all(bool(Witness(lw, vals, UFRegistry()).ev(c)) for c in cs) == want
        sat += want
    assert sat > 0


def _slot_steal_dag(n_vars, n_pairs):
    """Every spill slot taken and every register held by a value that can be neither
    recomputed nor evicted for free, at the moment a spilled variable is filled for its last
    use (the steal must not take the slot being filled).  Phase 1 spills the
    variables (each used again later); phase 2 computes two fresh products per root — each
    live to the end, so two spills per root against the one slot the root's variable frees."""
    dag = Dag()
    xs = [dag.var(f"x{i}", 256) for i in range(n_vars)]
    for i, x in enumerate(xs):
        dag.assert_(dag.op(ir.B_ULT, 256, x, dag.const((i + 1) << 200, 256)))
    live = []
    for k in range(n_pairs):
        y, z = dag.var(f"y{k}", 256), dag.var(f"z{k}", 256)
        q, r = dag.op(ir.W_MUL, 256, y, y), dag.op(ir.W_MUL, 256, z, z)
        live += [q, r]
        dag.assert_(dag.op(ir.B_ULT, 256, dag.op(ir.W_ADD, 256, xs[k % n_vars], q), r))
    acc = live[-1]
    for v in reversed(live[:-1]):
        acc = dag.op(ir.W_XOR, 256, acc, v)
    dag.assert_(dag.op(ir.B_ULT, 256, acc, dag.const(1 << 255, 256)))
    return dag


@pytest.mark.parametrize("n_vars", [30, 40])
def test_fill_never_loses_its_own_slot(n_vars):
    """At 7 registers the steal would have taken the slot of the variable being filled (a
    FILL from slot NONE / a KeyError that aborted check_sets); now that lowering is a clean
    LoweringError, the default policy moves to 15 registers, and the program validates and
    computes the DAG's value."""
    from mythril_amd.lower import lower_py

    dag = _slot_steal_dag(n_vars, 36)
    with pytest.raises(LoweringError):
        lower_py(dag, nw=ir.NW_NARROW)
    with pytest.raises(LoweringError):
        lower(dag, nw=ir.NW_NARROW)
    prog = lower(dag)
    b = ir.Batch([prog])           # validates: every FILL reads a slot a SPILL wrote
    w = prog.words if isinstance(prog, ir.PackedProgram) else \
        np.array([ins.words() for ins in prog.code], dtype=np.uint32).reshape(-1, 4)
    fills = w[(w[:, 0] & 0xFF) == ir.W_FILL]
    assert len(fills) and (fills[:, 2] < ir.MAX_SPILL).all()
    sv = O.SetView.from_batch(b, 0)
    rng = random.Random(11)
    for _ in range(6):
        vals = [rng.getrandbits(256) for _ in dag.vars]
        assert sv.evaluate(vals) == bool(eval_dag(dag, vals))
