"""CPU: the device form of a batch (pf_batch_create's peepholes, exported host-only as
pf_device_program) computes what the lowered program computes.

The kernel runs a rewritten program: an ASSERT folded into the compare before it
(PF_I_ASSERT) and a W_CONST folded into every reader of its register (PF_I_KA / PF_I_KB:
the register field holds the constant index).  ``eval_device`` below is the kernel's reading
of those flags, restated for the test; the oracle evaluates the program as lowered.  The GPU
parity tests then compare the kernel itself against the oracle."""

import ctypes
import random

import numpy as np
import pytest

import pyoracle as O
from mythril_amd import _lib, ir, synth

I_ASSERT, I_KA, I_KB, I_FA, I_FB = 1 << 24, 1 << 25, 1 << 26, 1 << 27, 1 << 28
TR_WW = 4 << 18


def device_program(batch):
    L = _lib.lib()
    code = np.ascontiguousarray(batch.code, dtype=np.uint32)
    descs = np.ascontiguousarray(batch.descs, dtype=np.uint32)
    out = np.zeros_like(code)
    dout = np.zeros_like(descs)
    n = ctypes.c_size_t()
    consts = np.ascontiguousarray(batch.consts, dtype=np.uint32)
    _lib.check(L.pf_device_program(_lib.ptr_u32(code), len(code),
                                   _lib.ptr_u32(consts.reshape(-1)) if consts.size else None, len(consts),
                                   _lib.ptr_u32(descs), len(descs),
                                   _lib.ptr_u32(out), ctypes.byref(n), _lib.ptr_u32(dout)),
               "pf_device_program")
    return out[:n.value], dout


def eval_device(sv, code_rows, values):
    """SetView.evaluate with the device flags: a KA / KB operand is const[a] / const[b], an
    FA / FB operand the previous instruction's W result (held here in spare register slots);
    a W result whose PF_TR_WW is cleared is not written back (its register keeps its old
    value, or none: a later read of it fails here); a PF_I_ASSERT op also asserts its B
    result."""
    W, B, S = {}, {}, {}
    root = True
    last = None
    for (w0, w1, aux0, aux1) in code_rows:
        op = w0 & 0xFF
        if op == O.OP["END"]:
            break
        if w0 & I_KA:
            W[0xFE] = sv.consts[(w1 >> 8) & 0xFF]
            w1 = (w1 & ~0xFF00) | (0xFE << 8)
        if w0 & I_KB:
            W[0xFD] = sv.consts[(w1 >> 16) & 0xFF]
            w1 = (w1 & ~0xFF0000) | (0xFD << 16)
        if w0 & I_FA:
            W[0xFC] = last
            w1 = (w1 & ~0xFF00) | (0xFC << 8)
        if w0 & I_FB:
            W[0xFB] = last
            w1 = (w1 & ~0xFF0000) | (0xFB << 16)
        w_result = op < O.OP["B_CONST"] and op != O.OP["W_SPILL"]
        d = w1 & 0xFF
        old = W.get(d)
        root = _step((w0 & ~(I_ASSERT | I_KA | I_KB | I_FA | I_FB), w1, aux0, aux1), sv.consts, W, B, S, values,
                     root)
        if w_result:
            last = W[d]
            if not (w0 & TR_WW):          # forwarded only: no write-back
                if old is None:
                    del W[d]
                else:
                    W[d] = old
        if w0 & I_ASSERT:
            root = root and B[w1 & 0xFF]
    return root


SPILL_LDS = 0x100


def _step(ins, consts, W, B, S, values, root):
    """One instruction of pyoracle's evaluator (SetView.evaluate) on shared registers.  A
    PF_SPILL_LDS slot (aux 0x100 | e) is LDS entry e of EXP's window table: a W_EXP rewrites
    entries 1..3 and a B_UMUL_NOOVF entry 1 — modelled by forgetting them, so a fill the
    peephole placed across one of them fails here."""
    w0, w1, aux0, aux1 = ins
    op, w = w0 & 0xFF, (w0 >> 8) & 0x3FF
    if op == O.OP["W_EXP"]:
        for e in (1, 2, 3):
            S.pop(SPILL_LDS | e, None)
    elif op == O.OP["B_UMUL_NOOVF"]:
        S.pop(SPILL_LDS | 1, None)
    d, a, b, c = w1 & 0xFF, (w1 >> 8) & 0xFF, (w1 >> 16) & 0xFF, (w1 >> 24) & 0xFF
    M = O.M
    if op == O.OP["W_CONST"]:
        W[d] = consts[aux0] & M(w)
    elif op == O.OP["W_VAR"]:
        W[d] = int(values[aux0]) & M(w)
    elif op == O.OP["W_MOV"]:
        W[d] = W[a] & M(w)
    elif op in O._WBIN:
        W[d] = O._WBIN[op](W[a], W[b], w)
    elif op == O.OP["W_NOT"]:
        W[d] = O.bvnot(W[a], w)
    elif op == O.OP["W_NEG"]:
        W[d] = O.bvneg(W[a], w)
    elif op == O.OP["W_EXTRACT"]:
        W[d] = O.extract(W[a], aux0, w)
    elif op == O.OP["W_CONCAT"]:
        W[d] = O.concat(W[a], W[b], aux0) & M(w)
    elif op == O.OP["W_SEXT"]:
        W[d] = O.sign_extend(W[a], aux0, w)
    elif op == O.OP["W_ITE"]:
        W[d] = W[a] if B[c] else W[b]
    elif op == O.OP["W_HASH"]:
        W[d] = O.uf_hash(W[a], aux0) & M(w)
    elif op == O.OP["W_SPILL"]:
        S[aux0] = W[a]
    elif op == O.OP["W_FILL"]:
        W[d] = S[aux0] & M(w)
    elif op == O.OP["B_SPILL"]:
        S[aux0] = int(B[a])
    elif op == O.OP["B_FILL"]:
        B[d] = bool(S[aux0] & 1)
    elif op == O.OP["B_CONST"]:
        B[d] = bool(aux0 & 1)
    elif op == O.OP["B_VAR"]:
        B[d] = bool(int(values[aux0]) & 1)
    elif op in O._BCMP:
        B[d] = bool(O._BCMP[op](W[a], W[b], w))
    elif op == O.OP["B_AND"]:
        B[d] = B[a] and B[b]
    elif op == O.OP["B_OR"]:
        B[d] = B[a] or B[b]
    elif op == O.OP["B_XOR"]:
        B[d] = B[a] != B[b]
    elif op == O.OP["B_NOT"]:
        B[d] = not B[a]
    elif op == O.OP["B_ITE"]:
        B[d] = B[a] if B[c] else B[b]
    elif op == O.OP["ASSERT"]:
        root = root and B[a]
    else:
        raise ValueError(op)
    return root


def _programs(monkeypatch):
    from mythril_amd import keccak_manager as KM
    from mythril_amd.smt import symbol_factory

    # concrete hashes from the oracle's Keccak (the corpus would ask the engine otherwise)
    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))
    progs = [synth.random_dag_set(i, plant=(i % 2 == 0))[0] for i in range(40)]
    from mythril_amd import corpus
    c = corpus.build(3, 2, seed=11)
    from mythril_amd.smt.independence import buckets
    from mythril_amd.smt.to_dag import TermLowering
    from mythril_amd.lower import LoweringError, lower
    n = 0
    for q in c.queries:
        for bk in buckets(q.constraints):
            try:
                lo = TermLowering(c.kfm.registry).lower(bk)
            except LoweringError:
                continue
            progs.append(lower(lo.dag, seed=n))
            n += 1
            if n >= 60:
                return progs
    return progs


def test_device_program_matches_the_lowered_program(monkeypatch):
    batch = ir.Batch(_programs(monkeypatch))
    code, descs = device_program(batch)
    n_const_fused = int(((code[:, 0] & (I_KA | I_KB)) != 0).sum())
    n_wconst = int(((batch.code[:, 0] & 0xFF) == ir.W_CONST).sum())
    n_wconst_dev = int(((code[:, 0] & 0xFF) == ir.W_CONST).sum())
    assert n_const_fused > 0 and n_wconst_dev < n_wconst
    ops = code[:, 0] & 0xFF
    spills = np.isin(ops, [ir.W_SPILL, ir.B_SPILL])
    n_lds = int((spills & ((code[:, 2] & SPILL_LDS) != 0)).sum())
    assert 0 < n_lds < int(spills.sum())     # some spills moved to LDS, not those across an EXP
    n_fwd = int(((code[:, 0] & (I_FA | I_FB)) != 0).sum())
    w_res = (ops < ir.B_CONST) & (ops != ir.END) & (ops != ir.W_SPILL)
    n_nowb = int((w_res & ((code[:, 0] & TR_WW) == 0)).sum())
    assert n_fwd > 0 and 0 < n_nowb <= n_fwd  # forwarded operands; results only they read
    rng = random.Random(3)
    for s in range(len(batch.descs)):
        sv = O.SetView.from_batch(batch, s)
        d = descs[s]
        rows = [tuple(int(x) for x in r) for r in code[d[0]:d[0] + d[1]]]
        assert rows[-1][0] & 0xFF == 0                      # still END-terminated
        cands = sv.gen_assignments(np.arange(24, dtype=np.uint64), 5)
        for vals in cands + [[rng.getrandbits(sv.var_width(v)) for v in range(len(sv.schema))]]:
            assert eval_device(sv, rows, vals) == sv.evaluate(vals), s


def test_out_of_width_constant_is_not_folded(monkeypatch):
    """a W_CONST masks its constant to its width at write-back, a folded operand
    (PF_I_KA / PF_I_KB) reads it raw — so a constant wider than its W_CONST stays a W_CONST,
    and the device program still computes what the lowered one does."""
    batch = ir.Batch(_programs(monkeypatch))     # corpus buckets carry narrow constants
    code0, descs0 = device_program(batch)

    def n_wconst(code, descs, s):
        d = descs[s]
        return int(((code[d[0]:d[0] + d[1], 0] & 0xFF) == ir.W_CONST).sum())

    tried = kept = 0
    for s, d in enumerate(batch.descs):
        for i in range(d[0], d[0] + d[1]):
            w0 = int(batch.code[i, 0])
            if w0 & 0xFF != ir.W_CONST or ((w0 >> 8) & 0x3FF) >= 224:
                continue
            k = int(d[2]) + int(batch.code[i, 2])
            saved = int(batch.consts[k, 7])
            batch.consts[k, 7] = saved | 0x80000000      # bit 255: outside any width < 224
            code1, descs1 = device_program(batch)
            tried += 1
            # folded before (the W_CONST was deleted) -> kept now
            if n_wconst(code1, descs1, s) == n_wconst(code0, descs0, s) + 1:
                kept += 1
            sv = O.SetView.from_batch(batch, s)
            e = descs1[s]
            rows = [tuple(int(x) for x in r) for r in code1[e[0]:e[0] + e[1]]]
            for vals in sv.gen_assignments(np.arange(16, dtype=np.uint64), 9):
                assert eval_device(sv, rows, vals) == sv.evaluate(vals)
            batch.consts[k, 7] = saved
            if tried >= 12:
                break
        if tried >= 12:
            break
    assert tried > 0 and kept > 0, (tried, kept)


def test_spill_heavy_device_programs_keep_their_values():
    """Three W registers: the LDS spill peephole under heavy pressure (entries reused, spills
    across EXPs left in scratch) — the device form, with EXP / UMUL_NOOVF clobbering the LDS
    entries, still computes the lowered program's verdict."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_gpu_parity import _spill_heavy_programs

    batch = ir.Batch(_spill_heavy_programs(n=16))
    code, descs = device_program(batch)
    ops = code[:, 0] & 0xFF
    spills = np.isin(ops, [ir.W_SPILL, ir.B_SPILL])
    lds = spills & ((code[:, 2] & SPILL_LDS) != 0)
    assert lds.sum() > 10 and (spills & ~lds).sum() > 10
    rng = random.Random(9)
    for s in range(len(batch.descs)):
        sv = O.SetView.from_batch(batch, s)
        d = descs[s]
        rows = [tuple(int(x) for x in r) for r in code[d[0]:d[0] + d[1]]]
        cands = sv.gen_assignments(np.arange(16, dtype=np.uint64), 3)
        for vals in cands + [[rng.getrandbits(sv.var_width(v)) for v in range(len(sv.schema))]]:
            assert eval_device(sv, rows, vals) == sv.evaluate(vals), s


def test_forwarding_keeps_the_write_back_of_a_result_read_again():
    """Pass 5 on a hand-built chain: r = x*y is forwarded into s = r - x and read again by
    u = s + r, so the MUL keeps its write-back while the SUB (read only by the next
    instruction) skips it; a result read as both operands of the next instruction is
    forwarded on both sides."""
    from mythril_amd.lower import Dag, lower

    dag = Dag()
    x, y, z = dag.var("x", 256), dag.var("y", 256), dag.var("z", 256)
    r = dag.op(ir.W_MUL, 256, x, y)
    s = dag.op(ir.W_SUB, 256, r, x)
    u = dag.op(ir.W_ADD, 256, s, r)
    v = dag.op(ir.W_XOR, 256, u, u)
    dag.assert_(dag.op(ir.B_ULT, 256, v, z))
    batch = ir.Batch([lower(dag)])
    code, descs = device_program(batch)
    rows = code[descs[0][0]:descs[0][0] + descs[0][1]]
    ops = [int(w0) & 0xFF for w0 in rows[:, 0]]
    w0 = {op: int(rows[ops.index(op), 0]) for op in (ir.W_MUL, ir.W_SUB, ir.W_ADD, ir.W_XOR)}
    assert w0[ir.W_MUL] & TR_WW                       # r is read again by the ADD
    assert w0[ir.W_SUB] & I_FA                        # r forwarded into the SUB ...
    assert not (w0[ir.W_SUB] & TR_WW)                 # ... whose result only the ADD reads
    assert w0[ir.W_ADD] & (I_FA | I_FB)
    assert w0[ir.W_XOR] & I_FA and w0[ir.W_XOR] & I_FB   # u ^ u: both operands forwarded
    sv = O.SetView.from_batch(batch, 0)
    rng = random.Random(5)
    rows_t = [tuple(int(q) for q in row) for row in rows]
    for _ in range(64):
        vals = [rng.getrandbits(256) for _ in range(3)]
        assert eval_device(sv, rows_t, vals) == sv.evaluate(vals)


def test_large_batch_program_equals_per_set_programs():
    """A batch large enough for the threaded preparation (>= 64 sets, >= 32,768 instructions:
    set ranges rewritten on host threads, then concatenated) gets, set by set, exactly the
    device program the set gets alone."""
    progs = [synth.mythril_like_set(i) for i in range(150)] + \
        [synth.random_dag_set(900 + i, plant=True)[0] for i in range(150)]
    b = ir.Batch(progs)
    assert len(b.descs) >= 64 and len(b.code) >= 32768
    out, dout = device_program(b)
    for s, p in enumerate(progs):
        one, d1 = device_program(ir.Batch([p]))
        lo, n = int(dout[s][0]), int(dout[s][1])
        assert n == int(d1[0][1]), s
        assert (out[lo:lo + n] == one[:n]).all(), s
