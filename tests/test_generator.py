"""The candidate generator's calldata-byte arm (include/pf_bytecode.h PF_VK_CDBYTE).

LASER reads every calldata word as 32 single-byte array reads (state/calldata.py:233-246),
so a dispatcher's ``selector == 0xa9059cbb`` is four byte variables that must all match
at once — hopeless for independent per-byte strategies.  The arm spells a whole ABI word
from one harvested constant per (candidate, word).  These CPU tests pin the contract in
both oracles (the GPU tests compare the kernel with them: test_gpu_parity.py's
materialize / LASER-shaped sets use the same synthetic sets).
"""

import numpy as np

import coracle_py
import pyoracle as O

from mythril_amd import ir, synth
from mythril_amd.lower import Dag, lower


def test_cdbyte_hints():
    assert ir.cdbyte_hints("1_calldata[0]") == (24, 0xFFFFFFFF)   # selector, big-endian
    assert ir.cdbyte_hints("1_calldata[3]") == (0, 0xFFFFFFFF)
    assert ir.cdbyte_hints("2_calldata[4]") == (248, 0)           # argument word 0, byte 0
    assert ir.cdbyte_hints("2_calldata[35]") == (0, 0)
    assert ir.cdbyte_hints("1_calldata[36]") == (248, 1)
    from mythril_amd.smt.to_dag import var_kind
    assert var_kind("3_calldata[7]", 8) == ir.VK_CDBYTE
    assert var_kind("3_calldata@2", 8) == ir.VK_GENERIC            # symbolic offset: generic
    assert var_kind("3_calldata[7]", 256) == ir.VK_GENERIC
    assert var_kind("call_value2", 256) == ir.VK_VALUE
    assert var_kind("callvalue7", 256) == ir.VK_VALUE


def _selector_dag(sel: int):
    dag = Dag()
    bs = []
    for i in range(4):
        name = f"1_calldata[{i}]"
        bs.append(dag.var(name, 8, ir.VK_CDBYTE, *ir.cdbyte_hints(name)))
    w = bs[0]
    for k, b in enumerate(bs[1:], start=1):
        w = dag.op(ir.W_CONCAT, 8 * (k + 1), w, b, aux=8)
    dag.assert_(dag.op(ir.B_EQ, 32, w, dag.const(sel, 32)))
    # a second constant in the pool, so the arm has to pick the right one
    dag.assert_(dag.op(ir.B_ULT, 32, dag.const(0x1234, 32), w))
    return dag


def test_word_bytes_share_one_constant():
    """In candidates where the arm fires, the four selector bytes spell one pool constant
    (or its neighbour +-1)."""
    prog = lower(_selector_dag(0xA9059CBB), seed=7)
    b = ir.Batch([prog])
    sv = O.SetView.from_batch(b, 0)
    consts = {(c + d) & 0xFFFFFFFF for c in prog.consts for d in (0, 1, -1)}
    vals = sv.gen_assignments(np.arange(4096, dtype=np.uint64), 5)
    words = [(v[0] << 24) | (v[1] << 16) | (v[2] << 8) | v[3] for v in vals]
    spelled = sum(1 for w in words if w in consts)
    assert spelled > 4096 // 4          # about half the candidates take the arm
    assert sum(1 for w in words if w == 0xA9059CBB) > 4096 // (4 * 2 * len(prog.consts))


def test_oracles_agree_on_the_arm():
    """The C restatement (the kernel's checker) and the Python one give the same SAT flags
    for LASER-shaped sets with calldata-byte variables."""
    progs = [synth.mythril_like_set(i) for i in range(4)] + [lower(_selector_dag(0xDEADBEEF), seed=3)]
    b = ir.Batch(progs)
    pk = coracle_py.Packed(b)
    cands = np.arange(512, dtype=np.uint64)
    for s in range(len(progs)):
        sv = O.SetView.from_batch(b, s)
        want = [sv.evaluate(v) for v in sv.gen_assignments(cands, 11)]
        got = pk.eval_generated(s, 11, 0, len(cands))
        assert list(got) == want, s


def test_dispatch_sets_found_without_hints():
    """A selector dispatch + caller actor set + argument bounds + non-payable check (the
    path-entry shape of every LASER query) is witnessed by the generator alone."""
    progs = [synth.mythril_like_set(i) for i in range(8)]
    pk = coracle_py.Packed(ir.Batch(progs))
    found = [pk.first_sat(s, 0x4D595448, 65536) for s in range(len(progs))]
    # (before the calldata-word, ABI-size and call-value arms: none of the eight)
    assert sum(f is not None for f in found) >= 6, found


def test_size_and_value_arms():
    """ABI-aligned calldata sizes and zero call values in about half the candidates."""
    dag = Dag()
    size = dag.var("1_calldatasize", 256, ir.VK_SMALL, hint0=4 + 32 * 8)
    val = dag.var("call_value1", 256, ir.VK_VALUE)
    dag.assert_(dag.op(ir.B_ULE, 256, size, val))
    prog = lower(dag, seed=1)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    vals = sv.gen_assignments(np.arange(2048, dtype=np.uint64), 9)
    sizes = [v[0] for v in vals]
    assert all(0 <= s <= 260 for s in sizes)
    aligned = sum(1 for s in sizes if (s - 4) % 32 == 0)
    assert 2048 * 0.45 < aligned < 2048 * 0.65
    zeros = sum(1 for v in vals if v[1] == 0)
    assert 2048 * 0.45 < zeros < 2048 * 0.6
