"""CPU: lowering preserves the conjunction's value (term-level oracle == bytecode oracle)."""

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


@pytest.mark.parametrize("dag_id", range(12))
def test_synth_lowering_agrees(dag_id):
    dag, prog, wit = _synth_dag(dag_id)
    assert eval_dag(dag, wit)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    assert sv.evaluate(wit)
    _programs_agree(dag, prog, n=16)


def test_remat_under_pressure():
    # 20 overlapping calldata-style words force rematerialisation of cheap interior values
    dag = Dag()
    size = dag.var("size", 256)
    words = [synth.calldata_word(dag, 1, off, size) for off in (0, 4, 8, 36)]
    for k, wd in enumerate(words):
        dag.assert_(dag.op(ir.B_ULE, 256, wd, dag.const(1 << (200 + k), 256)))
    prog = lower(dag)
    _programs_agree(dag, prog, n=8)


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
    # a DAG whose products are each used twice, far apart, cannot stay within 15 registers
    dag2 = Dag()
    ys = [dag2.var(f"y{i}", 256) for i in range(20)]
    ps = [dag2.op(ir.W_MUL, 256, ys[i], ys[i]) for i in range(20)]
    a1 = ps[0]
    for p in ps[1:]:
        a1 = dag2.op(ir.W_ADD, 256, a1, p)
    a2 = ps[-1]
    for p in reversed(ps[:-1]):
        a2 = dag2.op(ir.W_XOR, 256, a2, p)
    dag2.assert_(dag2.op(ir.B_EQ, 256, a1, a2))
    with pytest.raises(LoweringError):
        lower(dag2)


def test_mythril_like_lowers():
    for i in range(3):
        p = synth.mythril_like_set(i)
        p.validate()
        assert p.code[-1].op == ir.END
