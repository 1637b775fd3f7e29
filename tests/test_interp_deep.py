"""The host witness evaluator (smt/interp.py, Model.eval's interpretation) on terms nested
deeper than Python's recursion limit: a large LASER state's constraints are long and / or /
ite chains and thousands-deep storage store chains.  Values must equal a direct
(non-recursive) evaluation; found at 5x corpus scale, where the planted-model check raised
RecursionError."""

import sys

from mythril_amd import corpus
from mythril_amd.smt import terms as T
from mythril_amd.smt.to_dag import UFRegistry


def _eval(vars_, arrays=None):
    return corpus._PlantedEval(corpus.Planted(vars=dict(vars_), arrays=dict(arrays or {})), UFRegistry())


def test_deep_and_or_chain():
    depth = 4 * sys.getrecursionlimit()
    x = T.var("x", 256)
    t = T.cmp("bvult", x, T.const(10, 256))
    want = True
    for i in range(depth):
        c = T.eq(x, T.const(3 + (i % 5), 256))
        if i % 2:
            t = T.and_(t, T.or_(c, T.not_(c)))
        else:
            t = T.or_(t, T.and_(c, T.not_(c)))
    assert _eval({"x": 4}).ev(t) == want
    assert not _eval({"x": 40}).ev(t)


def test_deep_arithmetic_and_ite_chain():
    depth = 4 * sys.getrecursionlimit()
    x = T.var("x", 256)
    v, want, xv = x, 7, 7
    for i in range(depth):
        v = T.ite(T.cmp("bvult", v, T.const(1 << 200, 256)), T.binop("bvadd", v, T.const(i, 256)), v)
        want = (want + i) % (1 << 256) if want < (1 << 200) else want
    assert _eval({"x": xv}).ev(v) == want


def test_deep_store_chain_select():
    n = 4 * sys.getrecursionlimit()
    a = T.const_array(256, T.const(0, 256))
    for i in range(n):
        a = T.store(a, T.const(i, 256), T.const(i * i + 1, 256))
    ev = _eval({})
    assert ev.ev(T.select(a, T.const(0, 256))) == 1
    assert ev.ev(T.select(a, T.const(n - 1, 256))) == (n - 1) ** 2 + 1
    assert ev.ev(T.select(a, T.const(n + 5, 256))) == 0


def test_substitute_deep_chain():
    from mythril_amd.smt.subst import substitute

    depth = 4 * sys.getrecursionlimit()
    x, y = T.var("x", 256), T.var("y", 256)
    v = x
    for i in range(depth):
        v = T.binop("bvadd", T.binop("bvmul", v, T.const(3, 256)), T.const(i, 256))
    w = substitute(v, x, y)
    want = 5
    for i in range(depth):
        want = (want * 3 + i) % (1 << 256)
    assert _eval({"y": 5}).ev(w) == want
    folded = substitute(v, x, T.const(5, 256))   # the folding constructors reduce it to a constant
    assert folded.op == "bv" and folded.val == want


def test_smtlib_reader_deep_let_chain():
    """z3's --solver-log output nests a let per shared subterm."""
    from mythril_amd import smtlib

    depth = 6 * sys.getrecursionlimit()
    body = "x"
    for i in range(depth):
        body = f"(let ((a!{i} (bvadd {body} #x{(i % 251):064x}))) a!{i})"
    text = f"(declare-fun x () (_ BitVec 256))\n(assert (= {body} #x{0:064x}))\n(check-sat)\n"
    # the reader walks the nesting iteratively, on the caller's thread, with the process's
    # recursion limit untouched
    limit = sys.getrecursionlimit()
    q = smtlib.read_query(text)
    assert sys.getrecursionlimit() == limit
    assert len(q.assertions) == 1
    want = (-sum(i % 251 for i in range(depth))) % (1 << 256)
    assert _eval({"x": want}).ev(q.assertions[0])
    assert not _eval({"x": want + 1}).ev(q.assertions[0])


def test_native_lowering_leaves_over_deep_terms_to_z3():
    """The native term -> program passes recurse over the nesting; a term deeper than
    PF_MAX_TERM_DEPTH (5000) is a LoweringError (the bucket goes to z3) instead of a host
    stack overflow (a 25,000-deep chain segfaulted the process before)."""
    import pytest

    from mythril_amd.smt import gpu_check, native_terms
    if native_terms.batch_api() is None:
        pytest.skip("libpflower.so not built")
    x, y = T.var("x", 256), T.var("y", 256)

    def chain(depth):
        v = x
        for i in range(depth):
            v = T.binop("bvxor", T.binop("bvadd", v, y), T.const(i + 1, 256)) if i % 2 else T.binop("bvmul", v, y)
        return T.cmp("bvult", v, T.const(12345, 256))

    shallow, deep = chain(1000), chain(20000)
    res = native_terms.lower_many([([shallow], None), ([deep], None)], UFRegistry(), True,
                                  [gpu_check._set_seed([shallow]), gpu_check._set_seed([deep])], 1)
    assert res[0][2] is None and res[0][1] is not None
    assert res[1][0] is None and "left to z3" in res[1][2]
