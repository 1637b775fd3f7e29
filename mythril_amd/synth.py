"""Synthetic constraint-set workloads (BASELINE.json configs).

``random_dag_set(dag_id)`` is config 3: a random 256-bit BitVec DAG of depth >= 32 with the
MUL/DIV/EXP-heavy op mix, 4-8 free variables, constants drawn 50 % uniform / 50 % boundary,
and a root conjunction of 2-4 comparisons against values computed from a planted witness, so
every set is satisfiable.  The planted witness is attached as the parent model (candidate 0)
when ``plant=True``; otherwise the search has to find a witness on its own.

``mythril_like_set(i)`` builds the term shapes the LASER engine produces for a function
dispatcher path (calldata words as 32 x ite(i <s size, select, 0) bytes, the actor
disjunction for the caller, callvalue checks) — used until real --solver-log dumps exist.
"""

from __future__ import annotations

import bisect
from typing import List, Optional, Tuple

import numpy as np

from . import ir
from .lower import Dag, lower
from .ir import Program

DAG_GEN_SEED = 20260101
CAND_SEED_BASE = 0x4D595448

# op mix
_MIX = [
    (ir.W_MUL, 0.25), ("div", 0.20), ("rem", 0.10), (ir.W_EXP, 0.05), ("addsub", 0.15),
    ("logic", 0.10), ("shift", 0.05), ("itecmp", 0.10),
]
_BOUNDARY = [0, 1, 2, ir.mask(256), 1 << 255, (1 << 160) - 1]
_MIX_OPS = [m[0] for m in _MIX]
_MIX_CDF = [float(x) for x in (lambda c: c / c[-1])(np.cumsum(np.array([m[1] for m in _MIX]) /
                                                             sum(m[1] for m in _MIX)))]


def _boundary(rng) -> int:
    j = int(rng.integers(0, 9))
    if j < len(_BOUNDARY):
        return _BOUNDARY[j]
    k = int(rng.integers(0, 256))
    return ((1 << k) + (-1, 0, 1)[j - len(_BOUNDARY)]) & ir.mask(256)


def _rand256(rng) -> int:
    v = 0
    for w in rng.integers(0, 1 << 32, size=8, dtype=np.uint64):
        v = (v << 32) | int(w)
    return v


def _leaf_value(rng) -> int:
    return _rand256(rng) if rng.random() < 0.5 else _boundary(rng)


def _eval(op, a, b, w=256):
    # concrete semantics used only to compute the planted comparison targets; the
    # evaluation that decides SAT is the kernel's (checked against oracle/pyoracle.py)
    M = ir.mask(w)

    def sgn(x):
        return x - (1 << w) if x >> (w - 1) else x

    if op == ir.W_ADD:
        return (a + b) & M
    if op == ir.W_SUB:
        return (a - b) & M
    if op == ir.W_MUL:
        return (a * b) & M
    if op == ir.W_UDIV:
        return M if b == 0 else a // b
    if op == ir.W_UREM:
        return a if b == 0 else a % b
    if op in (ir.W_SDIV, ir.W_SREM):
        sa, sb = sgn(a), sgn(b)
        if b == 0:
            return ((1 if sa < 0 else M) if op == ir.W_SDIV else a)
        q = abs(sa) // abs(sb)
        if op == ir.W_SDIV:
            return (q if (sa < 0) == (sb < 0) else -q) & M
        r = abs(sa) % abs(sb)
        return (r if sa >= 0 else -r) & M
    if op == ir.W_AND:
        return a & b
    if op == ir.W_OR:
        return a | b
    if op == ir.W_XOR:
        return a ^ b
    if op == ir.W_NOT:
        return ~a & M
    if op == ir.W_SHL:
        return 0 if b >= w else (a << b) & M
    if op == ir.W_LSHR:
        return 0 if b >= w else a >> b
    if op == ir.W_ASHR:
        if b >= w:
            return M if a >> (w - 1) else 0
        return (sgn(a) >> b) & M
    if op == ir.W_EXP:
        return pow(a, b, 1 << w)
    raise ValueError(op)


def random_dag_set(dag_id: int, n_interior: int = 48, depth: int = 32, window: int = 6,
                   plant: bool = True) -> Tuple[Program, List[int]]:
    """Config-3 set number ``dag_id``; returns (program, planted witness values)."""
    rng = np.random.Generator(np.random.Philox(key=(DAG_GEN_SEED << 32) | (dag_id & 0xFFFFFFFF)))
    dag = Dag()
    n_vars = int(rng.integers(4, 9))
    witness = [_leaf_value(rng) for _ in range(n_vars)]
    leaves = []  # (node, concrete value under the witness)
    for v in range(n_vars):
        leaves.append((dag.var(f"x{v}", 256, parent=witness[v] if plant else None), witness[v]))
    for _ in range(4):
        c = _leaf_value(rng)
        leaves.append((dag.const(c, 256), c))
    interior: List[Tuple[int, int]] = []
    ops = _MIX_OPS

    def pick(first: bool):
        if first and interior and len(interior) <= depth:
            return interior[-1]
        pool = interior[-window:]
        if pool and rng.random() < 0.6:
            return pool[int(rng.integers(0, len(pool)))]
        return leaves[int(rng.integers(0, len(leaves)))]

    for _ in range(n_interior):
        # = rng.choice(len(ops), p=probs): numpy draws one double and searches the
        # normalised cumulative sum (side="right") — the same stream, 20x cheaper per call
        kind = ops[bisect.bisect_right(_MIX_CDF, rng.random())]
        a, va = pick(True)
        b, vb = pick(False)
        if kind == "div":
            op = ir.W_UDIV if rng.random() < 0.5 else ir.W_SDIV
        elif kind == "rem":
            op = ir.W_UREM if rng.random() < 0.5 else ir.W_SREM
        elif kind == "addsub":
            op = ir.W_ADD if rng.random() < 0.5 else ir.W_SUB
        elif kind == "logic":
            op = [ir.W_AND, ir.W_OR, ir.W_XOR, ir.W_NOT][int(rng.integers(0, 4))]
        elif kind == "shift":
            op = [ir.W_SHL, ir.W_LSHR, ir.W_ASHR][int(rng.integers(0, 3))]
            # shift amounts: keep them in range half the time so shifts are not all 0
            if rng.random() < 0.5:
                k = int(rng.integers(0, 256))
                b, vb = dag.op(ir.W_AND, 256, b, dag.const(0xFF, 256)), vb & 0xFF
                del k
        elif kind == "itecmp":
            c_op = [ir.B_ULT, ir.B_SLT, ir.B_EQ][int(rng.integers(0, 3))]
            c2, vc2 = pick(False)
            cond = dag.op(c_op, 256, a, c2)
            if c_op == ir.B_ULT:
                cv = va < vc2
            elif c_op == ir.B_EQ:
                cv = va == vc2
            else:
                s = lambda x: x - (1 << 256) if x >> 255 else x
                cv = s(va) < s(vc2)
            node = dag.op(ir.W_ITE, 256, cond, a, b)
            interior.append((node, va if cv else vb))
            continue
        else:
            op = kind
        if op == ir.W_NOT:
            node = dag.op(op, 256, a)
            val = _eval(op, va, 0)
        else:
            node = dag.op(op, 256, a, b)
            val = _eval(op, va, vb)
        interior.append((node, val))

    # root: 2-4 comparisons of late interior values against their planted values
    n_roots = int(rng.integers(2, 5))
    tail = interior[-max(n_roots * 2, 8):]
    for r in range(n_roots):
        node, val = tail[int(rng.integers(0, len(tail)))]
        cmp = int(rng.integers(0, 3))
        if cmp == 0:
            dag.assert_(dag.op(ir.B_EQ, 256, node, dag.const(val, 256)))
        elif cmp == 1:
            dag.assert_(dag.op(ir.B_ULE, 256, node, dag.const(val, 256)))
        else:
            dag.assert_(dag.op(ir.B_ULE, 256, dag.const(val, 256), node))
    prog = lower(dag, seed=(CAND_SEED_BASE ^ dag_id) & 0xFFFFFFFF, name=f"dag{dag_id}")
    return prog, witness


def random_dag_batch(first_id: int, n: int, **kw) -> List[Program]:
    return [random_dag_set(first_id + i, **kw)[0] for i in range(n)]


def random_dag_programs(first_id: int, n: int, plant: bool = False) -> Tuple[List[Program], List[List[int]]]:
    """``random_dag_set(first_id + i, plant=plant)`` for i < n — natively when libpflower.so
    has the generator (pflt_synth: numpy's Philox Generator stream, the DAG builder, the
    planted-value arithmetic and the lowering restated in C++, equal program for program:
    tests/test_synth_native.py), else in Python.  (programs, planted witnesses)."""
    from .smt import native_terms

    got = native_terms.synth_programs(first_id, n, plant, _MIX_CDF) if n else None
    if got is None:
        out = [random_dag_set(first_id + i, plant=plant) for i in range(n)]
        return [p for p, _ in out], [w for _, w in out]
    progs, wit, nv = got
    rows = wit.astype("<u4").tobytes()
    witnesses = [[int.from_bytes(rows[256 * i + 32 * v:256 * i + 32 * v + 32], "little") for v in range(int(nv[i]))]
                 for i in range(n)]
    return progs, witnesses


# ---- Mythril-shaped sets ------------------------------------------------------------
CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA


def calldata_word(dag: Dag, tx: int, offset: int, size_node: int) -> int:
    """CALLDATALOAD(offset) as LASER builds it: Concat of 32 bytes
    If(offset+i <s calldatasize, Select(calldata, offset+i), 0)
    (mythril/laser/ethereum/state/calldata.py:233-246, :47-54).  The array is modelled as
    one free 8-bit variable per concrete index."""
    parts = []
    for i in range(32):
        idx = offset + i
        name = f"{tx}_calldata[{idx}]"
        byte = dag.var(name, 8, ir.VK_CDBYTE, *ir.cdbyte_hints(name))
        cond = dag.op(ir.B_SLT, 256, dag.const(idx, 256), size_node)
        parts.append(dag.op(ir.W_ITE, 8, cond, byte, dag.const(0, 8)))
    acc = parts[0]
    wacc = 8
    for p in parts[1:]:
        acc = dag.op(ir.W_CONCAT, wacc + 8, acc, p, aux=8)
        wacc += 8
    return acc


def mythril_like_set(i: int, n_args: int = 2, parent: Optional[dict] = None) -> Program:
    """A function-dispatch path: selector match, caller in the actor set, argument bounds."""
    rng = np.random.default_rng(1000 + i)
    dag = Dag()
    tx = 1
    size = dag.var(f"{tx}_calldatasize", 256, ir.VK_SMALL, hint0=4 + 32 * n_args + 8)
    dag.assert_(dag.op(ir.B_ULE, 256, dag.const(4 + 32 * n_args, 256), size))
    word0 = calldata_word(dag, tx, 0, size)
    selector = int(rng.integers(0, 1 << 32))
    sel = dag.op(ir.W_LSHR, 256, word0, dag.const(224, 256))
    dag.assert_(dag.op(ir.B_EQ, 256, sel, dag.const(selector, 256)))
    # caller in {CREATOR, ATTACKER, SOMEGUY}
    actors = dag.force_consts((CREATOR, ATTACKER, SOMEGUY))
    caller = dag.var(f"sender_{tx}", 256, ir.VK_ACTOR, hint0=actors, hint1=3)
    eqs = [dag.op(ir.B_EQ, 256, caller, dag.const(a, 256)) for a in (CREATOR, ATTACKER, SOMEGUY)]
    dag.assert_(dag.op(ir.B_OR, 1, dag.op(ir.B_OR, 1, eqs[0], eqs[1]), eqs[2]))
    for k in range(n_args):
        arg = calldata_word(dag, tx, 4 + 32 * k, size)
        bound = int(rng.integers(1, 1 << 16))
        dag.assert_(dag.op(ir.B_ULT, 256, arg, dag.const(bound, 256)))
    value = dag.var(f"call_value{tx}", 256, ir.VK_VALUE)
    dag.assert_(dag.op(ir.B_EQ, 256, value, dag.const(0, 256)))
    return lower(dag, seed=i, name=f"myth{i}")
