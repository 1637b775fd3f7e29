"""Optional z3 back end: the reference's own solver for everything the GPU does not answer.

Used only where z3 is importable (z3-solver ">=4.8.8.0,<=4.13.0.0", reference
requirements.txt:25).  It is absent from this build container, so this module is exercised
only on a z3-bearing host; without it, unanswered objective-free queries report ``unknown``
(mythril/laser/smt/solver/solver.py:91-95 maps solver failures to unknown as well).
"""

from __future__ import annotations

from typing import Dict, List, Optional

from . import terms as T

try:  # pragma: no cover - depends on the host
    import z3  # type: ignore

    HAVE_Z3 = True
except Exception:  # pragma: no cover
    z3 = None
    HAVE_Z3 = False


def available() -> bool:
    return HAVE_Z3


class Converter:  # pragma: no cover - needs z3
    def __init__(self):
        self.memo: Dict[T.Term, object] = {}
        self.funcs: Dict[str, object] = {}

    def __call__(self, t: T.Term):
        r = self.memo.get(t)
        if r is None:
            r = self._conv(t)
            self.memo[t] = r
        return r

    def _conv(self, t: T.Term):
        op, a = t.op, [self(x) for x in t.args]
        if op == "bv":
            return z3.BitVecVal(t.val, t.width)
        if op == "true":
            return z3.BoolVal(True)
        if op == "false":
            return z3.BoolVal(False)
        if op == "var":
            return z3.BitVec(t.val, t.width)
        if op == "bvar":
            return z3.Bool(t.val)
        if op == "array":
            return z3.Array(t.val, z3.BitVecSort(t.sort[1]), z3.BitVecSort(t.sort[2]))
        if op == "K":
            return z3.K(z3.BitVecSort(t.sort[1]), a[0])
        table = {
            "bvadd": lambda: a[0] + a[1], "bvsub": lambda: a[0] - a[1], "bvmul": lambda: a[0] * a[1],
            "bvudiv": lambda: z3.UDiv(a[0], a[1]), "bvurem": lambda: z3.URem(a[0], a[1]),
            "bvsdiv": lambda: a[0] / a[1], "bvsrem": lambda: z3.SRem(a[0], a[1]),
            "bvsmod": lambda: a[0] % a[1], "bvand": lambda: a[0] & a[1], "bvor": lambda: a[0] | a[1],
            "bvxor": lambda: a[0] ^ a[1], "bvshl": lambda: a[0] << a[1],
            "bvlshr": lambda: z3.LShR(a[0], a[1]), "bvashr": lambda: a[0] >> a[1],
            "bvnot": lambda: ~a[0], "bvneg": lambda: -a[0],
            "bvult": lambda: z3.ULT(a[0], a[1]), "bvule": lambda: z3.ULE(a[0], a[1]),
            "bvslt": lambda: a[0] < a[1], "bvsle": lambda: a[0] <= a[1],
            "bvuadd_noovfl": lambda: z3.BVAddNoOverflow(a[0], a[1], False),
            "bvumul_noovfl": lambda: z3.BVMulNoOverflow(a[0], a[1], False),
            "=": lambda: a[0] == a[1], "iff": lambda: a[0] == a[1],
            "and": lambda: z3.And(*a), "or": lambda: z3.Or(*a), "not": lambda: z3.Not(a[0]),
            "xor": lambda: z3.Xor(a[0], a[1]), "ite": lambda: z3.If(a[0], a[1], a[2]),
            "concat": lambda: z3.Concat(*a), "select": lambda: z3.Select(a[0], a[1]),
            "store": lambda: z3.Store(a[0], a[1], a[2]),
        }
        if op in table:
            return table[op]()
        if op == "extract":
            return z3.Extract(t.val[0], t.val[1], a[0])
        if op == "zero_extend":
            return z3.ZeroExt(t.val, a[0])
        if op == "bvexp":
            raise ValueError("bvexp has no z3 counterpart (Mythril uses the Power UF)")
        if op == "apply":
            name, doms = t.val
            f = self.funcs.get(name)
            if f is None:
                f = z3.Function(name, *[z3.BitVecSort(d) for d in doms], z3.BitVecSort(t.width))
                self.funcs[name] = f
            return f(*a)
        raise ValueError(op)


class Z3Internal:  # pragma: no cover - needs z3
    """Internal model backed by a z3 ModelRef: evaluates our terms through the converter."""

    def __init__(self, model, conv: Converter):
        self.m = model
        self.conv = conv

    def decls(self):
        from .model import Decl

        return [Decl(d.name(), ("z3",)) for d in self.m.decls()]

    def __getitem__(self, item):
        for d in self.m.decls():
            if d.name() == item.name():
                return self.m[d]
        return None

    def eval(self, t, model_completion=False):
        return self.m.eval(self.conv(t), model_completion=model_completion)


def check(constraints: List[T.Term], minimize=(), maximize=(), timeout_ms: Optional[int] = None,
          optimize: bool = True):  # pragma: no cover - needs z3
    conv = Converter()
    s = z3.Optimize() if optimize else z3.Solver()
    if timeout_ms:
        s.set(timeout=int(timeout_ms))
    for c in constraints:
        s.add(conv(c))
    for e in minimize:
        s.minimize(conv(e))
    for e in maximize:
        s.maximize(conv(e))
    try:
        r = s.check()
    except z3.Z3Exception:
        r = z3.unknown
    model = Z3Internal(s.model(), conv) if r == z3.sat else None
    return r, model, s
