"""Hash-consed bit-vector / bool / array terms — the z3-free raw layer behind mythril_amd.smt.

``Term`` plays the role of z3's ``ExprRef`` in the reference facade (mythril/laser/smt/
expression.py:11-72): an immutable, structurally shared node.  Terms whose operands are all
constants are folded at construction (the reference relies on ``z3.simplify`` for that:
``BitVec.symbolic``/``value`` at bitvec.py:44-61, ``Bool.value`` at bool.py:34-46), so a
concrete computation never reaches the GPU.

Sorts: ('bv', w) | ('bool',) | ('array', dom, rng).
"""

from __future__ import annotations

from typing import Dict, Optional, Tuple

BOOL = ("bool",)


def bv_sort(w: int) -> tuple:
    return ("bv", w)


def array_sort(dom: int, rng: int) -> tuple:
    return ("array", dom, rng)


def M(w: int) -> int:
    return (1 << w) - 1


class Term:
    __slots__ = ("op", "sort", "args", "val", "__weakref__")
    _table: Dict[tuple, "Term"] = {}

    def __new__(cls, op: str, sort: tuple, args: Tuple["Term", ...] = (), val=None):
        key = (op, sort, tuple(id(a) for a in args), val)
        t = cls._table.get(key)
        if t is not None:
            return t
        t = object.__new__(cls)
        t.op, t.sort, t.args, t.val = op, sort, tuple(args), val
        cls._table[key] = t
        return t

    # pickling re-interns: a term sent to a lowering worker (or back) is rebuilt through
    # the constructor, so it is the receiving process's canonical node for that structure
    def __reduce__(self):
        return (Term, (self.op, self.sort, self.args, self.val))

    # identity semantics: hash-consing makes structural equality == object identity, so
    # object's own (C-level) __eq__ / __hash__ are the right ones — a Python-level __hash__
    # cost every bucket-key tuple lookup one interpreted call per conjunct

    @property
    def width(self) -> int:
        return self.sort[1] if self.sort[0] == "bv" else 0

    @property
    def is_bool(self) -> bool:
        return self.sort == BOOL

    @property
    def is_const(self) -> bool:
        return self.op in ("bv", "true", "false")

    def size(self) -> int:
        return self.width

    def __repr__(self):
        return to_sexpr(self)


# ---- constructors with constant folding ----------------------------------------------

def const(value: int, w: int) -> Term:
    return Term("bv", bv_sort(w), (), value & M(w))


TRUE = Term("true", BOOL)
FALSE = Term("false", BOOL)


def boolval(b: bool) -> Term:
    return TRUE if b else FALSE


def var(name: str, w: int) -> Term:
    return Term("var", bv_sort(w), (), name)


def boolvar(name: str) -> Term:
    return Term("bvar", BOOL, (), name)


def _sgn(x, w):
    return x - (1 << w) if x >> (w - 1) else x


def _udiv(a, b, w):
    return M(w) if b == 0 else a // b


def _urem(a, b, w):
    return a if b == 0 else a % b


def _sdiv(a, b, w):
    sa, sb = _sgn(a, w), _sgn(b, w)
    if b == 0:
        return 1 if sa < 0 else M(w)
    q = abs(sa) // abs(sb)
    return (q if (sa < 0) == (sb < 0) else -q) & M(w)


def _srem(a, b, w):
    if b == 0:
        return a
    sa, sb = _sgn(a, w), _sgn(b, w)
    r = abs(sa) % abs(sb)
    return (r if sa >= 0 else -r) & M(w)


def _smod(a, b, w):
    if b == 0:
        return a
    return (_sgn(a, w) % _sgn(b, w)) & M(w)


_FOLD2 = {
    "bvadd": lambda a, b, w: (a + b) & M(w),
    "bvsub": lambda a, b, w: (a - b) & M(w),
    "bvmul": lambda a, b, w: (a * b) & M(w),
    "bvudiv": _udiv, "bvurem": _urem, "bvsdiv": _sdiv, "bvsrem": _srem, "bvsmod": _smod,
    "bvand": lambda a, b, w: a & b, "bvor": lambda a, b, w: a | b,
    "bvxor": lambda a, b, w: a ^ b,
    "bvshl": lambda a, b, w: 0 if b >= w else (a << b) & M(w),
    "bvlshr": lambda a, b, w: 0 if b >= w else a >> b,
    "bvashr": lambda a, b, w: ((M(w) if a >> (w - 1) else 0) if b >= w else (_sgn(a, w) >> b) & M(w)),
    "bvexp": lambda a, b, w: pow(a, b, 1 << w),
}
_CMP = {
    "bvult": lambda a, b, w: a < b, "bvule": lambda a, b, w: a <= b,
    "bvslt": lambda a, b, w: _sgn(a, w) < _sgn(b, w), "bvsle": lambda a, b, w: _sgn(a, w) <= _sgn(b, w),
    "bvuadd_noovfl": lambda a, b, w: a + b <= M(w), "bvumul_noovfl": lambda a, b, w: a * b <= M(w),
}


def binop(op: str, a: Term, b: Term) -> Term:
    w = a.width
    if a.op == "bv" and b.op == "bv":
        return const(_FOLD2[op](a.val, b.val, w), w)
    return Term(op, a.sort, (a, b))


def bvnot(a: Term) -> Term:
    return const(~a.val, a.width) if a.op == "bv" else Term("bvnot", a.sort, (a,))


def bvneg(a: Term) -> Term:
    return const(-a.val, a.width) if a.op == "bv" else Term("bvneg", a.sort, (a,))


def cmp(op: str, a: Term, b: Term) -> Term:
    if a.op == "bv" and b.op == "bv":
        return boolval(_CMP[op](a.val, b.val, a.width))
    return Term(op, BOOL, (a, b))


def eq(a: Term, b: Term) -> Term:
    if a is b:
        return TRUE
    if a.is_bool:
        if a.is_const and b.is_const:
            return boolval(a is b)
        return Term("iff", BOOL, (a, b))
    if a.op == "bv" and b.op == "bv":
        return boolval(a.val == b.val)
    return Term("=", BOOL, (a, b))


def extract(hi: int, lo: int, a: Term) -> Term:
    w = hi - lo + 1
    if a.op == "bv":
        return const(a.val >> lo, w)
    if lo == 0 and hi == a.width - 1:
        return a
    return Term("extract", bv_sort(w), (a,), (hi, lo))


def concat(*parts: Term) -> Term:
    if len(parts) == 1:
        return parts[0]
    if all(p.op == "bv" for p in parts):
        v, w = 0, 0
        for p in parts:
            v = (v << p.width) | p.val
            w += p.width
        return const(v, w)
    return Term("concat", bv_sort(sum(p.width for p in parts)), tuple(parts))


def zero_extend(n: int, a: Term) -> Term:
    if n == 0:
        return a
    if a.op == "bv":
        return const(a.val, a.width + n)
    return Term("zero_extend", bv_sort(a.width + n), (a,), n)


def ite(c: Term, a: Term, b: Term) -> Term:
    if c is TRUE:
        return a
    if c is FALSE:
        return b
    if a is b:
        return a
    return Term("ite", a.sort, (c, a, b))


def and_(*args: Term) -> Term:
    out = []
    for a in args:
        if a is FALSE:
            return FALSE
        if a is TRUE:
            continue
        out.append(a)
    if not out:
        return TRUE
    if len(out) == 1:
        return out[0]
    return Term("and", BOOL, tuple(out))


def or_(*args: Term) -> Term:
    out = []
    for a in args:
        if a is TRUE:
            return TRUE
        if a is FALSE:
            continue
        out.append(a)
    if not out:
        return FALSE
    if len(out) == 1:
        return out[0]
    return Term("or", BOOL, tuple(out))


def not_(a: Term) -> Term:
    if a is TRUE:
        return FALSE
    if a is FALSE:
        return TRUE
    if a.op == "not":
        return a.args[0]
    return Term("not", BOOL, (a,))


def xor(a: Term, b: Term) -> Term:
    if a.is_const and b.is_const:
        return boolval((a is TRUE) != (b is TRUE))
    return Term("xor", BOOL, (a, b))


# ---- arrays and uninterpreted functions -------------------------------------------------

def array(name: str, dom: int, rng: int) -> Term:
    return Term("array", array_sort(dom, rng), (), name)


def const_array(dom: int, value: Term) -> Term:
    return Term("K", array_sort(dom, value.width), (value,))


def select(arr: Term, idx: Term) -> Term:
    # fold through stores whose index is provably equal / different
    a = arr
    while True:
        if a.op == "store":
            k = a.args[1]
            if k is idx:
                return a.args[2]
            if k.op == "bv" and idx.op == "bv":
                a = a.args[0]
                continue
            break
        if a.op == "K":
            return a.args[0]
        break
    return Term("select", bv_sort(arr.sort[2]), (arr, idx))


def store(arr: Term, idx: Term, val: Term) -> Term:
    return Term("store", arr.sort, (arr, idx, val))


def apply(fname: str, rng: int, *args: Term) -> Term:
    return Term("apply", bv_sort(rng), tuple(args), (fname, tuple(a.width for a in args)))


# ---- structural hash (stable across processes, unlike Term.__hash__) --------------------
_SHASH: Dict[Term, int] = {}


def struct_hash(t: Term) -> int:
    """32-bit hash of the term's structure (op, sort, value, operands), memoised."""
    import zlib

    r = _SHASH.get(t)
    if r is not None:
        return r
    stack = [t]
    while stack:
        x = stack[-1]
        if x in _SHASH:
            stack.pop()
            continue
        pend = [a for a in x.args if a not in _SHASH]
        if pend:
            stack.extend(pend)
            continue
        stack.pop()
        h = zlib.crc32(repr((x.op, x.sort, x.val)).encode())
        for a in x.args:
            h = zlib.crc32(_SHASH[a].to_bytes(4, "little"), h)
        _SHASH[x] = h
    return _SHASH[t]


# ---- printing (SMT-LIB2-ish, for sexpr()/--solver-log style dumps) --------------------

def to_sexpr(t: Term, _memo: Optional[dict] = None) -> str:
    if t.op == "bv":
        return f"#x{t.val:0{(t.width + 3) // 4}x}" if t.width % 4 == 0 else f"(_ bv{t.val} {t.width})"
    if t.op in ("true", "false"):
        return t.op
    if t.op in ("var", "bvar", "array"):
        return _q(t.val)
    if t.op == "extract":
        return f"((_ extract {t.val[0]} {t.val[1]}) {to_sexpr(t.args[0])})"
    if t.op == "zero_extend":
        return f"((_ zero_extend {t.val}) {to_sexpr(t.args[0])})"
    if t.op == "K":
        return f"((as const (Array (_ BitVec {t.sort[1]}) (_ BitVec {t.sort[2]}))) {to_sexpr(t.args[0])})"
    if t.op == "apply":
        return f"({_q(t.val[0])} " + " ".join(to_sexpr(a) for a in t.args) + ")"
    name = {"iff": "=", "bvexp": "bvexp"}.get(t.op, t.op)
    return f"({name} " + " ".join(to_sexpr(a) for a in t.args) + ")"


def _sort_str(sort: tuple) -> str:
    if sort == BOOL:
        return "Bool"
    if sort[0] == "bv":
        return f"(_ BitVec {sort[1]})"
    return f"(Array (_ BitVec {sort[1]}) (_ BitVec {sort[2]}))"


def _q(name: str) -> str:
    return name if str(name).isidentifier() else f"|{name}|"


def declarations(roots) -> list:
    """``declare-fun`` lines for every free symbol / UF reachable from ``roots`` (z3 order:
    first occurrence)."""
    out, seen, done = [], set(), set()
    stack = list(reversed(list(roots)))
    while stack:
        t = stack.pop()
        if t in done:
            continue
        done.add(t)
        if t.op in ("var", "bvar", "array"):
            if t.val not in seen:
                seen.add(t.val)
                out.append(f"(declare-fun {_q(t.val)} () {_sort_str(t.sort)})")
        elif t.op == "apply":
            name, doms = t.val
            if name not in seen:
                seen.add(name)
                d = " ".join(f"(_ BitVec {w})" for w in doms)
                out.append(f"(declare-fun {_q(name)} ({d}) (_ BitVec {t.width}))")
        stack.extend(reversed(t.args))
    return out
