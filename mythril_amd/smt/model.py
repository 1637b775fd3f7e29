"""Model — mirror of mythril.laser.smt.Model (mythril/laser/smt/model.py:6-59).

Wraps a list of internal models (GPU witnesses here, z3 models when the z3 fallback answered)
and offers the same ``decls()`` / ``__getitem__`` / ``eval(expr, model_completion)`` surface.
Values come back as :class:`BitVecNumVal` / :class:`BoolVal`, which behave like z3's
``BitVecNumRef`` (``as_long()``, comparison with ints) and ``BoolRef`` (truthiness).
"""

from __future__ import annotations

from typing import List, Union

from . import terms as T
from .interp import Witness


class Decl:
    """A declared symbol (z3 FuncDeclRef analogue): name + sort."""

    __slots__ = ("_name", "sort")

    def __init__(self, name: str, sort: tuple):
        self._name = name
        self.sort = sort

    def name(self) -> str:
        return self._name

    def __eq__(self, other):
        return isinstance(other, Decl) and other._name == self._name and other.sort == self.sort

    def __hash__(self):
        return hash((self._name, self.sort))

    def __repr__(self):
        return self._name


def decl_of(t: T.Term) -> Decl:
    if t.op in ("var", "bvar", "array"):
        return Decl(t.val, t.sort)
    if t.op == "apply":
        return Decl(t.val[0], ("fn",) + t.val[1] + (t.width,))
    raise ValueError(f"{t.op} term has no declaration")


# z3-style accessor on terms: x.raw.decl()
T.Term.decl = decl_of  # type: ignore[attr-defined]


class BitVecNumVal:
    __slots__ = ("v", "w")

    def __init__(self, v: int, w: int):
        self.v, self.w = v, w

    def as_long(self) -> int:
        return self.v

    def size(self) -> int:
        return self.w

    def __eq__(self, other):
        if isinstance(other, BitVecNumVal):
            return self.v == other.v
        return self.v == other

    def __hash__(self):
        return hash(self.v)

    def __int__(self):
        return self.v

    def __repr__(self):
        return str(self.v)


class BoolVal:
    __slots__ = ("b",)

    def __init__(self, b: bool):
        self.b = bool(b)

    def __bool__(self):
        return self.b

    def __eq__(self, other):
        return self.b == bool(other)

    def __hash__(self):
        return hash(self.b)

    def __repr__(self):
        return "True" if self.b else "False"


def _as_value(t: T.Term, v):
    return BoolVal(v) if t.is_bool else BitVecNumVal(int(v), t.width)


class WitnessModel:
    """Internal model of a GPU witness (one per satisfied set)."""

    def __init__(self, witness, constraints: List[T.Term]):
        # a Witness, or a function building it: check_sets defers decoding the native
        # lowering's metadata until a model is first read
        self._w = witness
        self.constraints = constraints
        self.origin = "search"   # set by check_sets: "hint" / "first" / "search" / "cache"
        self.parts = None        # check_sets: the buckets' (lowering, values), and the registry
        self.reg = None

    @property
    def w(self) -> Witness:
        if not hasattr(self._w, "ev"):
            self._w = self._w()
        return self._w

    def decls(self) -> List[Decl]:
        out: List[Decl] = []
        seen = set()
        for t in _symbols(self.constraints):
            d = decl_of(t)
            if d not in seen:
                seen.add(d)
                out.append(d)
        return out

    def __getitem__(self, item):
        if isinstance(item, Decl):
            name, sort = item.name(), item.sort
            if sort == T.BOOL:
                return BoolVal(self.w.bools.get(name, False)) if name in self.w.bools else None
            if sort[0] == "bv":
                return BitVecNumVal(self.w.vars[name], sort[1]) if name in self.w.vars else None
            return None
        if isinstance(item, int):
            return self.decls()[item]
        return None

    def eval(self, expression, model_completion: bool = False):
        t = expression.raw if hasattr(expression, "raw") else expression
        return _as_value(t, self.w.ev(t))


def _symbols(constraints: List[T.Term]):
    seen = set()
    stack = list(constraints)
    while stack:
        t = stack.pop()
        if t in seen:
            continue
        seen.add(t)
        if t.op in ("var", "bvar", "array"):
            yield t
        elif t.op == "apply":
            yield t
        stack.extend(t.args)


class Model:
    """Mirror of mythril.laser.smt.Model: a list of internal models."""

    def __init__(self, models: list = None):
        self.raw = models or []

    def decls(self) -> list:
        result = []
        for internal in self.raw:
            result.extend(internal.decls())
        return result

    def __getitem__(self, item):
        for i, internal in enumerate(self.raw):
            try:
                r = internal[item]
                if r is not None:
                    return r
            except IndexError:
                if i == len(self.raw) - 1:
                    raise
                continue
        return None

    def eval(self, expression, model_completion: bool = False) -> Union[None, object]:
        t = expression.raw if hasattr(expression, "raw") else expression
        for i, internal in enumerate(self.raw):
            is_last = i == len(self.raw) - 1
            relevant = False
            try:
                relevant = decl_of(t) in internal.decls()
            except ValueError:
                pass
            if relevant or is_last:
                return internal.eval(t, model_completion)
        return None
