"""Expression classes mirroring mythril.laser.smt (same names, operators and semantics).

Reference: mythril/laser/smt/{expression,bitvec,bitvec_helper,bool,array,function}.py.
Operator semantics follow the reference exactly — in particular ``<``/``>``/``<=``/``>=``
are *signed* (bitvec.py:138-180), ``/`` is bvsdiv (:96-103), ``>>`` is bvashr (:240-246),
``==``/``!=`` zero-pad the narrower side (:16-22, :182-216), and ``ULE``/``UGE`` are
``Or(ULT, ==)``/``Or(UGT, ==)`` (bitvec_helper.py:86-116).  ``raw`` is a
:class:`~mythril_amd.smt.terms.Term` instead of a z3 AST.
"""

from __future__ import annotations

from typing import Any, List, Optional, Set, Union, cast

from . import terms as T

Annotations = Set[Any]


class Expression:
    def __init__(self, raw: T.Term, annotations: Optional[Annotations] = None):
        self.raw = raw
        if annotations:
            assert isinstance(annotations, set)
        self._annotations = annotations or set()

    @property
    def annotations(self) -> Annotations:
        return self._annotations

    def annotate(self, annotation: Any) -> None:
        self._annotations.add(annotation)

    def simplify(self) -> None:
        """Constant folding happens at construction; nothing left to do."""

    def __repr__(self) -> str:
        return repr(self.raw)

    def size(self):
        return self.raw.size()

    def __hash__(self) -> int:
        return hash(self.raw)

    def get_annotations(self, annotation: Any):
        return list(filter(lambda x: isinstance(x, annotation), self.annotations))


def simplify(expression):
    expression.simplify()
    return expression


class Bool(Expression):
    @property
    def is_false(self) -> bool:
        return self.raw is T.FALSE

    @property
    def is_true(self) -> bool:
        return self.raw is T.TRUE

    @property
    def value(self) -> Union[bool, None]:
        if self.raw is T.TRUE:
            return True
        if self.raw is T.FALSE:
            return False
        return None

    def __eq__(self, other: object) -> "Bool":  # type: ignore
        if isinstance(other, Expression):
            return Bool(T.eq(self.raw, other.raw), self.annotations.union(other.annotations))
        return Bool(T.eq(self.raw, T.boolval(bool(other))), self.annotations)

    def __ne__(self, other: object) -> "Bool":  # type: ignore
        if isinstance(other, Expression):
            return Bool(T.not_(T.eq(self.raw, other.raw)), self.annotations.union(other.annotations))
        return Bool(T.not_(T.eq(self.raw, T.boolval(bool(other)))), self.annotations)

    def __bool__(self) -> bool:
        v = self.value
        return v if v is not None else False

    def substitute(self, original_expression, new_expression):
        from .subst import substitute

        self.raw = substitute(self.raw, original_expression.raw, new_expression.raw)

    def __hash__(self) -> int:
        return hash(self.raw)


def _bv(x, w: int) -> T.Term:
    return x.raw if isinstance(x, BitVec) else T.const(int(x), w)


def _padded(a: T.Term, b: T.Term):
    if a.width == b.width:
        return a, b
    if a.width < b.width:
        return T.zero_extend(b.width - a.width, a), b
    return a, T.zero_extend(a.width - b.width, b)


class BitVec(Expression):
    def size(self) -> int:
        return self.raw.width

    @property
    def symbolic(self) -> bool:
        return self.raw.op != "bv"

    @property
    def value(self) -> Optional[int]:
        return None if self.symbolic else self.raw.val

    def _ann(self, other):
        return self.annotations.union(other.annotations) if isinstance(other, Expression) else self.annotations

    def _bin(self, op, other):
        return BitVec(T.binop(op, self.raw, _bv(other, self.size())), annotations=self._ann(other))

    def __add__(self, other):
        return self._bin("bvadd", other)

    def __sub__(self, other):
        return self._bin("bvsub", other)

    def __mul__(self, other):
        return self._bin("bvmul", other)

    def __truediv__(self, other):
        return self._bin("bvsdiv", other)

    def __and__(self, other):
        return self._bin("bvand", other)

    def __or__(self, other):
        return self._bin("bvor", other)

    def __xor__(self, other):
        return self._bin("bvxor", other)

    def _cmp(self, op, a, b, other):
        return Bool(T.cmp(op, a, b), annotations=self._ann(other))

    def __lt__(self, other):
        o = _bv(other, self.size())
        return self._cmp("bvslt", self.raw, o, other)

    def __gt__(self, other):
        o = _bv(other, self.size())
        return self._cmp("bvslt", o, self.raw, other)

    def __le__(self, other):
        o = _bv(other, self.size())
        return self._cmp("bvsle", self.raw, o, other)

    def __ge__(self, other):
        o = _bv(other, self.size())
        return self._cmp("bvsle", o, self.raw, other)

    def __eq__(self, other) -> Bool:  # type: ignore
        if not isinstance(other, BitVec):
            return Bool(T.eq(self.raw, T.const(int(other), self.size())), annotations=self.annotations)
        a, b = _padded(self.raw, other.raw)
        return Bool(T.eq(a, b), annotations=self._ann(other))

    def __ne__(self, other) -> Bool:  # type: ignore
        if not isinstance(other, BitVec):
            return Bool(T.not_(T.eq(self.raw, T.const(int(other), self.size()))), annotations=self.annotations)
        a, b = _padded(self.raw, other.raw)
        return Bool(T.not_(T.eq(a, b)), annotations=self._ann(other))

    def __lshift__(self, other):
        return self._bin("bvshl", other)

    def __rshift__(self, other):
        return self._bin("bvashr", other)

    def __hash__(self) -> int:
        return hash(self.raw)


# ---- helpers (bitvec_helper.py / bool.py) -------------------------------------------

def _ann(*xs) -> Annotations:
    out: Annotations = set()
    for x in xs:
        if isinstance(x, Expression):
            out = out.union(x.annotations)
    return out


def LShR(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(T.binop("bvlshr", a.raw, b.raw), _ann(a, b))


def UDiv(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(T.binop("bvudiv", a.raw, b.raw), _ann(a, b))


def URem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(T.binop("bvurem", a.raw, b.raw), _ann(a, b))


def SRem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(T.binop("bvsrem", a.raw, b.raw), _ann(a, b))


def SMod(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(T.binop("bvsmod", a.raw, b.raw), _ann(a, b))


def UGT(a: BitVec, b: BitVec) -> Bool:
    return Bool(T.cmp("bvult", b.raw, a.raw), _ann(a, b))


def ULT(a: BitVec, b: BitVec) -> Bool:
    return Bool(T.cmp("bvult", a.raw, b.raw), _ann(a, b))


def UGE(a: BitVec, b: BitVec) -> Bool:
    return Or(UGT(a, b), a == b)


def ULE(a: BitVec, b: BitVec) -> Bool:
    return Or(ULT(a, b), a == b)


def If(a, b, c):
    if not isinstance(a, Bool):
        a = Bool(T.boolval(bool(a)))
    if isinstance(b, BaseArray) and isinstance(c, BaseArray):
        arr = Array.__new__(Array)
        BaseArray.__init__(arr, T.ite(a.raw, b.raw, c.raw))
        return arr
    w = 256
    if isinstance(b, BitVec):
        w = b.size()
    if isinstance(c, BitVec):
        w = c.size()
    bb = b.raw if isinstance(b, BitVec) else T.const(int(b), w)
    cc = c.raw if isinstance(c, BitVec) else T.const(int(c), w)
    return BitVec(T.ite(a.raw, bb, cc), _ann(a, b, c))


def Concat(*args) -> BitVec:
    bvs = args[0] if len(args) == 1 and isinstance(args[0], list) else list(args)
    return BitVec(T.concat(*[b.raw for b in bvs]), _ann(*bvs))


def Extract(high: int, low: int, bv: BitVec) -> BitVec:
    return BitVec(T.extract(high, low, bv.raw), annotations=bv.annotations)


def Sum(*args: BitVec) -> BitVec:
    acc = args[0].raw
    for a in args[1:]:
        acc = T.binop("bvadd", acc, a.raw)
    return BitVec(acc, _ann(*args))


def BVAddNoOverflow(a, b, signed: bool) -> Bool:
    a = a if isinstance(a, BitVec) else BitVec(T.const(int(a), 256))
    b = b if isinstance(b, BitVec) else BitVec(T.const(int(b), 256))
    if signed:
        raise NotImplementedError("signed BVAddNoOverflow is not used by Mythril")
    return Bool(T.cmp("bvuadd_noovfl", a.raw, b.raw))


def BVMulNoOverflow(a, b, signed: bool) -> Bool:
    a = a if isinstance(a, BitVec) else BitVec(T.const(int(a), 256))
    b = b if isinstance(b, BitVec) else BitVec(T.const(int(b), 256))
    if signed:
        raise NotImplementedError("signed BVMulNoOverflow is not used by Mythril")
    return Bool(T.cmp("bvumul_noovfl", a.raw, b.raw))


def BVSubNoUnderflow(a, b, signed: bool) -> Bool:
    a = a if isinstance(a, BitVec) else BitVec(T.const(int(a), 256))
    b = b if isinstance(b, BitVec) else BitVec(T.const(int(b), 256))
    if signed:
        raise NotImplementedError("signed BVSubNoUnderflow is not used by Mythril")
    # unsigned a - b does not underflow  <=>  b <=u a
    return Bool(T.cmp("bvule", b.raw, a.raw))


def _to_bool(x) -> Bool:
    return x if isinstance(x, Bool) else Bool(T.boolval(bool(x)))


def And(*args) -> Bool:
    xs = [_to_bool(a) for a in args]
    return Bool(T.and_(*[x.raw for x in xs]), _ann(*xs))


def Or(*args) -> Bool:
    xs = [_to_bool(a) for a in args]
    return Bool(T.or_(*[x.raw for x in xs]), _ann(*xs))


def Not(a: Bool) -> Bool:
    return Bool(T.not_(a.raw), a.annotations)


def Xor(a: Bool, b: Bool) -> Bool:
    return Bool(T.xor(a.raw, b.raw), _ann(a, b))


def is_true(a: Bool) -> bool:
    return a.raw is T.TRUE


def is_false(a: Bool) -> bool:
    return a.raw is T.FALSE


# ---- arrays and functions (array.py, function.py) ------------------------------------

class BaseArray:
    def __init__(self, raw):
        self.raw = raw

    def __getitem__(self, item: BitVec) -> BitVec:
        if isinstance(item, slice):
            raise ValueError("Instance of BaseArray, does not support getitem with slices")
        return BitVec(T.select(self.raw, item.raw))

    def __setitem__(self, key: BitVec, value: BitVec) -> None:
        self.raw = T.store(self.raw, key.raw, value.raw)

    def substitute(self, original_expression, new_expression):
        from .subst import substitute

        self.raw = substitute(self.raw, original_expression.raw, new_expression.raw)


class Array(BaseArray):
    def __init__(self, name: str, domain: int, value_range: int):
        self.domain = domain
        self.range = value_range
        super().__init__(T.array(name, domain, value_range))


class K(BaseArray):
    def __init__(self, domain: int, value_range: int, value: int):
        self.domain = domain
        self.value = value
        super().__init__(T.const_array(domain, T.const(value, value_range)))


class Function:
    def __init__(self, name: str, domain: List[int], value_range: int):
        self.name = name
        self.domain = list(domain)
        self.range = value_range

    def __call__(self, *items) -> BitVec:
        return BitVec(T.apply(self.name, self.range, *[i.raw for i in items]), _ann(*items))


class _SymbolFactory:
    """symbol_factory (mythril/laser/smt/__init__.py:85-153)."""

    @staticmethod
    def Bool(value: bool, annotations: Optional[Annotations] = None) -> Bool:
        return Bool(T.boolval(bool(value)), annotations)

    @staticmethod
    def BoolSym(name: str, annotations: Optional[Annotations] = None) -> Bool:
        return Bool(T.boolvar(name), annotations)

    @staticmethod
    def BitVecVal(value: int, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(T.const(value, size), annotations)

    @staticmethod
    def BitVecSym(name: str, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(T.var(name, size), annotations)


symbol_factory = _SymbolFactory()
