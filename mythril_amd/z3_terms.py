"""z3 AST -> engine terms, cached by AST id (the live-analysis front end).

In a Mythril process every constraint is a z3 AST (``Bool.raw``, mythril/laser/smt/bool.py).
The drop-in ``Optimize`` and the tx-boundary batch (mythril_amd/integration.py) turn them into
:mod:`mythril_amd.smt.terms` by walking the AST directly — no ``sexpr()`` printing and
re-parsing per query.  LASER's constraint lists share almost all of their elements across
states (a fork deep-copies the list and appends one condition, constraints.py:79-88,
instructions.py:1638,1662), so each AST is converted once: the cache maps ``get_id()`` to the
converted term *and keeps the AST itself*, so an id can never be recycled by z3 for a
different AST while its entry exists (z3 reuses the ids of freed ASTs).

Operator semantics are the SMT-LIB2 ones shared with the text reader (mythril_amd/smtlib.py
``apply_named`` / ``apply_indexed``); the z3 declaration kind selects the operator.  Symbols
are declared from the z3 sorts themselves, so an expression over symbols no query has seen
yet converts as well (needed by ``Model.eval(expr, model_completion=True)`` on later
expressions, mythril/support/support_utils.py:63-67).

z3 itself is imported lazily (``z3mod`` may be injected): importing this module never needs z3.
"""

from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

from .lower import LoweringError
from .smt import terms as T
from .smtlib import apply_indexed, apply_named

# z3 declaration kinds (Z3_OP_* constant names) -> SMT-LIB2 operator names
_KIND_NAMES = {
    "Z3_OP_BADD": "bvadd", "Z3_OP_BSUB": "bvsub", "Z3_OP_BMUL": "bvmul",
    "Z3_OP_BSDIV": "bvsdiv", "Z3_OP_BUDIV": "bvudiv", "Z3_OP_BSREM": "bvsrem",
    "Z3_OP_BUREM": "bvurem", "Z3_OP_BSMOD": "bvsmod",
    "Z3_OP_BSDIV_I": "bvsdiv", "Z3_OP_BUDIV_I": "bvudiv", "Z3_OP_BSREM_I": "bvsrem",
    "Z3_OP_BUREM_I": "bvurem", "Z3_OP_BSMOD_I": "bvsmod",
    "Z3_OP_BAND": "bvand", "Z3_OP_BOR": "bvor", "Z3_OP_BXOR": "bvxor", "Z3_OP_BNOT": "bvnot",
    "Z3_OP_BNEG": "bvneg", "Z3_OP_BNAND": "bvnand", "Z3_OP_BNOR": "bvnor",
    "Z3_OP_BXNOR": "bvxnor", "Z3_OP_BCOMP": "bvcomp",
    "Z3_OP_BSHL": "bvshl", "Z3_OP_BLSHR": "bvlshr", "Z3_OP_BASHR": "bvashr",
    "Z3_OP_ULEQ": "bvule", "Z3_OP_SLEQ": "bvsle", "Z3_OP_UGEQ": "bvuge", "Z3_OP_SGEQ": "bvsge",
    "Z3_OP_ULT": "bvult", "Z3_OP_SLT": "bvslt", "Z3_OP_UGT": "bvugt", "Z3_OP_SGT": "bvsgt",
    "Z3_OP_BUMUL_NO_OVFL": "bvumul_noovfl",
    "Z3_OP_CONCAT": "concat", "Z3_OP_EQ": "=", "Z3_OP_IFF": "=", "Z3_OP_DISTINCT": "distinct",
    "Z3_OP_ITE": "ite", "Z3_OP_AND": "and", "Z3_OP_OR": "or", "Z3_OP_NOT": "not",
    "Z3_OP_XOR": "xor", "Z3_OP_IMPLIES": "=>", "Z3_OP_SELECT": "select", "Z3_OP_STORE": "store",
}
_KIND_INDEXED = {
    "Z3_OP_EXTRACT": "extract", "Z3_OP_ZERO_EXT": "zero_extend", "Z3_OP_SIGN_EXT": "sign_extend",
    "Z3_OP_REPEAT": "repeat", "Z3_OP_ROTATE_LEFT": "rotate_left",
    "Z3_OP_ROTATE_RIGHT": "rotate_right",
}


def _z3():
    import z3  # noqa: WPS433 - only on z3-bearing hosts

    return z3


class Z3Converter:
    """Converts z3 ASTs of one z3 context to terms; thread-safe, bounded LRU by AST id."""

    def __init__(self, z3mod=None, max_entries: int = 1 << 20):
        self._z3 = z3mod
        self.max_entries = max_entries
        self._cache: "OrderedDict[int, Tuple[object, T.Term]]" = OrderedDict()
        # term -> one z3 AST it was converted from (the GPU-resident ModelCache evaluates a
        # query's leaf terms under z3 models: mythril_amd/model_cache.py)
        self._rev: Dict[T.Term, object] = {}
        self._lock = threading.Lock()
        self._kinds: Optional[Dict[int, Tuple[str, str]]] = None
        self.hits = 0
        self.misses = 0

    @property
    def z3(self):
        if self._z3 is None:
            self._z3 = _z3()
        return self._z3

    def _kind_table(self) -> Dict[int, Tuple[str, str]]:
        if self._kinds is None:
            z3 = self.z3
            tab: Dict[int, Tuple[str, str]] = {}
            for cname, name in _KIND_NAMES.items():
                if hasattr(z3, cname):
                    tab[getattr(z3, cname)] = ("named", name)
            for cname, name in _KIND_INDEXED.items():
                if hasattr(z3, cname):
                    tab[getattr(z3, cname)] = ("indexed", name)
            self._kinds = tab
        return self._kinds

    def clear(self) -> None:
        with self._lock:
            self._cache.clear()
            self._rev.clear()

    # ---- public -------------------------------------------------------------------------
    def term(self, e) -> T.Term:
        with self._lock:
            return self._convert(e)

    def ast_of(self, t: T.Term):
        """A z3 AST for a term: the AST it was converted from, else (for the leaf terms the
        explicit lowering synthesises — a base-array read below a store chain, a 256-bit
        chunk of a wide UF application — and for bare symbols) one built from its parts and
        kept, so the same term always gets the same AST (a model's ``eval`` then shares its
        subterms across leaves instead of re-walking a fresh copy per call)."""
        with self._lock:
            a = self._rev.get(t)
        if a is not None:
            return a
        z3 = self.z3
        op = t.op
        if op == "select":
            a = z3.Select(self.ast_of(t.args[0]), self.ast_of(t.args[1]))
        elif op == "extract":
            hi, lo = t.val
            a = z3.Extract(hi, lo, self.ast_of(t.args[0]))
        elif op == "var":
            a = z3.BitVec(t.val, t.width)
        elif op == "bvar":
            a = z3.Bool(t.val)
        elif op == "array":
            a = z3.Array(t.val, z3.BitVecSort(t.sort[1]), z3.BitVecSort(t.sort[2]))
        elif op == "bv":
            a = z3.BitVecVal(t.val, t.width)
        else:
            raise LoweringError(f"no z3 AST for a {op} term")
        with self._lock:
            self._store(a, t)
        return a

    def terms(self, es) -> List[T.Term]:
        with self._lock:
            return [self._convert(e) for e in es]

    # ---- walker -------------------------------------------------------------------------
    def _lookup(self, e) -> Optional[T.Term]:
        ent = self._cache.get(e.get_id())
        if ent is None:
            return None
        self._cache.move_to_end(e.get_id())
        return ent[1]

    def _store(self, e, t: T.Term) -> None:
        self._cache[e.get_id()] = (e, t)  # the AST is kept: its id cannot be recycled
        self._rev[t] = e
        if len(self._cache) > self.max_entries:
            _, (old, ot) = self._cache.popitem(last=False)
            if self._rev.get(ot) is old:
                del self._rev[ot]

    def _convert(self, root) -> T.Term:
        hit = self._lookup(root)
        if hit is not None:
            self.hits += 1
            return hit
        # iterative post-order: LASER terms nest deeply (32-byte calldata concatenations,
        # long store chains), beyond Python's recursion limit
        local: Dict[int, T.Term] = {}
        stack = [(root, False)]
        while stack:
            e, expanded = stack.pop()
            eid = e.get_id()
            if eid in local:
                continue
            cached = self._lookup(e)
            if cached is not None:
                local[eid] = cached
                continue
            kids = self._children(e)
            if not expanded and any(k.get_id() not in local for k in kids):
                stack.append((e, True))
                for k in reversed(kids):
                    if k.get_id() not in local:
                        stack.append((k, False))
                continue
            t = self._node(e, [local[k.get_id()] for k in kids])
            local[eid] = t
            self._store(e, t)
            self.misses += 1
        return local[root.get_id()]

    def _children(self, e) -> list:
        z3 = self.z3
        if z3.is_quantifier(e) or not z3.is_app(e):
            raise LoweringError("z3: quantifiers and bound variables are not lowered")
        return [e.arg(i) for i in range(e.num_args())]

    def _sort(self, s) -> tuple:
        z3 = self.z3
        k = s.kind()
        if k == z3.Z3_BOOL_SORT:
            return T.BOOL
        if k == z3.Z3_BV_SORT:
            return T.bv_sort(s.size())
        if k == z3.Z3_ARRAY_SORT:
            d, r = s.domain(), s.range()
            if d.kind() != z3.Z3_BV_SORT or r.kind() != z3.Z3_BV_SORT:
                raise LoweringError("z3: array over non-bit-vector sorts")
            return T.array_sort(d.size(), r.size())
        raise LoweringError(f"z3: unsupported sort {s}")

    def _node(self, e, args: List[T.Term]) -> T.Term:
        z3 = self.z3
        d = e.decl()
        k = d.kind()
        if k == z3.Z3_OP_BNUM:
            return T.const(e.as_long(), e.size())
        if k == z3.Z3_OP_TRUE:
            return T.TRUE
        if k == z3.Z3_OP_FALSE:
            return T.FALSE
        if k == z3.Z3_OP_UNINTERPRETED:
            name = d.name()
            srt = self._sort(e.sort())
            if not args:
                if srt == T.BOOL:
                    return T.boolvar(name)
                if srt[0] == "bv":
                    return T.var(name, srt[1])
                return T.array(name, srt[1], srt[2])
            if srt[0] != "bv":
                raise LoweringError(f"z3: UF {name} with range {srt}")
            return T.apply(name, srt[1], *args)
        if k == z3.Z3_OP_CONST_ARRAY:
            srt = self._sort(e.sort())
            return T.const_array(srt[1], args[0])
        ent = self._kind_table().get(k)
        if ent is None:
            raise LoweringError(f"z3: unsupported operator {d.name()}")
        how, name = ent
        if how == "indexed":
            return apply_indexed(name, [int(p) for p in d.params()], args)
        return apply_named(name, args)


_DEFAULT: Optional[Z3Converter] = None
_DEFAULT_LOCK = threading.Lock()


def converter(z3mod=None) -> Z3Converter:
    """The process-wide converter (Mythril uses z3's main context throughout)."""
    global _DEFAULT
    with _DEFAULT_LOCK:
        if _DEFAULT is None or (z3mod is not None and _DEFAULT._z3 is not z3mod):
            _DEFAULT = Z3Converter(z3mod)
        return _DEFAULT
