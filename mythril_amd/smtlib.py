"""SMT-LIB2 reader for Mythril's ``--solver-log`` dumps (``z3.Optimize.sexpr()``).

The reference writes one ``<hash>.smt2`` file per query (mythril/support/model.py:46-57):
``declare-fun`` lines, one ``assert`` per constraint, optional ``minimize``/``maximize``
directives and ``check-sat``.  This reader turns such a file into terms of
:mod:`mythril_amd.smt.terms`, which the engine lowers like any live query.  It understands
the z3 printer's forms: ``let`` bindings (``a!1`` …), ``(_ bvN w)`` / ``#x`` / ``#b``
literals, indexed operators (``(_ extract h l)``, ``(_ zero_extend n)``,
``(_ sign_extend n)``, ``(_ rotate_left n)``, ``(_ repeat n)``), ``(as const (Array …))``,
n-ary ``bvadd``/``bvmul``/``bvand``/``bvor``/``bvxor``/``concat``, z3's internal total
division names (``bvudiv_i`` …), ``bvumul_noovfl``, ``distinct``, ``=>``, and
``|quoted|`` symbols (``|keccak256_512-1|``).
"""

from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

from .lower import LoweringError
from .smt import terms as T

_TOKEN = re.compile(r"\s*(?:(\()|(\))|(\|[^|]*\|)|(\"(?:[^\"]|\"\")*\")|([^\s()|\";]+)|(;[^\n]*))")


def tokenize(text: str):
    pos = 0
    n = len(text)
    while pos < n:
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                return
            raise ValueError(f"smtlib: cannot tokenize at {pos}: {text[pos:pos + 30]!r}")
        pos = m.end()
        if m.group(1):
            yield "("
        elif m.group(2):
            yield ")"
        elif m.group(3):
            yield m.group(3)
        elif m.group(4):
            yield m.group(4)
        elif m.group(5):
            yield m.group(5)


def parse_sexprs(text: str) -> list:
    stack: list = [[]]
    for tok in tokenize(text):
        if tok == "(":
            stack.append([])
        elif tok == ")":
            top = stack.pop()
            stack[-1].append(top)
        else:
            stack[-1].append(tok)
    if len(stack) != 1:
        raise ValueError("smtlib: unbalanced parentheses")
    return stack[0]


def _sym(tok: str) -> str:
    return tok[1:-1] if tok.startswith("|") and tok.endswith("|") else tok


@dataclass
class Query:
    assertions: List[T.Term] = field(default_factory=list)
    minimize: List[T.Term] = field(default_factory=list)
    maximize: List[T.Term] = field(default_factory=list)
    decls: Dict[str, tuple] = field(default_factory=dict)

    @property
    def objective_free(self) -> bool:
        return not self.minimize and not self.maximize


def _sort(s) -> tuple:
    if s == "Bool":
        return T.BOOL
    if isinstance(s, list) and s[:2] == ["_", "BitVec"]:
        return T.bv_sort(int(s[2]))
    if isinstance(s, list) and s and s[0] == "Array":
        d, r = _sort(s[1]), _sort(s[2])
        return T.array_sort(d[1], r[1])
    raise LoweringError(f"smtlib: unsupported sort {s}")


_NARY = {"bvadd": "bvadd", "bvmul": "bvmul", "bvand": "bvand", "bvor": "bvor", "bvxor": "bvxor"}
_BIN = {
    "bvsub": "bvsub", "bvudiv": "bvudiv", "bvurem": "bvurem", "bvsdiv": "bvsdiv",
    "bvsrem": "bvsrem", "bvsmod": "bvsmod", "bvudiv_i": "bvudiv", "bvurem_i": "bvurem",
    "bvsdiv_i": "bvsdiv", "bvsrem_i": "bvsrem", "bvsmod_i": "bvsmod", "bvshl": "bvshl",
    "bvlshr": "bvlshr", "bvashr": "bvashr",
}
_CMPS = {
    "bvult": ("bvult", False), "bvule": ("bvule", False), "bvslt": ("bvslt", False),
    "bvsle": ("bvsle", False), "bvugt": ("bvult", True), "bvuge": ("bvule", True),
    "bvsgt": ("bvslt", True), "bvsge": ("bvsle", True), "bvumul_noovfl": ("bvumul_noovfl", False),
}
# overflow predicates of SMT-LIB 2.7 (newer z3 prints them): name -> (no-overflow form, negate)
_OVFL = {
    "bvuaddo": ("bvuadd_noovfl", True), "bvumulo": ("bvumul_noovfl", True),
    "bvusubo": ("bvult", False),
}


_EVAL, _LET, _RESTORE, _APPLY = range(4)
_UNBOUND = object()


class Reader:
    def __init__(self):
        self.q = Query()
        self.funs: Dict[str, Tuple[List[tuple], tuple]] = {}

    def read(self, text: str) -> Query:
        for cmd in parse_sexprs(text):
            if not isinstance(cmd, list) or not cmd:
                continue
            head = cmd[0]
            if head == "declare-fun":
                name = _sym(cmd[1])
                doms = [_sort(s) for s in cmd[2]]
                rng = _sort(cmd[3])
                self.funs[name] = (doms, rng)
                self.q.decls[name] = (tuple(doms), rng)
            elif head == "declare-const":
                name = _sym(cmd[1])
                self.funs[name] = ([], _sort(cmd[2]))
                self.q.decls[name] = ((), _sort(cmd[2]))
            elif head == "define-fun" and not cmd[2]:
                name = _sym(cmd[1])
                self.funs[name] = ([], _sort(cmd[3]))
                self._defs = getattr(self, "_defs", {})
                self._defs[name] = self.term(cmd[4], {})
            elif head == "assert":
                self.q.assertions.append(self.term(cmd[1], {}))
            elif head == "minimize":
                self.q.minimize.append(self.term(cmd[1], {}))
            elif head == "maximize":
                self.q.maximize.append(self.term(cmd[1], {}))
            # set-info / set-option / check-sat / get-model / exit: ignored
        return self.q

    # ---- terms ---------------------------------------------------------------------------
    def term(self, e, env: Dict[str, T.Term]) -> T.Term:
        """One s-expression as a term, without recursion: z3 prints every shared subterm as a
        nested ``let`` (``a!1`` …), so a large dump nests thousands deep.  An explicit work
        stack evaluates it on the caller's thread at any depth (the recursive
        reader had to re-run on a big-stack thread under a raised process-wide recursion
        limit, which made deep recursion on other threads segfault meanwhile).

        ``let`` is parallel (the bindings see the outer scope) and scoped: the bound names
        are set in one mutable environment for the body and restored after it."""
        env = dict(env)
        vals: List[T.Term] = []
        work: list = [(_EVAL, e)]
        while work:
            kind, x = work.pop()
            if kind == _EVAL:
                if isinstance(x, str):
                    vals.append(self._atom(x, env))
                    continue
                head = x[0]
                if head == "_" and len(x) == 3 and x[1].startswith("bv") and x[1][2:].isdigit():
                    vals.append(T.const(int(x[1][2:]), int(x[2])))  # (_ bvN w) literal
                    continue
                if head == "let":
                    work.append((_LET, x))
                    for binding in reversed(x[1]):
                        work.append((_EVAL, binding[1]))
                    continue
                work.append((_APPLY, x))
                for a in reversed(x[1:]):
                    work.append((_EVAL, a))
            elif kind == _LET:          # the bindings' values are on the stack: the body
                names = [_sym(b[0]) for b in x[1]]
                bound = vals[len(vals) - len(names):]
                del vals[len(vals) - len(names):]
                undo = [(nm, env.get(nm, _UNBOUND)) for nm in names]
                for nm, v in zip(names, bound):
                    env[nm] = v
                work.append((_RESTORE, undo))
                work.append((_EVAL, x[2]))
            elif kind == _RESTORE:      # leave the let's scope
                for nm, old in reversed(x):
                    if old is _UNBOUND:
                        env.pop(nm, None)
                    else:
                        env[nm] = old
            else:                       # _APPLY: the arguments are on the stack
                n = len(x) - 1
                args = vals[len(vals) - n:] if n else []
                del vals[len(vals) - n:]
                head = x[0]
                if isinstance(head, list):
                    vals.append(self._indexed(head, args))
                    continue
                h = _sym(head)
                if h in self.funs:
                    doms, rng = self.funs[h]
                    if rng[0] != "bv":
                        raise LoweringError(f"smtlib: UF {h} with range {rng}")
                    vals.append(T.apply(h, rng[1], *args))
                else:
                    vals.append(apply_named(h, args))
        return vals[0]

    def _atom(self, tok: str, env) -> T.Term:
        s = _sym(tok)
        if s in env:
            return env[s]
        if tok == "true":
            return T.TRUE
        if tok == "false":
            return T.FALSE
        if tok.startswith("#x"):
            return T.const(int(tok[2:], 16), 4 * (len(tok) - 2))
        if tok.startswith("#b"):
            return T.const(int(tok[2:], 2), len(tok) - 2)
        defs = getattr(self, "_defs", {})
        if s in defs:
            return defs[s]
        if s in self.funs:
            doms, rng = self.funs[s]
            if doms:
                raise LoweringError(f"smtlib: {s} used without arguments")
            if rng == T.BOOL:
                return T.boolvar(s)
            if rng[0] == "bv":
                return T.var(s, rng[1])
            return T.array(s, rng[1], rng[2])
        raise LoweringError(f"smtlib: unknown symbol {s}")

    def _indexed(self, head: list, args: List[T.Term]) -> T.Term:
        if head[0] == "_":
            return apply_indexed(head[1], [int(p) for p in head[2:]], args)
        if head[0] == "as" and head[1] == "const":
            srt = _sort(head[2])
            return T.const_array(srt[1], args[0])
        raise LoweringError(f"smtlib: unsupported indexed operator {head}")


def apply_named(h: str, args: List[T.Term]) -> T.Term:
    """An interpreted SMT-LIB2 / z3 operator applied to terms (shared by the text reader and
    the z3-AST walker, mythril_amd/z3_terms.py)."""
    if h in _NARY:
        acc = args[0]
        for a in args[1:]:
            acc = T.binop(_NARY[h], acc, a)
        return acc
    if h in _BIN:
        return T.binop(_BIN[h], args[0], args[1])
    if h == "bvneg":
        return T.bvneg(args[0])
    if h == "bvnot":
        return T.bvnot(args[0])
    if h in _CMPS:
        op, swap = _CMPS[h]
        a, b = (args[1], args[0]) if swap else (args[0], args[1])
        return T.cmp(op, a, b)
    if h in _OVFL:
        # SMT-LIB 2.7 overflow predicates (true iff the operation overflows)
        op, neg = _OVFL[h]
        r = T.cmp(op, args[0], args[1])
        return T.not_(r) if neg else r
    if h == "bvnand":
        return T.bvnot(T.binop("bvand", args[0], args[1]))
    if h == "bvnor":
        return T.bvnot(T.binop("bvor", args[0], args[1]))
    if h == "bvxnor":
        return T.bvnot(T.binop("bvxor", args[0], args[1]))
    if h == "bvcomp":
        return T.ite(T.eq(args[0], args[1]), T.const(1, 1), T.const(0, 1))
    if h == "concat":
        return T.concat(*args)
    if h == "=":
        if len(args) == 2:
            return T.eq(args[0], args[1])
        return T.and_(*[T.eq(args[i], args[i + 1]) for i in range(len(args) - 1)])
    if h == "distinct":
        return T.and_(*[T.not_(T.eq(args[i], args[j]))
                        for i in range(len(args)) for j in range(i + 1, len(args))])
    if h in ("ite", "if"):
        return T.ite(args[0], args[1], args[2])
    if h == "and":
        return T.and_(*args)
    if h == "or":
        return T.or_(*args)
    if h == "not":
        return T.not_(args[0])
    if h == "xor":
        acc = args[0]
        for a in args[1:]:
            acc = T.xor(acc, a)
        return acc
    if h == "=>":
        return T.or_(T.not_(args[0]), args[1])
    if h == "select":
        return T.select(args[0], args[1])
    if h == "store":
        return T.store(args[0], args[1], args[2])
    raise LoweringError(f"smtlib: unsupported operator {h}")


def apply_indexed(op: str, params: List[int], args: List[T.Term]) -> T.Term:
    """``((_ op p...) args)`` — extract / zero_extend / sign_extend / repeat / rotations."""
    if op == "extract":
        return T.extract(params[0], params[1], args[0])
    if op == "zero_extend":
        return T.zero_extend(params[0], args[0])
    if op == "sign_extend":
        n = params[0]
        a = args[0]
        if n == 0:
            return a
        msb = T.extract(a.width - 1, a.width - 1, a)
        fill = T.ite(T.eq(msb, T.const(1, 1)), T.const(-1, n), T.const(0, n))
        return T.concat(fill, a)
    if op == "repeat":
        return T.concat(*([args[0]] * params[0]))
    if op in ("rotate_left", "rotate_right"):
        a, k = args[0], params[0] % args[0].width
        if k == 0:
            return a
        w = a.width
        if op == "rotate_right":
            k = w - k
        return T.concat(T.extract(w - 1 - k, 0, a), T.extract(w - 1, w - k, a))
    raise LoweringError(f"smtlib: unsupported indexed operator {op}")


def read_query(text: str) -> Query:
    """One --solver-log query.  z3 prints shared subterms as nested ``let`` bindings, so a
    large dump nests thousands deep: the reader's term walk is iterative (Reader.term)."""
    return Reader().read(text)


def read_file(path: str) -> Query:
    with open(path) as f:
        return read_query(f.read())
