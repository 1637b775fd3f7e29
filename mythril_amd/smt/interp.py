"""Host-side term evaluation under a GPU witness — the ``Model.eval`` of this engine.

The reference's callers evaluate expressions with ``model.eval(expr, model_completion=True)``
(mythril/laser/smt/model.py:45-59; e.g. analysis/solver.py:185-214 concretises calldata,
callvalue and caller).  A witness found on the GPU is a (set, candidate) index; after
``pf_materialize`` returns the candidate's variable values, this module evaluates any term
under exactly the interpretation the kernel used (same arrays rule, same keccak/UF
interpretation, PF_W_HASH restated below), so host and device agree bit for bit.
"""

from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple

from . import terms as T
from .to_dag import KECCAK_MASK_BITS, Lowered, UFRegistry, salt_of

_KECCAK_RE = re.compile(r"^keccak256_(\d+)(-1)?$")
_M32 = 0xFFFFFFFF


def _philox(c, k0, k1):
    c0, c1, c2, c3 = c
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ c3 ^ k1) & _M32, p0 & _M32
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return c0, c1, c2, c3


def uf_hash(x: int, salt: int) -> int:
    """PF_W_HASH (include/pf_bytecode.h)."""
    xs = [(x >> (32 * i)) & _M32 for i in range(8)]
    h = _philox(tuple(xs[:4]), salt, 0x5BD1E995)
    g = _philox(tuple(xs[4 + i] ^ h[i] for i in range(4)), salt, 0x27D4EB2F)
    return sum(v << (32 * i) for i, v in enumerate(h + g))


def _sgn(x, w):
    return x - (1 << w) if x >> (w - 1) else x


def _chunks(v: int, w: int) -> List[int]:
    out = []
    while w > 0:
        out.append(v & T.M(min(w, 256)))
        v >>= 256
        w -= 256
    return out


class Witness:
    """One satisfying assignment plus the interpretation state to evaluate any term."""

    def __init__(self, lowered: Lowered, values: List[int], registry: UFRegistry):
        self.reg = registry
        self.vars: Dict[str, int] = {}
        self.bools: Dict[str, bool] = {}
        self.reads: Dict[T.Term, int] = {}      # select / inverse-app terms -> their own var value
        for term, val in zip(lowered.var_terms, values):
            if term.op == "var":
                self.vars[term.val] = val
            elif term.op == "bvar":
                self.bools[term.val] = bool(val & 1)
            elif term.op == "extract" and term.args[0].op == "var":
                # one 256-bit chunk of a wider free symbol (to_dag._lower_wide)
                name, lo = term.args[0].val, term.val[1]
                self.vars[name] = self.vars.get(name, 0) | (val << lo)
            else:
                self.reads[term] = val
        self.array_reads = lowered.array_reads
        self.uf_apps = lowered.uf_apps
        self._memo: Dict[T.Term, object] = {}
        self._tables: Optional[Dict[str, Dict[int, int]]] = None   # explicit arrays (planted models)
        self._pos: Optional[Dict[str, Dict[T.Term, int]]] = None
        self._keccak_tables: Dict[int, List[Tuple[int, int]]] = {}

    @classmethod
    def union(cls, parts: List["Witness"], registry: Optional[UFRegistry] = None) -> "Witness":
        """One witness from the witnesses of variable-disjoint buckets
        (mythril_amd/smt/independence.py): symbols, arrays and keccak families never span
        two buckets, so the interpretations merge without overlap."""
        if len(parts) == 1:
            return parts[0]
        w = cls.__new__(cls)
        w.reg = registry if registry is not None else (parts[0].reg if parts else None)
        w.vars, w.bools, w.reads, w.array_reads, w.uf_apps = {}, {}, {}, {}, []
        for p in parts:
            w.vars.update(p.vars)
            w.bools.update(p.bools)
            w.reads.update(p.reads)
            w.array_reads.update(p.array_reads)
            w.uf_apps.extend(p.uf_apps)
        w._memo, w._tables, w._pos, w._keccak_tables = {}, None, None, {}
        w._first = w._building = None
        return w

    # ---- array interpretation: first earlier index with an equal value ------------------
    # A read of base array A at index value iv is the value of the FIRST read of A, in the
    # lowering's lookup order (to_dag.TermLowering._select), whose index evaluates to iv —
    # for a read that is itself one of those entries, the first among the entries up to
    # and including it.  The scan is per read and in order because the index of entry p may
    # itself read A (or another array) through earlier entries (ABI dynamic offsets: a
    # calldata read at an offset read from calldata): a table built up front evaluated
    # those nested reads against an unfinished table (as 0), and the host re-check then
    # rejected witnesses the kernel had rightly found.
    def _entry_pos(self, name: str) -> Dict[T.Term, int]:
        if self._pos is None:
            self._pos = {}
        pos = self._pos.get(name)
        if pos is None:
            pos = {}
            for i, (_, sel) in enumerate(self.array_reads.get(name, ())):
                pos.setdefault(sel, i)
            self._pos[name] = pos
        return pos

    # The scan's answer is the FIRST read of the array, over all of its reads, whose index
    # evaluates to iv: for a read that is one of the entries, its own entry matches, so the
    # first match lies at or before it.  Once every index of an array has been evaluated (by
    # the scan's rules, so nested reads never see an unfinished table) that answer is a dict
    # lookup — a quick-sat leaf or a later query's read then costs O(1), not O(reads).
    _first: Optional[Dict[str, object]] = None     # array -> {index value: value} | False
    _building: Optional[set] = None

    def _first_table(self, name: str, reads):
        if self._first is None:
            self._first, self._building = {}, set()
        tab = self._first.get(name)
        if tab is not None:
            return tab
        if name in self._building:
            return False          # a nested read while the table is being built: scan
        self._building.add(name)
        try:
            tab = {}
            for it, sel in reads:
                v = self._evr(it)
                if v not in tab:
                    tab[v] = self.reads.get(sel, 0)
        except Exception:  # noqa: BLE001 - an index only the scan's early stop avoids: scan
            tab = False
        finally:
            self._building.discard(name)
        self._first[name] = tab
        return tab

    def _array_read(self, arr: T.Term, idx: Optional[T.Term], iv: int) -> int:
        name = arr.val
        reads = self.array_reads.get(name)
        if not reads:
            tabs = self._tables or {}
            return tabs.get(name, {}).get(iv, 0)     # model completion: 0
        tab = self._first_table(name, reads)
        if tab is not False:
            return tab.get(iv, 0)
        last = len(reads) - 1
        if idx is not None:
            r = self._entry_pos(name).get(T.select(arr, idx))
            if r is not None:
                last = r
        for i in range(last + 1):
            it, sel = reads[i]
            if self._evr(it) == iv:
                return self.reads.get(sel, 0)
        return 0

    def tables(self) -> Dict[str, Dict[int, int]]:
        """The arrays as {index value: value} maps (every read's index, first read wins)."""
        out: Dict[str, Dict[int, int]] = {}
        for name, reads in self.array_reads.items():
            tab: Dict[int, int] = {}
            for it, sel in reads:
                iv = self._evr(it)
                if iv not in tab:
                    tab[iv] = self.reads.get(sel, 0)
            out[name] = tab
        for name, tab in (self._tables or {}).items():
            out.setdefault(name, tab)
        return out

    def _select(self, arr: T.Term, iv: int, idx: Optional[T.Term] = None) -> int:
        while True:  # a loop, not recursion: LASER's store chains are thousands deep
            if arr.op == "store":
                if self._evr(arr.args[1]) == iv:
                    return self._evr(arr.args[2])
                arr = arr.args[0]
                continue
            if arr.op == "K":
                return self._evr(arr.args[0])
            if arr.op == "ite":
                arr = arr.args[1] if self._evr(arr.args[0]) else arr.args[2]
                continue
            if arr.op == "array":
                return self._array_read(arr, idx, iv)
            raise ValueError(f"select over {arr.op}")

    # ---- UFs ----------------------------------------------------------------------------
    def _keccak(self, n: int, x: int) -> int:
        spec = self.reg.keccak_for(n)
        if spec is not None and x in spec.concrete:
            return spec.concrete[x]
        h = None
        for c in _chunks(x, n):
            h = uf_hash(c if h is None else h ^ c, salt_of(f"keccak256_{n}"))
        if spec is None or spec.lo is None:
            return h
        return (spec.base + ((h & T.M(KECCAK_MASK_BITS)) << 6)) & T.M(256)

    def _keccak_inv(self, n: int, y: int, term: T.Term) -> int:
        # same lookup order as the lowering: f-applications lowered before this inverse
        # application first, then earlier inverse applications that own a variable
        before = []
        for (fname, args, app) in self.uf_apps:
            if app is term:
                break
            before.append((fname, args, app))
        for (fname, args, app) in before:
            if fname == f"keccak256_{n}":
                x = self._evr(args[0])
                if self._keccak(n, x) == y:
                    return x
        for (fname, args, app) in before:
            if fname == f"keccak256_{n}-1" and app in self.reads and self._evr(args[0]) == y:
                return self.reads[app]
        return self.reads.get(term, 0)

    def _apply(self, t: T.Term) -> int:
        fname = t.val[0]
        m = _KECCAK_RE.match(fname)
        if m:
            n = int(m.group(1))
            a = t.args[0]
            if m.group(2) is not None and a.op == "apply" and a.val[0] == f"keccak256_{n}":
                return self._evr(a.args[0])  # inv(f(x)) = x, as substituted by the lowering
            x = self._evr(a)
            return self._keccak(n, x) if m.group(2) is None else self._keccak_inv(n, x, t)
        if fname == "Power" and len(t.args) == 2 and t.width == 256:
            return self._power(t)
        h = None
        for a in t.args:
            for c in _chunks(self._evr(a), a.width):
                h = uf_hash(c if h is None else h ^ c, salt_of(fname))
        return h & T.M(t.width)

    def _power(self, t: T.Term) -> int:
        """The lowering's Power interpretation (to_dag.TermLowering._power), by value."""
        b, e = self._evr(t.args[0]), self._evr(t.args[1])
        apps = [(args, app) for (fname, args, app) in self.uf_apps if fname == "Power" and len(args) == 2]
        for args, _ in apps:
            if args[0].op == "bv" and args[1].op == "bv" and (args[0].val, args[1].val) == (b, e):
                return pow(b, e, 1 << 256)
        if b == 256:
            return 1 << (8 * (e % 32))
        for args, app in apps:
            if app in self.reads and (self._evr(args[0]), self._evr(args[1])) == (b, e):
                return self.reads[app]
        return 1   # model completion outside the set's applications: a positive value

    # ---- evaluator ------------------------------------------------------------------------
    def leaf_value(self, t: T.Term) -> int:
        """``ev`` of a quick-sat leaf (mythril_amd/model_cache.py: a symbol, a base-array read,
        a UF application), with the two answers that need no evaluation first: a symbol's own
        value, and 0 for a read of an array this witness holds no read of (completion)."""
        op = t.op
        if op == "var":
            return self.vars.get(t.val, 0)
        if op == "bvar":
            return int(self.bools.get(t.val, False))
        if op == "select" and t.args[0].op == "array":
            name = t.args[0].val
            if not self.array_reads.get(name) and name not in (self._tables or ()):
                return 0
        return int(self.ev(t))

    def ev(self, t: T.Term):
        """Value of ``t`` under this witness.  A term nested deeper than Python's recursion
        limit (long and / or / ite chains of a large LASER state) is first evaluated bottom-up
        without recursion — every subterm, in post-order, each from its memoised children —
        and the recursive evaluator then finishes on memo hits."""
        try:
            return self._evr(t)
        except RecursionError:
            self._prefill(t)
            return self._evr(t)

    def _prefill(self, root: T.Term) -> None:
        order, seen, stack = [], set(), [(root, False)]
        while stack:
            t, done = stack.pop()
            if done:
                order.append(t)
                continue
            if t in seen or t in self._memo:
                continue
            seen.add(t)
            stack.append((t, True))
            for a in t.args:
                if a not in seen and a not in self._memo:
                    stack.append((a, False))
        for t in order:
            if t in self._memo:
                continue
            try:
                self._memo[t] = self._ev(t)
            except Exception:  # array-sorted terms, or a value only a lazy branch may need
                pass

    def _evr(self, t: T.Term):
        r = self._memo.get(t)
        if r is not None:
            return r
        r = self._ev(t)
        self._memo[t] = r
        return r

    def _ev(self, t: T.Term):
        op = t.op
        if op == "bv":
            return t.val
        if op == "true":
            return True
        if op == "false":
            return False
        if op == "var":
            return self.vars.get(t.val, 0)          # model completion: 0
        if op == "bvar":
            return self.bools.get(t.val, False)
        w = t.width
        if op in T._FOLD2:
            return T._FOLD2[op](self._evr(t.args[0]), self._evr(t.args[1]), w)
        if op in T._CMP:
            a = t.args[0]
            return bool(T._CMP[op](self._evr(a), self._evr(t.args[1]), a.width))
        if op == "bvnot":
            return ~self._evr(t.args[0]) & T.M(w)
        if op == "bvneg":
            return -self._evr(t.args[0]) & T.M(w)
        if op == "extract":
            hi, lo = t.val
            return (self._evr(t.args[0]) >> lo) & T.M(hi - lo + 1)
        if op == "concat":
            v = 0
            for a in t.args:
                v = (v << a.width) | self._evr(a)
            return v
        if op == "zero_extend":
            return self._evr(t.args[0])
        if op == "ite":
            return self._evr(t.args[1]) if self._evr(t.args[0]) else self._evr(t.args[2])
        if op == "select":
            return self._select(t.args[0], self._evr(t.args[1]), t.args[1])
        if op == "apply":
            return self._apply(t)
        if op == "=":
            return self._evr(t.args[0]) == self._evr(t.args[1])
        if op == "iff":
            return bool(self._evr(t.args[0])) == bool(self._evr(t.args[1]))
        if op == "and":
            return all(self._evr(a) for a in t.args)
        if op == "or":
            return any(self._evr(a) for a in t.args)
        if op == "not":
            return not self._evr(t.args[0])
        if op == "xor":
            return bool(self._evr(t.args[0])) != bool(self._evr(t.args[1]))
        raise ValueError(f"cannot evaluate {op}")
