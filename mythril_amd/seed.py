"""Constraint-directed hint models: the parent values the candidate generator mutates.

Uniform 256-bit candidates essentially never satisfy ``==`` constraints (hard
part 3): a function-selector check over four calldata bytes, ``caller == owner`` or
``call_value == 0`` are each a 2^-32..2^-256 event for a random candidate.  The reference
side-steps nothing here — every such query goes to z3 (mythril/support/model.py:99-117).
This pass reads the lowered DAG (mythril_amd.lower.Dag) and derives, per free variable, a
*hint value* by propagating the asserted roots backwards:

* ``x == c`` through concat / extract / zero-extend / shifts and divisions by constants /
  and / or / xor / add / sub / mul-by-odd constants / not / neg, down to the variables
  (the LASER calldata word is a 32-way concat of ``ite(i <s size, cd[i], 0)`` bytes,
  mythril/laser/ethereum/state/calldata.py:233-246; the selector test is an extract or a
  division of that word, instructions.py:506-520,563-580,722-745);
* ``x <u c``, ``c <=u x``, signed forms: intervals on variables, a representative point on
  compound terms;
* disjunctions (the actor set ``Or(caller == a_i)``, transaction/symbolic.py:215) and
  ``ite`` branches are choices, taken in order, skipping alternatives that contradict what
  is already fixed; a choice that already holds under the current hints is left alone;
* a final repair loop re-asserts every root that still evaluates false, overriding.

The hint model is handed to the generator as the parent model: candidate 0 *is* the hint
model, and the odd candidates are few-variable mutations of it (include/pf_bytecode.h,
neighbourhood candidates).  Hints never decide anything: the GPU evaluates every candidate
exactly and every witness is re-checked on the host.  A caller-supplied parent model (the
parent state's z3 model) seeds the bits no constraint fixes.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from . import ir
from .lower import K_BCONST, K_BVAR, K_CONST, K_VAR, Dag
from .smt.interp import uf_hash
from .smt.terms import _FOLD2

M = ir.mask

_WB = {
    ir.W_ADD: _FOLD2["bvadd"], ir.W_SUB: _FOLD2["bvsub"], ir.W_MUL: _FOLD2["bvmul"],
    ir.W_UDIV: _FOLD2["bvudiv"], ir.W_UREM: _FOLD2["bvurem"], ir.W_SDIV: _FOLD2["bvsdiv"],
    ir.W_SREM: _FOLD2["bvsrem"], ir.W_SMOD: _FOLD2["bvsmod"], ir.W_AND: _FOLD2["bvand"],
    ir.W_OR: _FOLD2["bvor"], ir.W_XOR: _FOLD2["bvxor"], ir.W_SHL: _FOLD2["bvshl"],
    ir.W_LSHR: _FOLD2["bvlshr"], ir.W_ASHR: _FOLD2["bvashr"], ir.W_EXP: _FOLD2["bvexp"],
}


def _sgn(x: int, w: int) -> int:
    return x - (1 << w) if x >> (w - 1) else x


_BC = {
    ir.B_EQ: lambda a, b, w: a == b, ir.B_ULT: lambda a, b, w: a < b,
    ir.B_ULE: lambda a, b, w: a <= b,
    ir.B_SLT: lambda a, b, w: _sgn(a, w) < _sgn(b, w),
    ir.B_SLE: lambda a, b, w: _sgn(a, w) <= _sgn(b, w),
    ir.B_UADD_NOOVF: lambda a, b, w: a + b <= M(w),
    ir.B_UMUL_NOOVF: lambda a, b, w: a * b <= M(w),
}


class _Conflict(Exception):
    pass


class Seeder:
    """Backward propagation of root desires over one Dag (see module docstring)."""

    MAX_CHOICES = 4096
    REPAIR_ROUNDS = 4

    def __init__(self, dag: Dag, soft: Optional[Sequence[Optional[int]]] = None):
        self.dag = dag
        self.nodes = dag.nodes
        nv = len(dag.vars)
        self.soft = [(v if v is not None else 0) for v in (soft or [None] * nv)]
        self.bits: Dict[int, Tuple[int, int]] = {}     # var -> (value, known mask)
        self.rng: Dict[int, Tuple[int, int]] = {}      # var -> [lo, hi] unsigned
        self.queue: List[Tuple[int, bool]] = []        # deferred (bool node, wanted) choices
        self.force = False
        self._memo: Dict[int, int] = {}
        # users of every node, and the leaf node of every variable: a hint change only
        # invalidates the memoised values above the variable it touches
        self._users: List[List[int]] = [[] for _ in self.nodes]
        self._leaf: Dict[int, List[int]] = {}
        for i, nd in enumerate(self.nodes):
            for a in set(nd.args):
                self._users[a].append(i)
            if nd.kind in (K_VAR, K_BVAR):
                self._leaf.setdefault(nd.aux, []).append(i)

    # ---- current hint model ------------------------------------------------------------
    def value_of_var(self, v: int) -> int:
        w = self.dag.vars[v].width
        val, msk = self.bits.get(v, (0, 0))
        x = (self.soft[v] & ~msk | val) & M(w)
        lohi = self.rng.get(v)
        if lohi is not None and not (lohi[0] <= x <= lohi[1]):
            if msk == 0:
                x = lohi[0]
            else:  # keep the fixed bits, clear the free ones, then lift into the interval
                y = val & M(w)
                if y < lohi[0]:
                    free = ~msk & M(w)
                    y = (y | (lohi[0] & free)) & M(w)
                x = y if lohi[0] <= y <= lohi[1] else x
        return x

    def ev(self, n: int):
        """Value of node n under the current hint model (memoised until a hint changes)."""
        memo, nodes = self._memo, self.nodes
        if n in memo:
            return memo[n]
        stack = [n]
        while stack:
            i = stack[-1]
            if i in memo:
                stack.pop()
                continue
            nd = nodes[i]
            pend = [a for a in nd.args if a not in memo]
            if pend:
                stack.extend(pend)
                continue
            stack.pop()
            memo[i] = self._ev1(nd, [memo[a] for a in nd.args])
        return memo[n]

    def _ev1(self, nd, a):
        k, w = nd.kind, nd.width
        if k == K_VAR:
            return self.value_of_var(nd.aux)
        if k == K_CONST:
            return nd.aux & M(w)
        if k == K_BCONST:
            return bool(nd.aux)
        if k == K_BVAR:
            return bool(self.value_of_var(nd.aux) & 1)
        if k in _WB:
            return _WB[k](a[0], a[1], w) & M(w)
        if k in _BC:
            return bool(_BC[k](a[0], a[1], w))
        if k == ir.W_NOT:
            return ~a[0] & M(w)
        if k == ir.W_NEG:
            return -a[0] & M(w)
        if k == ir.W_MOV:
            return a[0] & M(w)
        if k == ir.W_EXTRACT:
            return (a[0] >> nd.aux) & M(w)
        if k == ir.W_CONCAT:
            return ((a[0] << nd.aux) | a[1]) & M(w)
        if k == ir.W_SEXT:
            x = a[0] & M(nd.aux)
            return (x - (1 << nd.aux) if x >> (nd.aux - 1) else x) & M(w)
        if k == ir.W_ITE:
            return a[1] if a[0] else a[2]
        if k == ir.W_HASH:
            return uf_hash(a[0], nd.aux) & M(w)
        if k == ir.B_AND:
            return a[0] and a[1]
        if k == ir.B_OR:
            return a[0] or a[1]
        if k == ir.B_XOR:
            return a[0] != a[1]
        if k == ir.B_NOT:
            return not a[0]
        if k == ir.B_ITE:
            return a[1] if a[0] else a[2]
        raise ValueError(f"seed: cannot evaluate {k}")

    def _changed(self, v: Optional[int] = None):
        if v is None:
            self._memo.clear()
            return
        memo, users = self._memo, self._users
        stack = [i for i in self._leaf.get(v, ()) if i in memo]
        while stack:
            i = stack.pop()
            memo.pop(i, None)
            for u in users[i]:
                if u in memo:
                    stack.append(u)

    # ---- variable-level desires ----------------------------------------------------------
    def _set_bits(self, v: int, val: int, msk: int):
        w = self.dag.vars[v].width
        msk &= M(w)
        val &= msk
        if not msk:
            return
        old_v, old_m = self.bits.get(v, (0, 0))
        if (old_v ^ val) & old_m & msk:
            if not self.force:
                raise _Conflict
            old_v &= ~msk
        nv, nm = (old_v & ~msk) | val, old_m | msk
        if (nv, nm) != (old_v, old_m):
            self.bits[v] = (nv, nm)
            self._changed(v)

    def _set_range(self, v: int, lo: int, hi: int):
        olo, ohi = self.rng.get(v, (0, M(self.dag.vars[v].width)))
        nlo, nhi = max(lo, olo), min(hi, ohi)
        if nlo > nhi:
            if not self.force:
                raise _Conflict
            nlo, nhi = lo, hi
        if (nlo, nhi) != (olo, ohi) or v not in self.rng:
            self.rng[v] = (nlo, nhi)
            self._changed(v)

    def _const(self, n: int) -> Optional[int]:
        nd = self.nodes[n]
        return nd.aux & M(nd.width) if nd.kind == K_CONST else None

    # ---- W desires: node value has bits `val` on `msk` -----------------------------------
    def want_val(self, n: int, val: int, msk: int):
        nd = self.nodes[n]
        k, w = nd.kind, nd.width
        msk &= M(w)
        val &= msk
        if not msk:
            return
        if k == K_VAR:
            self._set_bits(nd.aux, val, msk)
            return
        if k == K_CONST:
            if (nd.aux ^ val) & msk:
                raise _Conflict
            return
        a = nd.args
        full = msk == M(w)
        if k == ir.W_CONCAT:
            wl = nd.aux
            self.want_val(a[1], val & M(wl), msk & M(wl))
            self.want_val(a[0], val >> wl, msk >> wl)
        elif k == ir.W_EXTRACT:
            self.want_val(a[0], val << nd.aux, msk << nd.aux)
        elif k in (ir.W_MOV, ir.W_SEXT):
            ws = self.nodes[a[0]].width if k == ir.W_MOV else nd.aux
            if k == ir.W_MOV and (val >> ws):
                raise _Conflict
            self.want_val(a[0], val & M(ws), msk & M(ws))
        elif k == ir.W_ITE:
            self._choice_w(n, val, msk)
        elif k == ir.W_NOT:
            self.want_val(a[0], ~val, msk)
        elif k == ir.W_NEG and full:
            self.want_val(a[0], -val, msk)
        elif k in (ir.W_LSHR, ir.W_SHL, ir.W_UDIV):
            c = self._const(a[1])
            if c is None:
                if k == ir.W_UDIV:
                    return
                # a shift by a computed amount (a window lookup's byte, to_dag._window):
                # propagate through the amount's current value
                c = self.ev(a[1])
            if k == ir.W_UDIV:
                if c == 0:
                    return
                if c & (c - 1):  # general divisor: a in [T*c, T*c + c - 1]
                    if full:
                        self.want_val(a[0], val * c, M(w))
                    return
                c = c.bit_length() - 1
            if c >= w:
                if val & msk:
                    raise _Conflict
                return
            if k == ir.W_SHL:
                if val & msk & M(c):
                    raise _Conflict
                self.want_val(a[0], val >> c, msk >> c)
            else:
                if (val & msk) >> (w - c):
                    raise _Conflict
                self.want_val(a[0], val << c, msk << c)
        elif k in (ir.W_AND, ir.W_OR, ir.W_XOR, ir.W_ADD, ir.W_SUB, ir.W_MUL):
            c0, c1 = self._const(a[0]), self._const(a[1])
            if c0 is None and c1 is None:
                self._eval_propagate(n, val, msk)
                return
            x, c = (a[0], c1) if c1 is not None else (a[1], c0)
            if k == ir.W_AND:
                if val & ~c & msk:
                    raise _Conflict
                self.want_val(x, val & c, msk & c)
            elif k == ir.W_OR:
                if ~val & c & msk:
                    raise _Conflict
                self.want_val(x, val & ~c, msk & ~c)
            elif k == ir.W_XOR:
                self.want_val(x, val ^ c, msk)
            else:
                lo_run = (msk + 1) & msk == 0   # msk is a run of low bits
                if not lo_run:
                    return
                wl = msk.bit_length()
                if k == ir.W_ADD:
                    self.want_val(x, val - c, msk)
                elif k == ir.W_SUB:
                    self.want_val(x, (val + c) if x == a[0] else (c - val), msk)
                elif c & 1:  # W_MUL by an odd constant: multiply by its inverse mod 2^wl
                    self.want_val(x, val * pow(c, -1, 1 << wl), msk)

    def _eval_propagate(self, n: int, val: int, msk: int):
        """x op y = T with neither side constant: solve for one side given the other's
        current hint value (invertible ops only)."""
        nd = self.nodes[n]
        if msk != M(nd.width):
            return
        k, (x, y) = nd.kind, nd.args
        w = nd.width
        for tgt, other in ((x, y), (y, x)):
            o = self.ev(other)
            if k == ir.W_ADD:
                need = val - o
            elif k == ir.W_XOR:
                need = val ^ o
            elif k == ir.W_SUB:
                need = (val + o) if tgt == x else (o - val)
            else:
                return
            if self._has_var(tgt):
                self._try(lambda: self.want_val(tgt, need & M(w), M(w)))
                if self.ev(n) == val:
                    return

    def _has_var(self, n: int) -> bool:
        stack, seen = [n], set()
        while stack:
            i = stack.pop()
            if i in seen:
                continue
            seen.add(i)
            nd = self.nodes[i]
            if nd.kind == K_VAR or nd.kind == K_BVAR:
                return True
            stack.extend(nd.args)
        return False

    # ---- W interval desires ---------------------------------------------------------------
    def want_range(self, n: int, lo: int, hi: int):
        nd = self.nodes[n]
        w = nd.width
        lo, hi = max(lo, 0), min(hi, M(w))
        if lo > hi:
            raise _Conflict
        cur = self.ev(n)
        if nd.kind == K_VAR:
            self._set_range(nd.aux, lo, hi)
            return
        if lo <= cur <= hi:
            return
        if nd.kind == K_CONST:
            raise _Conflict
        if nd.kind == ir.W_MOV:
            ws = self.nodes[nd.args[0]].width
            self.want_range(nd.args[0], lo, min(hi, M(ws)))
            return
        if nd.kind == ir.W_ITE:
            c, a, b = nd.args
            self._alternatives([
                lambda: (self.want_bool(c, True), self.want_range(a, lo, hi)),
                lambda: (self.want_bool(c, False), self.want_range(b, lo, hi)),
            ])
            return
        if nd.kind in (ir.W_ADD, ir.W_SUB):
            c1 = self._const(nd.args[1])
            if c1 is not None and (nd.kind == ir.W_ADD or True):
                d = c1 if nd.kind == ir.W_SUB else -c1
                nlo, nhi = lo + d, hi + d
                if 0 <= nlo and nhi <= M(w):
                    self.want_range(nd.args[0], nlo, nhi)
                    return
        self.want_val(n, lo, M(w))  # a representative point

    def want_srange(self, n: int, slo: int, shi: int):
        """Signed interval [slo, shi] (Python ints) on a w-bit node."""
        w = self.nodes[n].width
        slo, shi = max(slo, -(1 << (w - 1))), min(shi, (1 << (w - 1)) - 1)
        if slo > shi:
            raise _Conflict
        if slo >= 0:
            self.want_range(n, slo, shi)
        elif shi < 0:
            self.want_range(n, slo + (1 << w), shi + (1 << w))
        else:  # straddles zero: prefer the small non-negative part
            self._alternatives([lambda: self.want_range(n, 0, shi),
                                lambda: self.want_range(n, slo + (1 << w), M(w))])

    # ---- Bool desires ----------------------------------------------------------------------
    def want_bool(self, n: int, v: bool):
        nd = self.nodes[n]
        k = nd.kind
        if k == K_BCONST:
            if bool(nd.aux) != v:
                raise _Conflict
            return
        if k == K_BVAR:
            self._set_bits(nd.aux, int(v), 1)
            return
        a = nd.args
        if k == ir.B_NOT:
            self.want_bool(a[0], not v)
        elif k == ir.B_AND and v or k == ir.B_OR and not v:
            self.want_bool(a[0], v)
            self.want_bool(a[1], v)
        elif k in (ir.B_AND, ir.B_OR, ir.B_XOR, ir.B_ITE):
            self.queue.append((n, v))
        elif k == ir.B_EQ:
            self._want_eq(n, v)
        elif k in (ir.B_ULT, ir.B_ULE, ir.B_SLT, ir.B_SLE):
            self._want_cmp(n, v)
        elif k in (ir.B_UADD_NOOVF, ir.B_UMUL_NOOVF) and not v:
            x, y = a
            c = self._const(y)
            if c:
                need = (1 << nd.width) - c if k == ir.B_UADD_NOOVF else -(-(1 << nd.width) // c)
                self.want_range(x, need, M(nd.width))

    def _want_eq(self, n: int, v: bool):
        nd = self.nodes[n]
        x, y = nd.args
        w = nd.width
        cx, cy = self._const(x), self._const(y)
        if v:
            if cy is not None:
                self.want_val(x, cy, M(w))
            elif cx is not None:
                self.want_val(y, cx, M(w))
            else:
                self.queue.append((n, v))
            return
        if self.ev(n) is False:
            return
        if cy is not None or cx is not None:
            t, c = (x, cy) if cy is not None else (y, cx)
            tn = self.nodes[t]
            if tn.kind == ir.W_ITE:
                cc, p, q = tn.args
                cp, cq = self._const(p), self._const(q)
                if cp is not None and cp != c:
                    self.want_bool(cc, True)
                    return
                if cq is not None and cq != c:
                    self.want_bool(cc, False)
                    return
            self.queue.append((n, v))

    def _want_cmp(self, n: int, v: bool):
        nd = self.nodes[n]
        k, (x, y), w = nd.kind, nd.args, nd.width
        if not v:  # not (x < y) == y <= x ; not (x <= y) == y < x
            k = {ir.B_ULT: ir.B_ULE, ir.B_ULE: ir.B_ULT, ir.B_SLT: ir.B_SLE, ir.B_SLE: ir.B_SLT}[k]
            x, y = y, x
        strict = k in (ir.B_ULT, ir.B_SLT)
        signed = k in (ir.B_SLT, ir.B_SLE)
        cx, cy = self._const(x), self._const(y)
        if cx is None and cy is None:
            self.queue.append((n, v))
            return
        if signed:
            top, bot = (1 << (w - 1)) - 1, -(1 << (w - 1))
            if cy is not None:
                self.want_srange(x, bot, _sgn(cy, w) - (1 if strict else 0))
            else:
                self.want_srange(y, _sgn(cx, w) + (1 if strict else 0), top)
        else:
            if cy is not None:
                self.want_range(x, 0, cy - (1 if strict else 0))
            else:
                self.want_range(y, cx + (1 if strict else 0), M(w))

    # ---- choices ------------------------------------------------------------------------------
    def _choice_w(self, n: int, val: int, msk: int):
        c, a, b = self.nodes[n].args
        ca, cb = self._const(a), self._const(b)
        alt_a = lambda: (self.want_bool(c, True), self.want_val(a, val, msk))
        alt_b = lambda: (self.want_bool(c, False), self.want_val(b, val, msk))
        cur = bool(self.ev(c))
        if (self.ev(n) ^ val) & msk == 0:
            # already right under the current hints: pin the branch that produces it
            self._alternatives([alt_a, alt_b] if cur else [alt_b, alt_a])
        elif cb is not None and (cb ^ val) & msk == 0 and not (ca is not None and (ca ^ val) & msk == 0):
            self._alternatives([alt_b, alt_a])
        elif ca is not None and (ca ^ val) & msk == 0:
            self._alternatives([alt_a, alt_b])
        else:
            # least change first: keep the branch the condition selects now (for the ite
            # chains of array reads that is "no alias" — index equalities stay false)
            self._alternatives([alt_a, alt_b] if cur else [alt_b, alt_a])

    def _snapshot(self):
        return dict(self.bits), dict(self.rng), len(self.queue)

    def _restore(self, snap):
        bits, rng = snap[0], snap[1]
        touched = {v for v in set(self.bits) | set(bits) if self.bits.get(v) != bits.get(v)}
        touched |= {v for v in set(self.rng) | set(rng) if self.rng.get(v) != rng.get(v)}
        self.bits, self.rng = dict(bits), dict(rng)
        del self.queue[snap[2]:]
        for v in touched:
            self._changed(v)

    def _try(self, fn) -> bool:
        snap = self._snapshot()
        try:
            fn()
            return True
        except _Conflict:
            self._restore(snap)
            return False

    def _alternatives(self, alts):
        for alt in alts:
            if self._try(alt):
                return
        if self.force and alts:
            alts[0]()
            return
        raise _Conflict

    def _resolve(self, n: int, v: bool):
        if self.ev(n) == v:
            return
        nd = self.nodes[n]
        k, a = nd.kind, nd.args
        if k in (ir.B_AND, ir.B_OR):
            # falsify one conjunct / satisfy one disjunct, over the flattened tree (the
            # actor set Or(Or(c == a0, c == a1), c == a2) is one three-way choice)
            leaves, stack = [], [n]
            while stack:
                i = stack.pop()
                if self.nodes[i].kind == k:
                    stack.extend(reversed(self.nodes[i].args))
                else:
                    leaves.append(i)
            self._alternatives([(lambda x: lambda: self.want_bool(x, v))(x) for x in leaves])
        elif k == ir.B_XOR:
            self._alternatives([lambda: (self.want_bool(a[0], v), self.want_bool(a[1], False)),
                                lambda: (self.want_bool(a[0], not v), self.want_bool(a[1], True))])
        elif k == ir.B_ITE:
            c, p, q = a
            self._alternatives([lambda: (self.want_bool(c, True), self.want_bool(p, v)),
                                lambda: (self.want_bool(c, False), self.want_bool(q, v))])
        elif k == ir.B_EQ:
            x, y = a
            w = nd.width
            if v:
                self.want_eqw(x, y)
            else:  # x != y: move the lowest bit of whichever side can move
                vx, vy = self.ev(x), self.ev(y)
                self._alternatives([lambda: self.want_val(x, vx ^ 1, M(w)),
                                    lambda: self.want_val(y, vy ^ 1, M(w)),
                                    lambda: self.want_val(x, vx ^ (1 << (w - 1)), M(w))])
        elif k in (ir.B_ULT, ir.B_ULE, ir.B_SLT, ir.B_SLE):
            x, y = a
            w = nd.width
            vx, vy = self.ev(x), self.ev(y)
            if not v:
                k = {ir.B_ULT: ir.B_ULE, ir.B_ULE: ir.B_ULT, ir.B_SLT: ir.B_SLE, ir.B_SLE: ir.B_SLT}[k]
                x, y, vx, vy = y, x, vy, vx
            strict = 1 if k in (ir.B_ULT, ir.B_SLT) else 0
            if k in (ir.B_ULT, ir.B_ULE):
                self._alternatives([lambda: self.want_range(x, 0, vy - strict),
                                    lambda: self.want_range(y, vx + strict, M(w))])
            else:
                self._alternatives([lambda: self.want_srange(x, -(1 << (w - 1)), _sgn(vy, w) - strict),
                                    lambda: self.want_srange(y, _sgn(vx, w) + strict, (1 << (w - 1)) - 1)])
        else:
            self.want_bool(n, v)

    def want_eqw(self, x: int, y: int, depth: int = 0):
        """Make W nodes x and y equal: constants pin the other side; two applications of
        the same operator (same aux / width) are made equal argument-wise (congruence —
        sufficient for any function, and what a keccak mapping-slot equality needs:
        keccak(caller . slot) == keccak(key . slot), keccak_function_manager.py:95-114);
        otherwise one side's current value is copied into the other."""
        if x == y or self.ev(x) == self.ev(y):
            return
        w = self.nodes[x].width
        cx, cy = self._const(x), self._const(y)
        if cy is not None:
            self.want_val(x, cy, M(w))
            return
        if cx is not None:
            self.want_val(y, cx, M(w))
            return
        nx, ny = self.nodes[x], self.nodes[y]
        alts = []
        if (depth < 8 and nx.kind == ny.kind and nx.aux == ny.aux and nx.width == ny.width
                and len(nx.args) == len(ny.args) and nx.kind not in (K_VAR, K_CONST)):
            def congruence():
                for a, b in zip(nx.args, ny.args):
                    if a == b:
                        continue
                    if self.nodes[a].is_bool:
                        self.want_bool(a, bool(self.ev(b))) if self._const(b) is None else None
                    else:
                        self.want_eqw(a, b, depth + 1)
            alts.append(congruence)
        vx, vy = self.ev(x), self.ev(y)
        alts.append(lambda: self.want_val(x, vy, M(w)))
        alts.append(lambda: self.want_val(y, vx, M(w)))
        self._alternatives(alts)

    def _drain(self):
        steps = 0
        while self.queue and steps < self.MAX_CHOICES:
            n, v = self.queue.pop(0)
            steps += 1
            if not self._try(lambda: self._resolve(n, v)):
                continue

    # ---- driver -------------------------------------------------------------------------------
    def run(self) -> List[int]:
        roots = list(dict.fromkeys(self.dag.roots))
        for r in roots:                      # deterministic desires first
            self._try(lambda: self.want_bool(r, True))
        self._drain()                        # then the choices, in order
        for _ in range(self.REPAIR_ROUNDS):  # repair what still fails, overriding
            bad = [r for r in roots if not self.ev(r)]
            if not bad:
                break
            self.force = True
            for r in bad:
                try:
                    self.want_bool(r, True)
                    self._drain()
                except _Conflict:
                    pass
            self.force = False
        return [self.value_of_var(v) for v in range(len(self.dag.vars))]


def hints_py(dag: Dag) -> Tuple[List[int], int]:
    """Python reference: (hint value of every variable, number of distinct roots the hint
    model satisfies).  Caller parents seed the bits no constraint fixes."""
    s = Seeder(dag, [v.parent for v in dag.vars])
    vals = s.run()
    return vals, sum(1 for r in dict.fromkeys(dag.roots) if s.ev(r))


def hints(dag: Dag) -> Tuple[List[int], int]:
    """:func:`hints_py`, computed by libpflower.so (pfl_hints) when it is built — the same
    values decision for decision (tests/test_native_seed.py)."""
    from .lower import _native, limbs, pack_nodes

    L = _native()
    if not L or any(v.width > 256 for v in dag.vars):
        return hints_py(dag)
    import ctypes

    import numpy as np

    nodes, pool_a, pool = pack_nodes(dag)
    nv = len(dag.vars)
    widths = np.array([v.width for v in dag.vars], dtype=np.uint32)
    soft = limbs([(v.parent or 0) & M(v.width) for v in dag.vars])
    roots = np.array(dag.roots or [0], dtype=np.uint32)
    out = np.zeros((nv, 8), dtype=np.uint32)
    n_sat = ctypes.c_int()
    p = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    rc = L.pfl_hints(p(nodes), len(dag.nodes), p(pool_a), len(pool), p(roots), len(dag.roots),
                     p(widths), nv, p(soft), p(out), ctypes.byref(n_sat))
    if rc != 0:
        raise ValueError(f"pfl_hints failed ({rc})")
    o = out.astype(np.uint64)
    vals = [sum(int(x) << (32 * j) for j, x in enumerate(row)) for row in o]
    return vals, n_sat.value


def derive_hints(dag: Dag) -> List[int]:
    """Hint value of every variable of ``dag`` (caller parents seed the unfixed bits)."""
    return hints(dag)[0]


def apply_hints(dag: Dag) -> int:
    """Install the hint model as the parent model of ``dag``'s variables; returns the number
    of roots the hint model itself satisfies (diagnostic)."""
    if not dag.vars:
        return 0
    vals, n_sat = hints(dag)
    for var, val in zip(dag.vars, vals):
        var.parent = val & M(var.width)
    return n_sat
