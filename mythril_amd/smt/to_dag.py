"""Constraint terms -> bytecode DAG (mythril_amd.lower.Dag), with arrays and UFs interpreted
by construction.

The conjunction handed to ``get_model`` (mythril/support/model.py:87-93) is lowered so that
every GPU candidate *is* a complete model:

* free BitVec/Bool symbols become candidate variables (schema kind from the LASER naming
  scheme: ``sender_*`` -> actor set, ``*_calldatasize`` -> small sizes, see
  mythril/laser/ethereum/transaction/symbolic.py:122-139, state/calldata.py:229-230);
* ``select`` over ``store``/``K``/``ite`` chains is resolved structurally; a base array
  becomes one variable per distinct index term, and a later index term reads the value of
  the first earlier index that evaluates equal (``ite`` chain) — a total, consistent array
  interpretation for every candidate (no Ackermann side constraints needed);
* ``keccak256_<n>`` (keccak_function_manager.py:71-84) is interpreted as
  ``c_i -> keccak(c_i)`` for the registered concrete hashes and
  ``x -> lo_n + 64 * (H(x) mod 2^117)`` otherwise (H = PF_W_HASH), which satisfies the
  interval / ``% 64`` / concrete-equality conditions of ``_create_condition`` (:150-179) by
  construction; ``keccak256_<n>-1`` is substituted through ``inv(f(t)) = t`` and otherwise
  looked up among the set's f-applications, with the injectivity of f on the set added as
  side constraints (f(a) = f(b) -> a = b) so the interpretation stays a function;
* ``Power`` (exponent_function_manager.py:29-68) is interpreted so that its conditions hold
  by construction (``TermLowering._power``): concrete facts c1^c2, base 256 as
  256^(e mod 32), other symbolic applications as candidate variables kept functional by
  argument value; any other UF as a keyed hash of its arguments.
Values wider than 256 bits are carried as 256-bit chunks: keccak256_512 inputs, zero-padded
``==`` (bitvec.py:16-22), and z3's expansion of ``BVAddNoOverflow(a, b, False)`` —
``((_ extract 256 256) (bvadd ((_ zero_extend 1) a) ((_ zero_extend 1) b)))``, the 257-bit
sum's carry (bitvec_helper.py:199-213, used by every IntegerArithmetics query,
integer.py:144-158).  Chunked ops: concat / zero_extend / extract (across chunks) / ite /
add / sub (carry rippled as a B value) / neg / and / or / xor / not / shifts by a constant /
= / unsigned and signed orderings.  Anything else raises LoweringError -> z3.
"""

from __future__ import annotations

import re
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .. import ir
from ..lower import Dag, LoweringError
from . import terms as T

_KECCAK_RE = re.compile(r"^keccak256_(\d+)(-1)?$")

ACTORS = (
    0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,  # CREATOR  (transaction/symbolic.py:26-37)
    0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,  # ATTACKER
    0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA,  # SOMEGUY
)
KECCAK_MASK_BITS = 117
_WINDOW_MIN = 8   # runs of a byte array's indices this long become window lookups
_NO_RUN = object()


@dataclass
class KeccakSpec:
    lo: Optional[int]                         # interval start (keccak_function_manager.py:165);
                                              # None while the width has only concrete hashes
    concrete: Dict[int, int] = field(default_factory=dict)   # input value -> keccak

    @property
    def base(self) -> int:
        """First multiple of 64 in the interval: base + 64*k stays inside [lo, lo + PART)
        for k < 2^117 (PART = (2^256-1) // 10^40 > 2^123 + 64) and satisfies ``% 64 == 0``."""
        return (self.lo + 63) & ~63


class UFRegistry:
    """Per-width keccak interpretation data, mirrored from the KeccakFunctionManager."""

    def __init__(self):
        self.keccak: Dict[int, KeccakSpec] = {}
        self.actors: Tuple[int, ...] = ACTORS

    def keccak_for(self, n: int) -> Optional[KeccakSpec]:
        return self.keccak.get(n)


DEFAULT_REGISTRY = UFRegistry()


def salt_of(name: str) -> int:
    return zlib.crc32(name.encode()) & 0xFFFFFFFF


def var_kind(name: str, w: int):
    """Candidate-generator kind for a LASER symbol name."""
    if name.startswith("sender_") and w == 256:
        return ir.VK_ACTOR
    if name.endswith("_calldatasize"):
        return ir.VK_SMALL
    if w == 8 and ir.CDBYTE_RE.match(name):
        return ir.VK_CDBYTE
    if w == 256 and (name.startswith("call_value") or name.startswith("callvalue")):
        return ir.VK_VALUE   # transaction/symbolic.py:137-138, transaction_models.py:121-124
    return ir.VK_GENERIC


@dataclass
class Lowered:
    dag: Dag
    var_terms: List[T.Term]                    # candidate variable i <-> term (var / select / apply)
    uf_apps: List[Tuple[str, tuple, T.Term]]   # (name, arg terms, app term) for model tables
    array_reads: Dict[str, List[Tuple[T.Term, T.Term]]]  # array -> (index, select term) in lookup order


class TermLowering:
    def __init__(self, registry: Optional[UFRegistry] = None, parent: Optional[dict] = None):
        self.reg = registry or DEFAULT_REGISTRY
        self.dag = Dag()
        self.parent = parent or {}
        self.memo: Dict[T.Term, object] = {}
        self.var_terms: List[T.Term] = []
        # base array name -> [(idx term, select term, idx node, value node)] in lookup order
        self.arrays: Dict[str, List[Tuple[T.Term, T.Term, int, object]]] = {}
        self.keccak_apps: Dict[int, List[Tuple[T.Term, object, object]]] = {}  # n -> [(arg term, arg val, f node)]
        self.inv_apps: Dict[int, List[Tuple[object, object]]] = {}  # n -> [(key node, value node)]
        self.uf_apps: List[Tuple[str, tuple, T.Term]] = []
        self.side: List[int] = []
        self._actor_consts: Optional[int] = None
        self.power_apps: List[Tuple[T.Term, T.Term, int, bool]] = []  # (b, e, value node, symbolic)
        self.power_facts: Dict[Tuple[int, int], int] = {}            # concrete (b, e) -> b^e

    # ---- leaves -----------------------------------------------------------------------
    def _var(self, name: str, w: int, term: T.Term, parent: Optional[int] = None) -> int:
        kind = var_kind(name, w)
        hint0 = hint1 = 0
        if kind == ir.VK_ACTOR:
            hint0, hint1 = self._actor_table()
        elif kind == ir.VK_SMALL:
            hint0 = 4 + 32 * 8
        elif kind == ir.VK_CDBYTE:
            hint0, hint1 = ir.cdbyte_hints(name)
        before = len(self.dag.vars)
        if parent is None and self.parent:
            # parent models are keyed by symbol name, or by the read's own (hash-consed)
            # select term for array reads (gpu_check._recent_parent)
            parent = self.parent.get(name)
            if parent is None:
                parent = self.parent.get(term)
        node = self.dag.var(name, w, kind, hint0, hint1, parent)
        if len(self.dag.vars) > before:
            self.var_terms.append(term)
        return node

    def _actor_table(self):
        if self._actor_consts is None:
            self._actor_consts = self.dag.force_consts(self.reg.actors)
        return self._actor_consts, len(self.reg.actors)

    # ---- generic lowering ---------------------------------------------------------------
    def w(self, t: T.Term):
        """Lower a BitVec term: a node (width <= 256) or a chunk list for wider values."""
        r = self.memo.get(t)
        if r is None:
            r = self._lower_bv(t)
            self.memo[t] = r
        return r

    def node(self, t: T.Term) -> int:
        r = self.w(t)
        if isinstance(r, list):
            raise LoweringError(f"{t.width}-bit value used where <= 256 bits are required")
        return r

    def b(self, t: T.Term) -> int:
        r = self.memo.get(t)
        if r is None:
            r = self._lower_bool(t)
            self.memo[t] = r
        return r

    def chunks(self, t: T.Term) -> List[Tuple[int, int]]:
        """Little-endian 256-bit-aligned chunks (node, width) of a value of any width."""
        return self._rechunk(self._pieces(t))

    def _rechunk(self, pieces: List[Tuple[int, int]]) -> List[Tuple[int, int]]:
        """LSB-first pieces (node, width) -> 256-bit-aligned chunks."""
        out: List[Tuple[int, int]] = []
        cur: List[Tuple[int, int]] = []   # pieces of the current chunk (LSB first)
        fill = 0
        for node, wd in pieces:
            off = 0
            while off < wd:
                take = min(256 - fill, wd - off)
                if off == 0 and take == wd:
                    part = node
                else:
                    part = self.dag.op(ir.W_EXTRACT, take, node, aux=off)
                cur.append((part, take))
                fill += take
                off += take
                if fill == 256:
                    out.append(self._join(cur))
                    cur, fill = [], 0
        if cur:
            out.append(self._join(cur))
        return out

    def _join(self, cur):
        # cur is LSB-first; concat high..low
        node, wd = cur[-1]
        for part, pw in reversed(cur[:-1]):
            node = self.dag.op(ir.W_CONCAT, wd + pw, node, part, aux=pw)
            wd += pw
        return node, wd

    def _pieces(self, t: T.Term) -> List[Tuple[int, int]]:
        if t.width <= 256:
            return [(self.node(t), t.width)]
        if t.op == "concat":
            out = []
            for p in reversed(t.args):
                out.extend(self._pieces(p))
            return out
        if t.op == "zero_extend":
            out = self._pieces(t.args[0])
            rest = t.val
            while rest > 0:
                k = min(rest, 256)
                out.append((self.dag.const(0, k), k))
                rest -= k
            return out
        if t.op == "bv":
            out, v, rest = [], t.val, t.width
            while rest > 0:
                k = min(rest, 256)
                out.append((self.dag.const(v & ir.mask(k), k), k))
                v >>= k
                rest -= k
            return out
        r = self.w(t)
        if isinstance(r, list):
            return r
        raise LoweringError(f"wide op {t.op}")

    def _lower_bv(self, t: T.Term):
        op, wd = t.op, t.width
        if wd > 256:
            return self._lower_wide(t)
        if op == "bv":
            return self.dag.const(t.val, wd)
        if op == "var":
            return self._var(t.val, wd, t)
        if op in _WBIN:
            return self.dag.op(_WBIN[op], wd, self.node(t.args[0]), self.node(t.args[1]))
        if op == "bvnot":
            return self.dag.op(ir.W_NOT, wd, self.node(t.args[0]))
        if op == "bvneg":
            return self.dag.op(ir.W_NEG, wd, self.node(t.args[0]))
        if op == "extract":
            hi, lo = t.val
            src = t.args[0]
            if src.width <= 256:
                return self.dag.op(ir.W_EXTRACT, wd, self.node(src), aux=lo)
            (node, _), = self._slice(self.chunks(src), lo, wd)
            return node
        if op == "concat":
            parts = t.args
            node, acc = self.node(parts[0]), parts[0].width
            for p in parts[1:]:
                node = self.dag.op(ir.W_CONCAT, acc + p.width, node, self.node(p), aux=p.width)
                acc += p.width
            return node
        if op == "zero_extend":
            return self.dag.op(ir.W_MOV, wd, self.node(t.args[0]))
        if op == "ite":
            return self.dag.op(ir.W_ITE, wd, self.b(t.args[0]), self.node(t.args[1]), self.node(t.args[2]))
        if op == "select":
            return self._select(t.args[0], t.args[1], t)
        if op == "apply":
            return self._apply(t)
        raise LoweringError(f"unsupported bit-vector op {op}")

    # ---- values wider than 256 bits (z3's 257-bit no-overflow expansions, 512-bit keccak
    # inputs, zero-padded comparisons: bitvec.py:16-22, bitvec_helper.py:199-245) ---------
    def _slice(self, chunks: List[Tuple[int, int]], lo: int, width: int) -> List[Tuple[int, int]]:
        """Bits [lo, lo + width) of a chunked value, as chunks."""
        d = self.dag
        pieces, base = [], 0
        for node, cw in chunks:
            a, b = max(lo, base), min(lo + width, base + cw)
            if a < b:
                if a == base and b == base + cw:
                    pieces.append((node, cw))
                else:
                    pieces.append((d.op(ir.W_EXTRACT, b - a, node, aux=a - base), b - a))
            base += cw
        return self._rechunk(pieces)

    def _bit_to_w(self, bnode: int, w: int) -> int:
        d = self.dag
        return d.op(ir.W_ITE, w, bnode, d.const(1, w), d.const(0, w))

    def _wide_addsub(self, A, B, sub: bool):
        """Chunked add / subtract with the carry (borrow) rippled as a B value."""
        d = self.dag
        opc = ir.W_SUB if sub else ir.W_ADD
        out, carry = [], None
        for i, ((x, wx), (y, _)) in enumerate(zip(A, B)):
            t = d.op(opc, wx, x, y)
            s_, cw = t, None
            if carry is not None:
                cw = self._bit_to_w(carry, wx)
                s_ = d.op(opc, wx, t, cw)
            if i + 1 < len(A):   # carry out of a full 256-bit chunk
                c1 = d.op(ir.B_ULT, wx, x, y) if sub else d.op(ir.B_ULT, wx, t, x)
                if carry is not None:
                    c2 = d.op(ir.B_ULT, wx, t, cw) if sub else d.op(ir.B_ULT, wx, s_, t)
                    c1 = d.op(ir.B_OR, 1, c1, c2)
                carry = c1
            out.append((s_, wx))
        return out

    def _wide_cmp(self, op: str, a: T.Term, b: T.Term) -> int:
        """bvult / bvule / bvslt / bvsle over chunks: decided by the highest differing chunk
        (the top chunk compared signed for the signed forms)."""
        d = self.dag
        A, B = self.chunks(a), self.chunks(b)
        signed = op in ("bvslt", "bvsle")
        strict = op in ("bvult", "bvslt")
        # lt over chunks 0..i, built from the bottom: lt_i = lt(x_i, y_i) | (x_i == y_i & lt_{i-1})
        lt = None
        for i, ((x, wx), (y, _)) in enumerate(zip(A, B)):
            top = i == len(A) - 1
            cmp = ir.B_SLT if (signed and top) else ir.B_ULT
            li = d.op(cmp, wx, x, y)
            if lt is not None:
                li = d.op(ir.B_OR, 1, li, d.op(ir.B_AND, 1, d.op(ir.B_EQ, wx, x, y), lt))
            lt = li
        if strict:
            return lt
        # a <= b  <=>  not (b < a)
        return d.op(ir.B_NOT, 1, self._wide_cmp("bvslt" if signed else "bvult", b, a))

    def _lower_wide(self, t: T.Term):
        op, wd = t.op, t.width
        d = self.dag
        if op in ("concat", "zero_extend", "bv"):
            return self.chunks(t)
        if op == "var":
            # a free symbol wider than 256 bits: one candidate variable per chunk, each
            # recorded as its extract term (the witness reassembles the symbol's value)
            out, lo, pv = [], 0, self.parent.get(t.val)
            while lo < wd:
                cw = min(256, wd - lo)
                part = T.extract(lo + cw - 1, lo, t)
                out.append((self._var(f"{t.val}#{lo // 256}", cw, part,
                                      None if pv is None else (pv >> lo) & ir.mask(cw)), cw))
                lo += cw
            return out
        if op == "apply":
            return self._apply(t)
        if op == "ite":
            c = self.b(t.args[0])
            a, b = self.chunks(t.args[1]), self.chunks(t.args[2])
            return [(d.op(ir.W_ITE, x[1], c, x[0], y[0]), x[1]) for x, y in zip(a, b)]
        if op == "extract":
            hi, lo = t.val
            return self._slice(self.chunks(t.args[0]), lo, wd)
        if op in ("bvadd", "bvsub"):
            return self._wide_addsub(self.chunks(t.args[0]), self.chunks(t.args[1]), op == "bvsub")
        if op == "bvneg":
            zero = [(d.const(0, w), w) for _, w in self.chunks(t.args[0])]
            return self._wide_addsub(zero, self.chunks(t.args[0]), True)
        if op in ("bvand", "bvor", "bvxor"):
            opc = {"bvand": ir.W_AND, "bvor": ir.W_OR, "bvxor": ir.W_XOR}[op]
            return [(d.op(opc, wx, x, y), wx)
                    for (x, wx), (y, _) in zip(self.chunks(t.args[0]), self.chunks(t.args[1]))]
        if op == "bvnot":
            return [(d.op(ir.W_NOT, wx, x), wx) for x, wx in self.chunks(t.args[0])]
        if op in ("bvshl", "bvlshr") and t.args[1].op == "bv":
            # shift by a constant k: bits move between chunks, zeros fill in
            k = t.args[1].val
            if k >= wd:
                return self.chunks(T.const(0, wd))
            A = self.chunks(t.args[0])
            zeros = self.chunks(T.const(0, k)) if k else []
            if op == "bvshl":   # concat(a[wd-1-k : 0], 0_k)
                return self._rechunk(zeros + self._slice(A, 0, wd - k))
            return self._rechunk(self._slice(A, k, wd - k) + zeros)
        raise LoweringError(f"{wd}-bit {op}")

    def _lower_bool(self, t: T.Term) -> int:
        op = t.op
        d = self.dag
        if op == "true":
            return d.bconst(True)
        if op == "false":
            return d.bconst(False)
        if op == "bvar":
            return self._bvar(t)
        if op == "not":
            return d.op(ir.B_NOT, 1, self.b(t.args[0]))
        if op in ("and", "or"):
            opc = ir.B_AND if op == "and" else ir.B_OR
            acc = self.b(t.args[0])
            for a in t.args[1:]:
                acc = d.op(opc, 1, acc, self.b(a))
            return acc
        if op == "xor":
            return d.op(ir.B_XOR, 1, self.b(t.args[0]), self.b(t.args[1]))
        if op == "iff":
            return d.op(ir.B_NOT, 1, d.op(ir.B_XOR, 1, self.b(t.args[0]), self.b(t.args[1])))
        if op == "ite":
            return d.op(ir.B_ITE, 1, self.b(t.args[0]), self.b(t.args[1]), self.b(t.args[2]))
        if op == "=":
            a, b = t.args
            if a.width > 256 or b.width > 256:
                ca, cb = self.chunks(a), self.chunks(b)
                acc = None
                for (x, wx), (y, wy) in zip(ca, cb):
                    e = d.op(ir.B_EQ, wx, x, y)
                    acc = e if acc is None else d.op(ir.B_AND, 1, acc, e)
                return acc
            return d.op(ir.B_EQ, a.width, self.node(a), self.node(b))
        if op in _BCMP:
            a, b = t.args
            if a.width > 256 and op in ("bvult", "bvule", "bvslt", "bvsle"):
                return self._wide_cmp(op, a, b)
            return d.op(_BCMP[op], a.width, self.node(a), self.node(b))
        raise LoweringError(f"unsupported bool op {op}")

    def _bvar(self, t: T.Term) -> int:
        before = len(self.dag.vars)
        node = self.dag.var(t.val, 1, ir.VK_BOOL, parent=self.parent.get(t.val))
        if len(self.dag.vars) > before:
            self.var_terms.append(t)
        return node

    # ---- arrays ---------------------------------------------------------------------------
    @staticmethod
    def _offset_form(t: T.Term) -> Tuple[Optional[T.Term], int]:
        """(base, c) with t = base + c mod 2^w — constant additions and subtractions peeled
        off (base None for a constant).  Two indices with the same base and different c can
        never be equal: LASER's dynamic-ABI reads ``calldata[off + 4 + k]`` (ABI words and
        string bytes at one symbolic offset) then need no aliasing test among themselves."""
        m = (1 << t.width) - 1
        c = 0
        while True:
            if t.op == "bv":
                return None, (c + t.val) & m
            if t.op == "bvadd" and len(t.args) == 2:
                if t.args[1].op == "bv":
                    c, t = c + t.args[1].val, t.args[0]
                    continue
                if t.args[0].op == "bv":
                    c, t = c + t.args[0].val, t.args[1]
                    continue
            elif t.op == "bvsub" and len(t.args) == 2 and t.args[1].op == "bv":
                c, t = c - t.args[1].val, t.args[0]
                continue
            return t, c & m

    def _select(self, arr: T.Term, idx: T.Term, term: T.Term) -> int:
        d = self.dag
        if arr.op == "store":
            base, k, v = arr.args
            if k is idx:
                return self.node(v)
            (kb, kc), (ib, ic) = self._offset_form(k), self._offset_form(idx)
            if kb is ib:  # the same base: the offsets decide (both constants: their values)
                return self._select(base, idx, term) if kc != ic else self.node(v)
            rest = self._select(base, idx, T.select(base, idx))
            c = d.op(ir.B_EQ, idx.width, self.node(idx), self.node(k))
            return d.op(ir.W_ITE, arr.sort[2], c, self.node(v), rest)
        if arr.op == "K":
            return self.node(arr.args[0])
        if arr.op == "ite":
            c = self.b(arr.args[0])
            a = self._select(arr.args[1], idx, T.select(arr.args[1], idx))
            b = self._select(arr.args[2], idx, T.select(arr.args[2], idx))
            return d.op(ir.W_ITE, arr.sort[2], c, a, b)
        if arr.op != "array":
            raise LoweringError(f"select over {arr.op}")
        name, rng = arr.val, arr.sort[2]
        if idx.width > 256:
            raise LoweringError("array index wider than 256 bits")
        entries = self.arrays.setdefault(name, [])
        for (it, _, _, val) in entries:
            if it is idx:
                return val
        inode = self.node(idx)
        if idx.op == "bv":
            vname = f"{name}[{idx.val}]"
        else:
            vname = f"{name}@{len(entries)}"
        sel_term = T.select(arr, idx)
        val = self._var(vname, rng, sel_term)
        # first earlier index with an equal value wins (consistent array interpretation)
        ib, ic = self._offset_form(idx)
        # runs: entries next to each other in lookup order with one base other than idx's
        # (constants: base None) — distinct offsets, so at most one of them can match
        run: List[Tuple[int, int, object]] = []
        run_base: object = _NO_RUN
        for (it, _, inn, v) in reversed(entries):
            tb, tc = self._offset_form(it)
            if tb is ib and tc != ic:
                continue  # the same base at another offset (distinct constants) never aliases
            if tb is ib:
                val = self._run(run, run_base, idx, inode, rng, val)
                run, run_base = [], _NO_RUN
                val = d.op(ir.W_ITE, rng, d.op(ir.B_EQ, idx.width, inode, inn), v, val)
                continue
            if run and tb is not run_base:
                val = self._run(run, run_base, idx, inode, rng, val)
                run = []
            run_base = tb
            run.append((tc, inn, v))
        val = self._run(run, run_base, idx, inode, rng, val)
        entries.append((idx, sel_term, inode, val))
        return val

    def _run(self, run, base, idx: T.Term, inode: int, rng: int, val):
        """The part of a read's ``ite`` chain that tests a run of indices base + c (entries
        next to each other in lookup order, so at most one of them can match and their order
        is free).  Short runs stay ``ite(idx == base + c, v_c, ...)`` in lookup order.  A byte
        array's contiguous offsets c .. c + n - 1 (8 <= n <= 32: LASER's calldata header and
        ABI words at a constant or a symbolic offset, calldata.py:233-246) become one window
        lookup per read: the n bytes concatenated (v_c lowest), shifted right by
        8 * (idx - (base + c)) and cut to a byte, selected when that difference is < n — a
        dozen nodes instead of 4 * n, the same value for every assignment (the single
        query's longest programs were these chains: DESIGN.md §4)."""
        d = self.dag
        if (len(run) < _WINDOW_MIN or rng != 8 or idx.width != 256
                or len({e[0] for e in run}) != len(run)):
            for (_, inn, v) in run:
                val = d.op(ir.W_ITE, rng, d.op(ir.B_EQ, idx.width, inode, inn), v, val)
            return val
        items = sorted(run, key=lambda e: e[0])
        i = 0
        while i < len(items):
            j = i + 1
            while j < len(items) and items[j][0] == items[j - 1][0] + 1 and j - i < 32:
                j += 1
            piece = items[i:j]
            if len(piece) < _WINDOW_MIN:
                for (_, inn, v) in piece:
                    val = d.op(ir.W_ITE, rng, d.op(ir.B_EQ, idx.width, inode, inn), v, val)
            else:
                val = self._window(piece, base is None, inode, val)
            i = j
        return val

    def _window(self, piece, const_base: bool, inode: int, val) -> int:
        d = self.dag
        lo, n = piece[0][0], len(piece)
        acc = piece[0][2]
        for j in range(1, n):
            acc = d.op(ir.W_CONCAT, 8 * (j + 1), piece[j][2], acc, aux=8 * j)
        # idx - (base + lo): the piece's lowest index node
        t = inode if const_base and lo == 0 else d.op(ir.W_SUB, 256, inode, piece[0][1])
        hit = d.op(ir.B_ULT, 256, t, d.const(n, 256))
        amt = d.op(ir.W_EXTRACT, 8 * n, d.op(ir.W_SHL, 256, t, d.const(3, 256)), aux=0)
        byte = d.op(ir.W_EXTRACT, 8, d.op(ir.W_LSHR, 8 * n, acc, amt), aux=0)
        return d.op(ir.W_ITE, 8, hit, byte, val)

    # ---- uninterpreted functions --------------------------------------------------------
    def _hash_args(self, args, salt) -> int:
        d = self.dag
        h = None
        for a in args:
            for node, wd in self.chunks(a):
                x = node if wd == 256 else d.op(ir.W_MOV, 256, node)
                h = d.op(ir.W_HASH, 256, x if h is None else d.op(ir.W_XOR, 256, h, x), aux=salt)
        return h

    def _apply(self, t: T.Term):
        d = self.dag
        fname, _ = t.val
        args = t.args
        m = _KECCAK_RE.match(fname)
        if m:
            n = int(m.group(1))
            if m.group(2) is None:
                return self._keccak(n, args[0], t)
            return self._keccak_inv(n, args[0], t)
        if fname == "Power" and len(args) == 2 and t.width == 256:
            return self._power(t)
        self.uf_apps.append((fname, args, t))
        h = self._hash_args(args, salt_of(fname))
        return h if t.width == 256 else d.op(ir.W_EXTRACT, t.width, h, aux=0)

    def _power(self, t: T.Term) -> int:
        """``Power(b, e)``, the UF Mythril uses for symbolic EXP
        (exponent_function_manager.py:40-68; instructions.py:625-639).  Its conditions are
        ``Power(b, e) >s 0`` per symbolic EXP, the 32 table entries ``Power(256, i) = 256^i``,
        ``Power(256, e %u 32) == Power(256, e)`` for base 256, and ``Power(c1, c2) =
        c1^c2 mod 2^256`` for a concrete EXP.  Interpretation, by argument value:
        1. (b, e) equal to a concrete application's arguments (c1, c2) in the set ->
           c1^c2 mod 2^256 (functional consistency with the concrete facts);
        2. b == 256 -> 256^(e mod 32) = 2^(8 (e mod 32)) — satisfies the table, the
           ``e %u 32`` condition and ``>s 0`` (at most 2^248) for every e;
        3. otherwise a free candidate variable per symbolic application, equal to the first
           earlier application whose arguments evaluate equal (a function, like the array
           reads); the set's own ``>s 0`` constraint then decides the candidate.
        Real modular EXP is not a model: ``Power(256, e) = 256^e mod 2^256`` is 0 for every
        e >= 32, which the conditions forbid."""
        d = self.dag
        b_t, e_t = t.args
        for (bt, et, node, _) in self.power_apps:
            if bt is b_t and et is e_t:
                return node
        if b_t.op == "bv" and e_t.op == "bv":
            val = d.const(pow(b_t.val, e_t.val, 1 << 256), 256)
        else:
            bn, en = self.node(b_t), self.node(e_t)
            val = self._var(f"Power@{sum(1 for a in self.power_apps if a[3])}", 256, t)
            for (bt, et, node, sym) in reversed(self.power_apps):
                if sym:
                    same = d.op(ir.B_AND, 1, d.op(ir.B_EQ, 256, bn, self.node(bt)),
                                d.op(ir.B_EQ, 256, en, self.node(et)))
                    val = d.op(ir.W_ITE, 256, same, node, val)
            rule = d.op(ir.W_SHL, 256, d.const(1, 256),
                        d.op(ir.W_SHL, 256, d.op(ir.W_AND, 256, en, d.const(31, 256)), d.const(3, 256)))
            val = d.op(ir.W_ITE, 256, d.op(ir.B_EQ, 256, bn, d.const(256, 256)), rule, val)
            for (c1, c2), pv in self.power_facts.items():
                same = d.op(ir.B_AND, 1, d.op(ir.B_EQ, 256, bn, d.const(c1, 256)),
                            d.op(ir.B_EQ, 256, en, d.const(c2, 256)))
                val = d.op(ir.W_ITE, 256, same, d.const(pv, 256), val)
        self.power_apps.append((b_t, e_t, val, not (b_t.op == "bv" and e_t.op == "bv")))
        self.uf_apps.append(("Power", (b_t, e_t), t))
        return val

    def _collect_power_facts(self, constraints: List[T.Term]) -> None:
        seen, stack = set(), list(constraints)
        while stack:
            x = stack.pop()
            if x in seen:
                continue
            seen.add(x)
            if (x.op == "apply" and x.val[0] == "Power" and len(x.args) == 2
                    and x.args[0].op == "bv" and x.args[1].op == "bv"):
                c1, c2 = x.args[0].val, x.args[1].val
                self.power_facts[(c1, c2)] = pow(c1, c2, 1 << 256)
            stack.extend(x.args)

    def _keccak(self, n: int, arg: T.Term, t: T.Term) -> int:
        d = self.dag
        apps = self.keccak_apps.setdefault(n, [])
        for (a, _, node) in apps:
            if a is arg:
                return node
        spec = self.reg.keccak_for(n)
        h = self._hash_args([arg], salt_of(f"keccak256_{n}"))
        if spec is not None:
            if spec.lo is not None:
                k = d.op(ir.W_AND, 256, h, d.const(ir.mask(KECCAK_MASK_BITS), 256))
                val = d.op(ir.W_ADD, 256, d.const(spec.base, 256),
                           d.op(ir.W_SHL, 256, k, d.const(6, 256)))
            else:
                val = h
            for c, kv in spec.concrete.items():
                eqs = self._eq_value(arg, c)
                if eqs is not None:
                    val = d.op(ir.W_ITE, 256, eqs, d.const(kv, 256), val)
        else:
            val = h
        # injectivity on the set: f(a) = f(b) -> a = b
        for (a, _, node) in apps:
            same_f = d.op(ir.B_EQ, 256, val, node)
            same_x = self._eq_terms(arg, a)
            self.side.append(d.op(ir.B_OR, 1, d.op(ir.B_NOT, 1, same_f), same_x))
        apps.append((arg, None, val))
        self.uf_apps.append((f"keccak256_{n}", (arg,), t))  # registration order = lookup order
        return val

    def _keccak_inv(self, n: int, y: T.Term, t: T.Term):
        d = self.dag
        if y.op == "apply" and y.val[0] == f"keccak256_{n}":
            self.w(y)  # make sure f(x) is registered (injectivity constraints)
            return self.w(y.args[0])
        if n > 256:
            raise LoweringError("inverse keccak of a wide input on a non-application")
        ynode = self.node(y)
        val = self._var(f"keccak256_{n}-1@{len(self.inv_apps.get(n, []))}", n, t)
        entries = self.inv_apps.setdefault(n, [])
        for (knode, vnode) in reversed(entries):
            val = d.op(ir.W_ITE, n, d.op(ir.B_EQ, 256, ynode, knode), vnode, val)
        for (a, _, fnode) in reversed(self.keccak_apps.get(n, [])):
            val = d.op(ir.W_ITE, n, d.op(ir.B_EQ, 256, ynode, fnode), self.node(a), val)
        entries.append((ynode, val))
        self.uf_apps.append((f"keccak256_{n}-1", (y,), t))
        return val

    def _eq_value(self, t: T.Term, c: int) -> Optional[int]:
        return self._eq_terms(t, T.const(c, t.width))

    def _eq_terms(self, a: T.Term, b: T.Term) -> int:
        d = self.dag
        if a.width != b.width:
            return d.bconst(False)
        if a.width <= 256:
            return d.op(ir.B_EQ, a.width, self.node(a), self.node(b))
        acc = None
        for (x, wx), (y, _) in zip(self.chunks(a), self.chunks(b)):
            e = d.op(ir.B_EQ, wx, x, y)
            acc = e if acc is None else d.op(ir.B_AND, 1, acc, e)
        return acc

    # ---- driver ---------------------------------------------------------------------------
    def lower(self, constraints: List[T.Term]) -> Lowered:
        self._collect_power_facts(constraints)
        for c in constraints:
            if not c.is_bool:
                raise LoweringError("constraint is not a Bool")
            if c is T.TRUE:
                continue
            self.dag.assert_(self.b(c))
        for s in self.side:
            self.dag.assert_(s)
        arrays = {k: [(it, st) for (it, st, _, _) in v] for k, v in self.arrays.items()}
        return Lowered(self.dag, self.var_terms, self.uf_apps, arrays)


class ExplicitLowering(TermLowering):
    """Lowering for evaluation under EXPLICIT models — the GPU-resident ``ModelCache``
    (mythril_amd/model_cache.py; ref support/support_utils.py:57-71 evaluates a query under up
    to 100 cached models).  A cached model (a z3 model, or a GPU witness) interprets arrays
    and UFs its own way, so nothing is interpreted by construction here: every read of a
    base array (``select(A, i)`` at the bottom of a store / ite chain) and every UF
    application (keccak and its inverse, ``Power``, any other) is a LEAF variable whose value
    the caller evaluates under each model; only the operators above the leaves are lowered.
    A leaf wider than 256 bits (``keccak256_512-1``) is one variable per 256-bit chunk, each
    recorded as its ``extract`` term.  No side constraints, no concrete-``Power`` facts, no
    ``inv(f(x)) = x`` substitution: the program computes exactly the conjunction's value
    under whatever leaf values it is given."""

    def __init__(self):
        super().__init__(UFRegistry())
        self.reg.actors = ()   # no generator tables: values come from the models
        self.leaves: Dict[T.Term, int] = {}

    def _leaf(self, term: T.Term, w: int) -> int:
        node = self.leaves.get(term)
        if node is None:
            node = self._var(f"@leaf{len(self.leaves)}", w, term)
            self.leaves[term] = node
        return node

    def _select(self, arr: T.Term, idx: T.Term, term: T.Term) -> int:
        if arr.op == "array":
            if idx.width > 256:
                raise LoweringError("array index wider than 256 bits")
            return self._leaf(T.select(arr, idx), arr.sort[2])
        return super()._select(arr, idx, term)

    def _apply(self, t: T.Term):
        if t.width <= 256:
            return self._leaf(t, t.width)
        out, lo = [], 0
        while lo < t.width:
            cw = min(256, t.width - lo)
            out.append((self._leaf(T.extract(lo + cw - 1, lo, t), cw), cw))
            lo += cw
        return out

    def _lower_bv(self, t: T.Term):
        if t.op == "bvlshr" and t.width <= 256 and t.args[1].op == "bv" and t.args[0].op == "concat":
            r = self._lshr_concat(t.args[0].args, t.args[1].val, t.width)
            if r is not None:
                return r
        return super()._lower_bv(t)

    def _lshr_concat(self, parts, k: int, wd: int) -> Optional[int]:
        """``bvlshr(concat(p0 .. pn-1), k)``: the low parts the shift discards whole are not
        lowered — their bits never reach the result (LASER's selector test shifts a 32-byte
        calldata word right by 224: 4 of its 32 guarded byte reads matter).  The kept parts
        ``concat(p0 .. pj)`` shifted by what is left of k, zero-extended back to ``wd``; None
        when no part is dropped.  Mirrored by pf_terms.cpp (PFLT_EXPLICIT)."""
        j, drop = len(parts), 0
        while j > 1 and drop + parts[j - 1].width <= k:
            drop += parts[j - 1].width
            j -= 1
        if j == len(parts):
            return None
        d = self.dag
        hi, hw = self.node(parts[0]), parts[0].width
        for p in parts[1:j]:
            hi = d.op(ir.W_CONCAT, hw + p.width, hi, self.node(p), aux=p.width)
            hw += p.width
        rem = k - drop
        if rem >= hw:
            return d.const(0, wd)
        if rem:
            hi = d.op(ir.W_LSHR, hw, hi, d.const(rem, hw))
        return d.op(ir.W_MOV, wd, hi)

    def lower(self, constraints: List[T.Term]) -> Lowered:
        for c in constraints:
            if not c.is_bool:
                raise LoweringError("constraint is not a Bool")
            if c is T.TRUE:
                continue
            self.dag.assert_(self.b(c))
        return Lowered(self.dag, self.var_terms, [], {})


_WBIN = {
    "bvadd": ir.W_ADD, "bvsub": ir.W_SUB, "bvmul": ir.W_MUL, "bvudiv": ir.W_UDIV,
    "bvurem": ir.W_UREM, "bvsdiv": ir.W_SDIV, "bvsrem": ir.W_SREM, "bvsmod": ir.W_SMOD,
    "bvand": ir.W_AND, "bvor": ir.W_OR, "bvxor": ir.W_XOR, "bvshl": ir.W_SHL,
    "bvlshr": ir.W_LSHR, "bvashr": ir.W_ASHR, "bvexp": ir.W_EXP,
}
_BCMP = {
    "bvult": ir.B_ULT, "bvule": ir.B_ULE, "bvslt": ir.B_SLT, "bvsle": ir.B_SLE,
    "bvuadd_noovfl": ir.B_UADD_NOOVF, "bvumul_noovfl": ir.B_UMUL_NOOVF,
}
