"""Lower a bit-vector DAG (a Mythril constraint set) to the flat register bytecode.

Input is a :class:`Dag`: hash-consed nodes in topological order (leaves: variables and
constants; interior nodes: one IR opcode each) plus the list of root Bool nodes whose
conjunction is the query — exactly what ``get_model`` receives as ``constraints``
(mythril/support/model.py:87-93) after ``Constraints.get_all_constraints`` appended the
keccak conditions (mythril/laser/ethereum/state/constraints.py:132-133).

Register allocation is a linear scan over an emission order that evaluates one root at a
time (so PF_ASSERT can short-circuit a wave as early as possible).  Interior values stay
resident until their last use; leaves (PF_W_VAR / PF_W_CONST / bool leaves) are
rematerialised when registers run out (Belady: evict the leaf used farthest in the future).
A set that would need more than PF_NW live interior values raises :class:`LoweringError`
and is left to z3 (the engine never guesses).
"""

from __future__ import annotations

import bisect
import os

from dataclasses import dataclass, field
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple  # noqa: F401

from . import ir
from .ir import Ins, Program, Var

# node kinds beyond IR opcodes
K_VAR = "var"       # aux = variable index      (W or B by width: width 0 => bool var)
K_CONST = "const"   # aux = value
K_BCONST = "bconst"  # aux = 0/1
K_BVAR = "bvar"     # aux = variable index


class LoweringError(ValueError):
    """The set uses a shape the GPU bytecode does not cover; it falls back to z3."""


class Node(NamedTuple):
    """One DAG node; a tuple, so it is its own hash-consing key (Dag.add)."""
    kind: object          # IR opcode (int) or one of the K_* leaf kinds
    width: int            # result width for W nodes, operand width for compares, 1 for bools
    args: Tuple[int, ...] = ()
    aux: int = 0
    is_bool: bool = False


@dataclass
class Dag:
    nodes: List[Node] = field(default_factory=list)
    roots: List[int] = field(default_factory=list)
    vars: List[Var] = field(default_factory=list)
    forced: List[int] = field(default_factory=list)  # constants pinned at pool index 0..
    _memo: Dict[tuple, int] = field(default_factory=dict)
    _var_index: Dict[str, int] = field(default_factory=dict)

    def force_consts(self, values) -> int:
        """Pin constants at known pool indices (schema hints refer to them)."""
        start = len(self.forced)
        self.forced.extend(int(v) & ir.mask(ir.MAX_WIDTH) for v in values)
        return start

    def add(self, kind, width, args=(), aux=0, is_bool=False) -> int:
        node = Node(kind, width, args if type(args) is tuple else tuple(args), aux, is_bool)
        i = self._memo.get(node)
        if i is None:
            i = len(self.nodes)
            self.nodes.append(node)
            self._memo[node] = i
        return i

    # ---- leaves --------------------------------------------------------------------
    def var(self, name: str, width: int, kind: int = ir.VK_GENERIC, hint0: int = 0,
            hint1: int = 0, parent: Optional[int] = None) -> int:
        idx = self._var_index.get(name)
        if idx is None:
            idx = len(self.vars)
            self.vars.append(Var(name, width, kind, hint0, hint1, parent))
            self._var_index[name] = idx
        if kind == ir.VK_BOOL:
            return self.add(K_BVAR, 1, (), idx, True)
        return self.add(K_VAR, width, (), idx)

    def const(self, value: int, width: int) -> int:
        return self.add(K_CONST, width, (), value & ir.mask(width))

    def bconst(self, value: bool) -> int:
        return self.add(K_BCONST, 1, (), int(bool(value)), True)

    # ---- interior ------------------------------------------------------------------
    def op(self, opcode: int, width: int, *args: int, aux: int = 0) -> int:
        r = self._simplify(opcode, width, args, aux)
        if r is not None:
            return r
        is_bool = opcode >= ir.B_CONST
        return self.add(opcode, width, args, aux, is_bool)

    def _cval(self, i: int) -> Optional[int]:
        n = self.nodes[i]
        return n.aux if n.kind == K_CONST else None

    def _simplify(self, op: int, w: int, args, aux) -> Optional[int]:
        """Word-slicing rewrites z3.simplify applies to every stored constraint
        (constraints.py:60-70): selector and address extraction from a CALLDATALOAD word
        (a 32-byte concat, calldata.py:233-246) keep only the bytes they read, so the
        program and the hint derivation see 4 / 20 byte variables instead of 32."""
        nodes = self.nodes
        if op == ir.W_UDIV:                       # x / 2^k -> x >> k
            c = self._cval(args[1])
            if c is not None and c and c & (c - 1) == 0:
                k = c.bit_length() - 1
                return args[0] if k == 0 else self.op(ir.W_LSHR, w, args[0], self.const(k, w))
        elif op == ir.W_LSHR:
            k = self._cval(args[1])
            x = nodes[args[0]]
            if k is not None and k < w:
                if k == 0:
                    return args[0]
                if x.kind == ir.W_MOV:                # zero-extended: shift the inner value
                    inner = x.args[0]
                    wi = nodes[inner].width
                    if k >= wi:
                        return self.const(0, w)
                    return self.op(ir.W_MOV, w, self.op(ir.W_EXTRACT, wi - k, inner, aux=k))
                if x.kind == ir.W_CONCAT:
                    return self.op(ir.W_MOV, w, self.op(ir.W_EXTRACT, w - k, args[0], aux=k))
        elif op == ir.W_AND:
            for xi, ci in ((0, 1), (1, 0)):
                c = self._cval(args[ci])
                if c is not None and c and (c + 1) & c == 0 and c.bit_length() < w:
                    k = c.bit_length()                # x & (2^k - 1) -> zext(x[k-1:0])
                    return self.op(ir.W_MOV, w, self.op(ir.W_EXTRACT, k, args[xi], aux=0))
        elif op == ir.W_EXTRACT:
            x = nodes[args[0]]
            if aux == 0 and w == x.width:
                return args[0]
            if x.kind == ir.W_CONCAT:
                hi, lo = x.args
                wl = x.aux
                if aux >= wl:
                    return self.op(ir.W_EXTRACT, w, hi, aux=aux - wl)
                if aux + w <= wl:
                    return self.op(ir.W_EXTRACT, w, lo, aux=aux)
                top = self.op(ir.W_EXTRACT, aux + w - wl, hi, aux=0)
                bot = self.op(ir.W_EXTRACT, wl - aux, lo, aux=aux)
                return self.op(ir.W_CONCAT, w, top, bot, aux=wl - aux)
            if x.kind == ir.W_MOV:
                inner = x.args[0]
                wi = nodes[inner].width
                if aux + w <= wi:
                    return self.op(ir.W_EXTRACT, w, inner, aux=aux)
                if aux >= wi:
                    return self.const(0, w)
            if x.kind == K_CONST:
                return self.const(x.aux >> aux, w)
        elif op == ir.W_MOV:
            x = nodes[args[0]]
            if x.width == w:
                return args[0]
            if x.kind == ir.W_MOV:
                return self.op(ir.W_MOV, w, x.args[0])
            if x.kind == K_CONST:
                return self.const(x.aux, w)
        elif op == ir.B_EQ:
            for xi, ci in ((0, 1), (1, 0)):
                c = self._cval(args[ci])
                x = nodes[args[xi]]
                if c is not None and x.kind == ir.W_MOV:   # zext(y) == c  ->  y == c  (or false)
                    wy = nodes[x.args[0]].width
                    if c >> wy:
                        return self.bconst(False)
                    return self.op(ir.B_EQ, wy, x.args[0], self.const(c, wy))
        return None

    _CMP_OPS = (ir.B_EQ, ir.B_ULT, ir.B_ULE, ir.B_SLT, ir.B_SLE)

    def word_constants(self) -> List[int]:
        """Constants the set compares values against (selectors, bounds, addresses): the
        calldata-byte generator arm spells whole ABI words from these (include/pf_bytecode.h
        PF_VK_CDBYTE).  Comparisons with a size variable (LASER's per-byte ``i <s size``
        guards, calldata.py:233-246) are skipped: their index constants would crowd out
        the words that matter."""
        nodes, out, seen = self.nodes, [], set()
        for nd in nodes:
            if nd.kind not in self._CMP_OPS:
                continue
            a, b = (nodes[x] for x in nd.args)
            for c, other in ((a, b), (b, a)):
                if c.kind != K_CONST:
                    continue
                if other.kind == K_VAR and self.vars[other.aux].kind == ir.VK_SMALL:
                    continue
                if c.aux not in seen:
                    seen.add(c.aux)
                    out.append(c.aux)
        return out[:0xFFF]

    def finalize_word_hints(self) -> None:
        """Pin the word constants in the pool and point every calldata-byte variable at them
        (hint0 bits 8..31: count and start); idempotent."""
        if getattr(self, "_words_done", False):
            return
        self._words_done = True
        cds = [v for v in self.vars if v.kind == ir.VK_CDBYTE]
        if not cds:
            return
        words = self.word_constants()
        if not words or len(self.forced) >= 0xFFF:
            return
        start = self.force_consts(words)
        for v in cds:
            v.hint0 = (v.hint0 & 0xFF) | (len(words) << 8) | (start << 20)

    def assert_(self, b: int) -> None:
        if not self.nodes[b].is_bool:
            raise LoweringError("root is not a Bool")
        self.roots.append(b)

    def width(self, i: int) -> int:
        return self.nodes[i].width


_LEAF_KINDS = (K_VAR, K_CONST, K_BCONST, K_BVAR)


def _subtree_sizes(dag: Dag) -> List[int]:
    """Interior nodes below each node (shared subterms counted once per path, capped)."""
    size = [0] * len(dag.nodes)
    for i, n in enumerate(dag.nodes):   # topological: operands come first
        if n.kind not in _LEAF_KINDS:
            size[i] = min(1 + sum(size[a] for a in n.args), 1 << 20)
    return size


def _emission_order(dag: Dag) -> List[Tuple[str, int]]:
    """Post-order per root (roots in order); ('node', i) and ('assert', i) events.

    Operands are visited largest subtree first (Sethi-Ullman): the small operand is then
    computed right before its use instead of being held live across the big one.  That is
    what keeps an ``ite`` chain (an array read checked against every earlier index,
    mythril_amd/smt/to_dag.py) at two live values instead of one per link."""
    size = _subtree_sizes(dag)
    seen = set()
    events: List[Tuple[str, int]] = []
    for r in dag.roots:
        stack = [(r, False)]
        while stack:
            i, done = stack.pop()
            n = dag.nodes[i]
            if n.kind in _LEAF_KINDS:
                continue
            if done:
                if i not in seen:
                    seen.add(i)
                    events.append(("node", i))
                continue
            if i in seen:
                continue
            stack.append((i, True))
            # the stack pops the last push first: push the smallest operand first
            for a in sorted(n.args, key=lambda x: size[x]):
                if dag.nodes[a].kind not in _LEAF_KINDS and a not in seen:
                    stack.append((a, False))
        events.append(("assert", r))
    return events


class _RegFile:
    def __init__(self, n: int, cls: str):
        self.n = n
        self.cls = cls
        self.free = list(range(n - 1, -1, -1))
        self.holder: Dict[int, int] = {}   # reg -> node
        self.where: Dict[int, int] = {}    # node -> reg

    def alloc(self, node: int, evict_rank, pinned, spill=None, far=None, on_evict=None) -> int:
        """Take a free register, else evict the cheapest-to-restore value (evict_rank;
        on_evict(reg, node) may spill it first), else spill the value used farthest in the
        future (spill(reg, node) emits it)."""
        if self.free:
            # the lowest free register: the narrow kernels keep their highest register out
            # of VGPRs when pressure demands (pf_eval.hip), so it should be the rarest one
            r = min(self.free)
            self.free.remove(r)
        else:
            cands = [(evict_rank(nd), rg) for rg, nd in self.holder.items() if rg not in pinned]
            cands = [c for c in cands if c[0] is not None]
            if cands:
                _, r = min(cands)
                if on_evict is not None:
                    on_evict(r, self.holder[r])
            else:
                victims = [(far(nd), rg) for rg, nd in self.holder.items() if rg not in pinned]
                if not victims or spill is None or not spill(max(victims)[1], self.holder[max(victims)[1]]):
                    raise LoweringError(f"more than {self.n} live {self.cls} values")
                r = max(victims)[1]
            old = self.holder.pop(r)
            del self.where[old]
        self.holder[r] = node
        self.where[node] = r
        return r

    def release(self, node: int) -> None:
        r = self.where.pop(node, None)
        if r is not None:
            del self.holder[r]
            self.free.append(r)


_REMAT_MAX = 6     # nodes re-emitted to restore one evicted interior value
_REMAT_OPCOST = 16  # only cheap ops (compare/ite/logic/extract/concat) are recomputed
# eviction price of re-emitting a variable, in cheap instructions: a generator run (three
# Philox blocks + the strategy arms) measured ~6x a cheap op's time on the GPU, so under the
# 7-register file a constant or a short recomputation is evicted before a variable
_VAR_REMAT_COST = 6
# ... but an evicted variable that is used again is spilled while a slot is free (one
# W_SPILL now, one W_FILL per restore: scratch round trips, no generator run): storage-heavy
# LASER buckets re-read their ~70 symbols across ~1,200 array-aliasing compares, which at 7
# registers re-ran the generator for every read (1,186 W_VAR for 69 variables in the
# heaviest corpus bucket — most of its search time)
_VAR_SPILL_COST = 2
# ... only when at least this many uses remain after the eviction (1 = any later use); the
# native lowering reads the same environment variable (pf_lower.cpp)
def _var_spill_uses() -> int:
    return max(1, int(os.environ.get("PF_VAR_SPILL_USES", "1")))


# ... and at least this many when a W_EXP runs before the variable's last use: the device
# program's LDS spill slots (pathfeas.hip pass 4) are EXP's window-table entries, so such a
# spill lands in scratch — config 3 regenerates instead (WRITE_SIZE 34 -> 13 MB per launch
# at -0.3 %, profiles/r05z_spillexp_ab.md).  0 or <= PF_VAR_SPILL_USES: the one rule everywhere
def _var_spill_uses_exp() -> int:
    return max(0, int(os.environ.get("PF_VAR_SPILL_USES_EXP", "99")))


# ---- native lowering (libpflower.so, include/pf_lower.h) ----------------------------------
_KIND_CODE = {K_VAR: 200, K_CONST: 201, K_BCONST: 202, K_BVAR: 203}
_NATIVE = None


def _native():
    """ctypes handle of libpflower.so (host-only C ABI), or False if it is not built."""
    global _NATIVE
    if _NATIVE is None:
        import ctypes
        import os

        path = os.environ.get("PF_LOWER_SO") or os.path.join(
            os.path.dirname(os.path.abspath(__file__)), "libpflower.so")  # override: diagnostics
        if os.environ.get("PF_LOWER_PY") or not os.path.exists(path):
            _NATIVE = False
        else:
            L = ctypes.CDLL(path)
            u32p, szp = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t)
            L.pfl_lower.argtypes = [u32p, ctypes.c_size_t, u32p, ctypes.c_size_t, u32p,
                                    ctypes.c_size_t, u32p, ctypes.c_size_t, ctypes.c_uint32, u32p,
                                    ctypes.c_size_t, szp, u32p, ctypes.c_size_t, szp]
            L.pfl_lower.restype = ctypes.c_int
            L.pfl_hints.argtypes = [u32p, ctypes.c_size_t, u32p, ctypes.c_size_t, u32p,
                                    ctypes.c_size_t, u32p, ctypes.c_size_t, u32p, u32p,
                                    ctypes.POINTER(ctypes.c_int)]
            L.pfl_hints.restype = ctypes.c_int
            L.pfl_last_error.restype = ctypes.c_char_p
            _NATIVE = L
    return _NATIVE


def limbs(vals):
    """256-bit values as rows of 8 little-endian u32 limbs (one zero row if empty)."""
    import numpy as np

    return ir.limbs_array(vals) if vals else np.zeros((1, 8), dtype=np.uint32)


def pack_nodes(dag: Dag):
    """The node table of include/pf_lower.h (8 u32 per node; constants moved to a pool):
    (nodes array, pool limbs, pool values)."""
    import numpy as np

    cached = getattr(dag, "_packed", None)
    if cached is not None and cached[0] == len(dag.nodes):
        return cached[1]
    flat: List[int] = []
    pool: List[int] = []
    kc = _KIND_CODE
    for n in dag.nodes:
        aux = n.aux
        if n.kind == K_CONST:
            aux = len(pool)
            pool.append(n.aux)
        a = n.args
        la = len(a)
        flat += (kc.get(n.kind, n.kind), n.width, la, a[0] if la > 0 else 0, a[1] if la > 1 else 0,
                 a[2] if la > 2 else 0, aux & 0xFFFFFFFF, 1 if n.is_bool else 0)
    out = (np.array(flat or [0] * 8, dtype=np.uint32), limbs(pool), pool)
    dag._packed = (len(dag.nodes), out)  # nodes are append-only: hints and lower share it
    return out


def _spill_code(prog) -> Tuple[int, int]:
    """(instructions, W spill + fill instructions) of a program."""
    if isinstance(prog, ir.PackedProgram):
        ops = prog.words[:, 0] & 0xFF
        return len(ops), int(((ops == ir.W_SPILL) | (ops == ir.W_FILL)).sum())
    return len(prog.code), sum(1 for ins in prog.code if ins.op in (ir.W_SPILL, ir.W_FILL))


def _spill_heavy(prog) -> bool:
    """More than an eighth of the program is W spill / fill code.  A program with a few
    spills still runs faster in the 8-register kernels (4 waves/SIMD, the scratch round trips
    of a spill cost about a cheap op) than in the 16-register ones at 2 waves/SIMD — and its
    batch then needs no second launch (config 3: 0.4 % of the DAGs, 2-8 spill/fill
    instructions each, were the whole 0.2 ms r16 launch per step).  pf_terms.cpp applies the
    same policy."""
    n, ns = _spill_code(prog)
    return 8 * ns > n


def lower(dag: Dag, seed: int = 0, name: str = "", nw: Optional[int] = None) -> Program:
    """Register allocation + emission.  Without ``nw``: over ir.NW_NARROW registers first —
    such a program runs the 8-register, 4-waves/SIMD search kernels — and over all ir.NW
    when that would make it spill-heavy (:func:`_spill_heavy`) or cannot fit (the
    16-register kernels then run its batch).  The native library when built (identical output, tests/test_native_lower.py),
    else the Python reference :func:`lower_py`."""
    if nw is None:
        dag.finalize_word_hints()
        narrow = None
        try:
            narrow = lower(dag, seed, name, ir.NW_NARROW)
            if not _spill_heavy(narrow):
                return narrow
        except LoweringError:
            pass
        try:
            wide = lower(dag, seed, name, ir.NW)
        except (LoweringError, ValueError, OverflowError):
            # any failure of the wide lowering keeps a valid narrow program (pf_terms.cpp
            # does the same)
            if narrow is None:
                raise
            return narrow
        # a spill-heavy narrow program moves to the wide register file only when that at
        # least halves its spill code (storage-heavy buckets whose evicted symbols spill
        # under 15 registers too stay at 4 waves/SIMD)
        if narrow is not None and 2 * _spill_code(wide)[1] > _spill_code(narrow)[1]:
            return narrow
        return wide
    L = _native()
    if not L:
        return lower_py(dag, seed, name, nw)
    import ctypes

    import numpy as np

    nn = len(dag.nodes)
    arr, pool_a, pool = pack_nodes(dag)
    forced_a = limbs(dag.forced)
    roots = np.array(dag.roots or [0], dtype=np.uint32)
    cap_i = 16 * nn + 64 + 4 * len(dag.roots)
    cap_c = len(pool) + len(dag.forced) + 1
    ni, nc = ctypes.c_size_t(), ctypes.c_size_t()
    p = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))  # noqa: E731
    for _ in range(4):
        code = np.zeros((cap_i, 4), dtype=np.uint32)
        consts = np.zeros((cap_c, 8), dtype=np.uint32)
        rc = L.pfl_lower(p(arr), nn, p(pool_a), len(pool), p(roots), len(dag.roots), p(forced_a),
                         len(dag.forced), nw, p(code), cap_i, ctypes.byref(ni), p(consts), cap_c,
                         ctypes.byref(nc))
        if rc != -3:
            break
        # output capacity: rematerialisation and spill code under register pressure can
        # exceed the estimate; the library checks before writing, so retry larger
        cap_i, cap_c = 4 * cap_i, 4 * cap_c
    if rc != 0:
        msg = L.pfl_last_error().decode(errors="replace")
        if rc == -2:
            raise LoweringError(msg)
        raise ValueError(f"pfl_lower failed ({rc}): {msg}")
    raw = consts[:nc.value].astype("<u4").tobytes()
    cvals = [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(nc.value)]
    return ir.PackedProgram(code[:ni.value].copy(), cvals, list(dag.vars), seed, name)


def lower_py(dag: Dag, seed: int = 0, name: str = "", nw: int = ir.NW) -> Program:
    """Python reference of the lowering (the native library reproduces it exactly)."""
    prog = Program(vars=list(dag.vars), seed=seed, name=name)
    prog.consts.extend(dag.forced)  # schema hints index these (actor tables, keccak bases)
    events = _emission_order(dag)
    uses: Dict[int, List[int]] = {}
    for t, (kind, i) in enumerate(events):
        if kind == "node":
            for a in dag.nodes[i].args:
                uses.setdefault(a, []).append(t)
        else:
            uses.setdefault(i, []).append(t)

    def next_use(nd: int, now: int) -> int:
        lst = uses.get(nd, [])
        lo, hi = 0, len(lst)
        while lo < hi:  # first use > now
            mid = (lo + hi) // 2
            if lst[mid] <= now:
                lo = mid + 1
            else:
                hi = mid
        return lst[lo] if lo < len(lst) else 1 << 30

    remat_memo: Dict[int, Optional[int]] = {}

    def remat_size(nd: int) -> Optional[int]:
        """Nodes to re-emit to restore nd (None = must stay resident)."""
        if nd in remat_memo:
            return remat_memo[nd]
        n = dag.nodes[nd]
        if n.kind in _LEAF_KINDS:
            res: Optional[int] = 1
        elif ir.op_cost(n.kind, n.width) > _REMAT_OPCOST or n.kind == ir.W_EXP:
            res = None
        else:
            tot = 1
            for a in n.args:
                sa = remat_size(a)
                if sa is None:
                    tot = None
                    break
                tot += sa
            res = tot if tot is not None and tot <= _REMAT_MAX else None
        remat_memo[nd] = res
        return res

    cost_memo: Dict[int, int] = {}

    def remat_cost(nd: int) -> int:
        """GPU price of re-emitting nd (only called when remat_size(nd) is not None)."""
        c = cost_memo.get(nd)
        if c is None:
            n = dag.nodes[nd]
            if n.kind in (K_VAR, K_BVAR):
                c = _VAR_REMAT_COST
            elif n.kind in _LEAF_KINDS:
                c = 1
            else:
                c = 1 + sum(remat_cost(a) for a in n.args)
            cost_memo[nd] = c
        return c

    W = _RegFile(nw, "W")
    B = _RegFile(ir.NB, "B")
    # spill slots (PF_W_SPILL / PF_B_SPILL): values that can neither stay resident nor be
    # recomputed cheaply; a spilled value keeps its slot until its last use, so evicting
    # it again costs nothing and restoring it is one fill
    slot_of: Dict[int, int] = {}
    free_slots = list(range(ir.MAX_SPILL - 1, -1, -1))
    filling: List[Optional[int]] = [None]   # the spilled node materialize() is restoring

    min_uses = _var_spill_uses()
    exp_uses = _var_spill_uses_exp()
    exp_at = [t for t, (kind, i) in enumerate(events) if kind == "node" and dag.nodes[i].kind == ir.W_EXP]

    def uses_after(nd: int, now: int) -> int:
        lst = uses.get(nd, [])
        return len(lst) - bisect.bisect_right(lst, now)

    def var_min_uses(nd: int, now: int) -> int:
        """Uses a variable evicted at ``now`` must still have to be spilled, not regenerated."""
        lst = uses.get(nd, [])
        if exp_uses <= min_uses or not lst:
            return min_uses
        k = bisect.bisect_right(exp_at, now)
        return exp_uses if k < len(exp_at) and exp_at[k] < lst[-1] else min_uses

    def rank(t):
        def f(nd):
            if nd in slot_of:
                cost = 1
            elif remat_size(nd) is None:
                return None
            elif dag.nodes[nd].kind == K_VAR and free_slots and uses_after(nd, t) >= var_min_uses(nd, t):
                cost = _VAR_SPILL_COST
            else:
                cost = remat_cost(nd)
            # cheapest restore first, then farthest next use (Belady)
            return (cost, -next_use(nd, t))
        return f

    def spill(rg: int, nd: int, t: int = 0, steal: bool = True) -> bool:
        if not free_slots:
            # a value that cannot be recomputed takes the slot of a spilled variable (the
            # one used farthest in the future; its later restores re-run the generator)
            # (never the variable materialize() is filling now: its slot is read after the
            # register is allocated)
            vs = [v for v in sorted(slot_of) if dag.nodes[v].kind == K_VAR and v != filling[0]] \
                if steal else []
            if not vs:
                return False
            far_v = vs[0]
            for v in vs[1:]:
                if next_use(v, t) >= next_use(far_v, t):
                    far_v = v
            free_slots.append(slot_of.pop(far_v))
        s = free_slots.pop()
        n = dag.nodes[nd]
        if n.is_bool:
            prog.emit(ir.B_SPILL, 1, a=rg, aux0=s)
        else:
            prog.emit(ir.W_SPILL, n.width, a=rg, aux0=s)
        slot_of[nd] = s
        return True

    def alloc(rf, nd, t, pinned):
        def on_evict(rg, old):
            if dag.nodes[old].kind == K_VAR and old not in slot_of and free_slots \
                    and uses_after(old, t) >= var_min_uses(old, t):
                spill(rg, old, t, False)
        return rf.alloc(nd, rank(t), pinned, lambda rg, x: spill(rg, x, t), lambda x: next_use(x, t),
                        on_evict)

    def done(nd):
        regfile(nd).release(nd)
        s = slot_of.pop(nd, None)
        if s is not None:
            free_slots.append(s)

    def regfile(nd):
        return B if dag.nodes[nd].is_bool else W

    def emit_node(i: int, t: int, pinned_w: set, pinned_b: set) -> int:
        n = dag.nodes[i]
        rf = regfile(i)
        if n.kind in _LEAF_KINDS:
            r = alloc(rf, i, t, pinned_b if n.is_bool else pinned_w)
            if n.kind == K_VAR:
                prog.emit(ir.W_VAR, n.width, dst=r, aux0=n.aux)
            elif n.kind == K_CONST:
                prog.emit(ir.W_CONST, n.width, dst=r, aux0=prog.const_index(n.aux))
            elif n.kind == K_BCONST:
                prog.emit(ir.B_CONST, 1, dst=r, aux0=n.aux)
            else:
                prog.emit(ir.B_VAR, 1, dst=r, aux0=n.aux)
            return r
        pw, pb = set(pinned_w), set(pinned_b)
        regs = []
        for a in n.args:
            r = materialize(a, t, pw, pb)
            (pb if dag.nodes[a].is_bool else pw).add(r)
            regs.append(r)
        # operands whose last use is this node may be reused as destination — except an
        # operand the caller has pinned: when this node is being rematerialised as an operand
        # of an enclosing node, that node may already hold the same value as one of its own
        # operands (a remat's use shares the enclosing event time t), and releasing it here
        # let this node's result overwrite it
        for a in dict.fromkeys(n.args):   # distinct operands, in argument order
            r = regs[n.args.index(a)]
            if next_use(a, t) >= (1 << 30) and r not in (pinned_b if dag.nodes[a].is_bool else pinned_w):
                done(a)
                (pb if dag.nodes[a].is_bool else pw).discard(r)
        dst = alloc(rf, i, t, pb if n.is_bool else pw)
        op = n.kind
        if op in (ir.W_ITE, ir.B_ITE):      # args: cond(B), then, else
            prog.emit(op, n.width if op == ir.W_ITE else 1, dst=dst, a=regs[1], b=regs[2], c=regs[0])
        else:
            a = regs[0] if len(regs) > 0 else 0
            b = regs[1] if len(regs) > 1 else 0
            prog.emit(op, n.width, dst=dst, a=a, b=b, aux0=n.aux)
        return dst

    def materialize(nd: int, t: int, pinned_w: set, pinned_b: set) -> int:
        rf = regfile(nd)
        if nd in rf.where:
            return rf.where[nd]
        if nd in slot_of:
            n = dag.nodes[nd]
            slot, outer = slot_of[nd], filling[0]
            filling[0] = nd
            r = alloc(rf, nd, t, pinned_b if n.is_bool else pinned_w)
            filling[0] = outer
            if n.is_bool:
                prog.emit(ir.B_FILL, 1, dst=r, aux0=slot)
            else:
                prog.emit(ir.W_FILL, n.width, dst=r, aux0=slot)
            return r
        if dag.nodes[nd].kind not in _LEAF_KINDS and remat_size(nd) is None:
            raise LoweringError("non-rematerialisable value was evicted")
        return emit_node(nd, t, pinned_w, pinned_b)

    for t, (kind, i) in enumerate(events):
        if kind == "assert":
            rb = materialize(i, t, set(), set())
            prog.emit(ir.ASSERT, 1, a=rb)
            if next_use(i, t) >= (1 << 30):
                done(i)
            continue
        if i in regfile(i).where or i in slot_of:
            continue  # already (re)computed as an operand of an earlier node
        emit_node(i, t, set(), set())
        if next_use(i, t) >= (1 << 30):
            done(i)
    prog.finish()
    prog.validate()
    return prog
