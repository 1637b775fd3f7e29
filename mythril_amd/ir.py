"""Flat register bytecode for batched path-feasibility (Python mirror of include/pf_bytecode.h).

A :class:`Program` is one constraint set — the conjunction Mythril hands to
``get_model`` (mythril/support/model.py:63-125) — lowered to 4-word instructions over
two register classes (W: 256-bit, B: bool).  A :class:`Batch` concatenates many
programs into the flat arrays the C ABI (include/pathfeas.h) consumes.

The opcode numbers are checked against the C header by tests/test_abi.py.
"""

from __future__ import annotations

import re
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

NW = 15  # usable W registers; register 15 is the kernel's write sink
NW_NARROW = 7  # PF_NW_NARROW: programs within it run the 8-register, 3-waves/SIMD kernels
NB = 32
LIMBS = 8
MAX_WIDTH = 256
MAX_SPILL = 64   # spill slots per lane (PF_MAX_SPILL)
NO_PARENT = 0xFFFFFFFF

# ---- opcodes (pf_bytecode.h enum pf_opcode) ------------------------------------
END = 0
W_CONST = 1
W_VAR = 2
W_MOV = 3
W_ADD = 4
W_SUB = 5
W_MUL = 6
W_UDIV = 7
W_UREM = 8
W_SDIV = 9
W_SREM = 10
W_SMOD = 11
W_AND = 12
W_OR = 13
W_XOR = 14
W_NOT = 15
W_NEG = 16
W_SHL = 17
W_LSHR = 18
W_ASHR = 19
W_EXP = 20
W_EXTRACT = 21
W_CONCAT = 22
W_SEXT = 23
W_ITE = 24
W_HASH = 25
W_SPILL = 26
W_FILL = 27
B_CONST = 40
B_VAR = 41
B_EQ = 42
B_ULT = 43
B_ULE = 44
B_SLT = 45
B_SLE = 46
B_AND = 47
B_OR = 48
B_XOR = 49
B_NOT = 50
B_ITE = 51
B_UADD_NOOVF = 52
B_UMUL_NOOVF = 53
B_FILL = 54
B_SPILL = 55
ASSERT = 60

OPNAMES = {v: k for k, v in dict(globals()).items()
           if k.isupper() and isinstance(v, int) and (k.startswith(("W_", "B_")) or k in ("END", "ASSERT"))}

# binary W -> W ops
W_BINARY = (W_ADD, W_SUB, W_MUL, W_UDIV, W_UREM, W_SDIV, W_SREM, W_SMOD, W_AND, W_OR,
            W_XOR, W_SHL, W_LSHR, W_ASHR, W_EXP)
W_UNARY = (W_NOT, W_NEG, W_MOV, W_HASH)
B_CMP = (B_EQ, B_ULT, B_ULE, B_SLT, B_SLE, B_UADD_NOOVF, B_UMUL_NOOVF)
B_LOGIC = (B_AND, B_OR, B_XOR)

# ---- datapath units (w0 bits 21..23, set by pf_batch_create from the opcode) --------
U_ALU = 0
U_MUL = 1
U_DIV = 2
U_SHIFT = 3
U_GEN = 4
U_CMP = 5
U_BOOL = 6
U_END = 7

# ---- variable kinds --------------------------------------------------------------
VK_GENERIC = 0
VK_ACTOR = 1
VK_KECCAK = 2
VK_SMALL = 3
VK_BOOL = 4
VK_CDBYTE = 5
VK_VALUE = 6
CDBYTE_RE = re.compile(r"^\d+_calldata\[(\d+)\]$")


def cdbyte_hints(name: str) -> Tuple[int, int]:
    """Schema hints of the PF_VK_CDBYTE variable ``{tx}_calldata[i]``: (bit position of the
    byte in its big-endian ABI word, word id).  LASER reads calldata words big-endian
    (state/calldata.py:233-246): bytes 0..3 are the selector (word id 0xFFFFFFFF), byte
    4 + 32 k + j is byte j of argument word k."""
    i = int(CDBYTE_RE.match(name).group(1))
    if i < 4:
        return 8 * (3 - i), 0xFFFFFFFF
    k, j = divmod(i - 4, 32)
    return 8 * (31 - j), k

# ---- flags -----------------------------------------------------------------------
FLAG_SHORTCIRCUIT = 1
FLAG_EARLY_EXIT = 2
FLAG_COUNT_OPS = 4
FLAG_NO_PROBE = 8     # include/pf_bytecode.h: skip the candidate-0 probe launch

# ---- algorithmic int32-op cost table -----------------------------
# Ops not in the table (moves, constant loads, candidate generation) cost 0: they are
# bookkeeping, not constraint arithmetic.  Width-generic ops scale by ceil(w/32)/8.
_COST256 = {
    W_ADD: 8, W_SUB: 8, W_NOT: 8, W_AND: 8, W_OR: 8, W_XOR: 8, W_NEG: 8,
    W_ITE: 8, W_EXTRACT: 8, W_CONCAT: 8, W_SEXT: 8, W_HASH: 0,
    B_EQ: 8, B_ULT: 8, B_ULE: 8, B_SLT: 8, B_SLE: 8,
    W_SHL: 16, W_LSHR: 16, W_ASHR: 16,
    W_MUL: 72, B_UMUL_NOOVF: 72, B_UADD_NOOVF: 8,
    W_UDIV: 256, W_UREM: 256, W_SDIV: 280, W_SREM: 280, W_SMOD: 280,
    W_EXP: 512 * 72,
}


# ---- reachable int32-op cost table (the roofline's `achieved`) -----------------------
# The §8(d) table prices EXP as square-and-always-multiply (512 products) and division as
# an 8-digit schoolbook quotient; the kernel's algorithms need far less, so that table's
# "achieved" can exceed the VALU peak.  This table prices each node at the work of the
# algorithm the kernel actually runs, so achieved <= peak:
#   EXP      2-adic split: ~35 256-bit product equivalents (2-bit window over 8 exponent
#            bits, 7 truncated squarings, ~25-term truncated Horner chain) x 72 = 2,520
#   UDIV/UREM  Knuth algorithm D on 8 x 32-bit digits, worst case over divisor length n:
#            (9 - n) quotient digits x (n mads + n subtracts + 4 estimate ops) + 2 x 16
#            normalisation shifts, max at n = 4 -> 92, rounded to 96
#   SDIV/SREM/SMOD  + three 8-limb negations = 120;  UMUL_NOOVF is one division = 96
#   HASH     two Philox4x32-10 blocks = 20 rounds x 6 ops = 120
_COST256_REACH = dict(_COST256)
_COST256_REACH.update({
    W_EXP: 35 * 72, W_UDIV: 96, W_UREM: 96, W_SDIV: 120, W_SREM: 120, W_SMOD: 120,
    B_UMUL_NOOVF: 96, W_HASH: 120,
})


def _scaled(c: Optional[int], width: int) -> int:
    if c is None:
        return 0
    nl = (max(1, width) + 31) // 32
    return (c * nl + 7) // 8


def op_cost(op: int, width: int) -> int:
    """Algorithmic int32 ops of one node, scaled by width."""
    return _scaled(_COST256.get(op), width)


def reach_cost(op: int, width: int) -> int:
    """Int32 ops of one node at the kernel's own algorithms (``_COST256_REACH``)."""
    return _scaled(_COST256_REACH.get(op), width)


def mask(w: int) -> int:
    return (1 << w) - 1


def to_limbs(v: int, n: int = LIMBS) -> List[int]:
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def limbs_array(values: Sequence[int]) -> np.ndarray:
    """Many 256-bit values as rows of 8 little-endian u32 limbs (bulk to_limbs)."""
    if not values:
        return np.zeros((0, LIMBS), dtype=np.uint32)
    m = (1 << (32 * LIMBS)) - 1
    buf = b"".join((int(v) & m).to_bytes(4 * LIMBS, "little") for v in values)
    return np.frombuffer(buf, dtype="<u4").reshape(-1, LIMBS).astype(np.uint32)


def from_limbs(limbs: Sequence[int]) -> int:
    v = 0
    for i, x in enumerate(limbs):
        v |= int(x) << (32 * i)
    return v


@dataclass
class Var:
    """One free symbol of a constraint set (candidate schema entry)."""

    name: str
    width: int
    kind: int = VK_GENERIC
    hint0: int = 0
    hint1: int = 0
    parent: Optional[int] = None  # parent-model value, if known


@dataclass
class Ins:
    op: int
    width: int = 256
    dst: int = 0
    a: int = 0
    b: int = 0
    c: int = 0
    aux0: int = 0
    aux1: int = 0
    flags: int = 0

    def words(self):
        return (
            (self.op & 0xFF) | ((self.width & 0x3FF) << 8) | ((self.flags & 0x3FFF) << 18),
            (self.dst & 0xFF) | ((self.a & 0xFF) << 8) | ((self.b & 0xFF) << 16) | ((self.c & 0xFF) << 24),
            self.aux0 & 0xFFFFFFFF,
            self.aux1 & 0xFFFFFFFF,
        )

    def __repr__(self):
        return (f"{OPNAMES.get(self.op, self.op)}/w{self.width} d={self.dst} a={self.a} "
                f"b={self.b} c={self.c} x={self.aux0}")


@dataclass
class Program:
    """One lowered constraint set."""

    code: List[Ins] = field(default_factory=list)
    consts: List[int] = field(default_factory=list)
    vars: List[Var] = field(default_factory=list)
    seed: int = 0
    name: str = ""

    def const_index(self, value: int) -> int:
        value &= mask(MAX_WIDTH)
        try:
            return self.consts.index(value)
        except ValueError:
            self.consts.append(value)
            return len(self.consts) - 1

    def emit(self, *args, **kw) -> Ins:
        ins = Ins(*args, **kw)
        self.code.append(ins)
        return ins

    def finish(self) -> "Program":
        if not self.code or self.code[-1].op != END:
            self.code.append(Ins(END, 1))
        return self

    @property
    def has_parent(self) -> bool:
        return any(v.parent is not None for v in self.vars)

    def node_cost(self) -> int:
        return sum(op_cost(i.op, i.width) for i in self.code)

    def reach_cost(self) -> int:
        return sum(reach_cost(i.op, i.width) for i in self.code)

    def sched_cost(self) -> int:
        """Relative device time of one candidate evaluation: measured SIMD cycles per
        instruction (EXP ~11x, division ~4x, MUL ~1.2x a cheap op) — the model
        pf_batch_create orders waves by, used here to balance shards across devices."""
        c = 0
        for i in self.code:
            c += (110 if i.op == W_EXP else 12 if i.op == W_MUL
                  else 40 if (W_UDIV <= i.op <= W_SMOD or i.op == B_UMUL_NOOVF) else 10)
        return c

    def validate(self) -> None:
        """Host-side shape check run before anything is launched (kernel assumes these)."""
        spilled = set()
        for i, ins in enumerate(self.code):
            if ins.op not in OPNAMES:
                raise ValueError(f"ins {i}: unknown opcode {ins.op}")
            if ins.op != END and not (1 <= ins.width <= MAX_WIDTH):
                raise ValueError(f"ins {i}: width {ins.width} out of range")
            w_regs, b_regs = _reg_classes(ins.op)
            for r in w_regs(ins):
                if r >= NW:
                    raise ValueError(f"ins {i}: W register {r} >= {NW}")
            for r in b_regs(ins):
                if r >= NB:
                    raise ValueError(f"ins {i}: B register {r} >= {NB}")
            if ins.op in (W_VAR, B_VAR) and ins.aux0 >= len(self.vars):
                raise ValueError(f"ins {i}: variable {ins.aux0} out of range")
            if ins.op == W_CONST and ins.aux0 >= len(self.consts):
                raise ValueError(f"ins {i}: constant {ins.aux0} out of range")
            if ins.op in (W_SPILL, W_FILL, B_SPILL, B_FILL):
                if ins.aux0 >= MAX_SPILL:
                    raise ValueError(f"ins {i}: spill slot {ins.aux0} >= {MAX_SPILL}")
                if ins.op in (W_SPILL, B_SPILL):
                    spilled.add(ins.aux0)
                elif ins.aux0 not in spilled:
                    raise ValueError(f"ins {i}: spill slot {ins.aux0} filled before it was spilled")
        if not self.code or self.code[-1].op != END:
            raise ValueError("program must end with END")


def _reg_classes(op):
    """(W registers used, B registers used) of an instruction, as accessor functions."""
    if op in (W_CONST, W_VAR, W_FILL):
        return (lambda i: (i.dst,)), (lambda i: ())
    if op == W_SPILL:
        return (lambda i: (i.a,)), (lambda i: ())
    if op == B_FILL:
        return (lambda i: ()), (lambda i: (i.dst,))
    if op == B_SPILL:
        return (lambda i: ()), (lambda i: (i.a,))
    if op in W_UNARY or op in (W_EXTRACT, W_SEXT):
        return (lambda i: (i.dst, i.a)), (lambda i: ())
    if op in W_BINARY or op == W_CONCAT:
        return (lambda i: (i.dst, i.a, i.b)), (lambda i: ())
    if op == W_ITE:
        return (lambda i: (i.dst, i.a, i.b)), (lambda i: (i.c,))
    if op in B_CMP:
        return (lambda i: (i.a, i.b)), (lambda i: (i.dst,))
    if op in (B_CONST, B_VAR):
        return (lambda i: ()), (lambda i: (i.dst,))
    if op in B_LOGIC:
        return (lambda i: ()), (lambda i: (i.dst, i.a, i.b))
    if op == B_NOT:
        return (lambda i: ()), (lambda i: (i.dst, i.a))
    if op == B_ITE:
        return (lambda i: ()), (lambda i: (i.dst, i.a, i.b, i.c))
    if op == ASSERT:
        return (lambda i: ()), (lambda i: (i.a,))
    return (lambda i: ()), (lambda i: ())


class PackedProgram(Program):
    """A Program whose instructions are held packed, 4 x u32 each (the native lowering's
    output, include/pf_lower.h); ``code`` decodes them into :class:`Ins` on first use."""

    def __init__(self, words: np.ndarray, consts: List[int], vars: List[Var], seed: int = 0,
                 name: str = ""):
        self.words = np.ascontiguousarray(words, dtype=np.uint32).reshape(-1, 4)
        self.consts = consts
        self.vars = vars
        self.seed = seed
        self.name = name
        self._code: Optional[List[Ins]] = None

    @property
    def code(self) -> List[Ins]:  # type: ignore[override]
        if self._code is None:
            out = []
            for w0, w1, a0, a1 in self.words.tolist():
                out.append(Ins(w0 & 0xFF, (w0 >> 8) & 0x3FF, w1 & 0xFF, (w1 >> 8) & 0xFF,
                               (w1 >> 16) & 0xFF, (w1 >> 24) & 0xFF, a0, a1, (w0 >> 18) & 0x3FFF))
            self._code = out
        return self._code

    def __len__(self):
        return len(self.words)


class Batch:
    """Many programs packed into the flat arrays of the C ABI (pf_set_desc et al.)."""

    def __init__(self, programs: Sequence[Program]):
        self.programs = list(programs)
        if self.programs and all(getattr(p, "native_result", None) is not None for p in self.programs):
            # natively lowered (smt/native_terms.py): packed from the results in C++
            from .smt.native_terms import pack_batch

            self.code, self.consts, self.schema, self.parents, self.descs = pack_batch(self.programs)
            return
        code, consts, schema, parents, descs = [], [], [], [], []
        packed = []   # (offset in code, words) of natively lowered programs
        for p in self.programs:
            d_code = len(code)
            if isinstance(p, PackedProgram):
                # validated by pf_batch_create (ranges, def-before-use, spill slots)
                packed.append((d_code, p.words))
                code.extend([None] * len(p.words))
            else:
                p.validate()
                for ins in p.code:
                    w0, w1, a0, _ = ins.words()
                    # aux1 carries the node's int32-op cost at the kernel's algorithms
                    # (PF_FLAG_COUNT_OPS; reach_cost, so the roofline's achieved <= peak)
                    code.append((w0, w1, a0, reach_cost(ins.op, ins.width) if ins.op != END else 0))
            d_const = len(consts)
            consts.extend(p.consts)
            d_var = len(schema)
            has_par = p.has_parent
            d_par = len(parents) if has_par else NO_PARENT
            for v in p.vars:
                slot = NO_PARENT
                if has_par and v.parent is not None:
                    slot = len(parents)
                    parents.append(v.parent & mask(v.width))
                schema.append((v.kind | (v.width << 8), v.hint0 & 0xFFFFFFFF,
                               v.hint1 & 0xFFFFFFFF, slot))
            descs.append((d_code, len(code) - d_code, d_const, len(p.consts), d_var, len(p.vars),
                          p.seed & 0xFFFFFFFF, d_par))
        if packed:
            arr = np.zeros((len(code), 4), dtype=np.uint32)
            rows = [i for i, c in enumerate(code) if c is not None]
            if rows:
                arr[rows] = np.asarray([code[i] for i in rows], dtype=np.uint32)
            for off, words in packed:
                w = words.copy()
                w[:, 3] = _reach_cost_words(w)
                arr[off:off + len(w)] = w
            self.code = arr
        else:
            self.code = np.asarray(code, dtype=np.uint32).reshape(-1, 4)
        self.consts = limbs_array(consts)
        self.schema = np.asarray(schema, dtype=np.uint32).reshape(-1, 4)
        self.parents = limbs_array(parents)
        self.descs = np.asarray(descs, dtype=np.uint32).reshape(-1, 8)

    def __len__(self):
        return len(self.programs)

    def node_costs(self) -> np.ndarray:
        return np.array([p.node_cost() for p in self.programs], dtype=np.int64)


_REACH_LUT = None


def reach_lut() -> np.ndarray:
    """reach_cost by (op, width): a 256 x 1024 u32 table."""
    global _REACH_LUT
    if _REACH_LUT is None:
        lut = np.zeros((256, 1024), dtype=np.uint32)
        for op in _COST256_REACH:
            for w in range(1, MAX_WIDTH + 1):
                lut[op, w] = reach_cost(op, w)
        _REACH_LUT = lut
    return _REACH_LUT


_OP_LUT = None


def op_cost_words(words: np.ndarray) -> int:
    """Sum of ``op_cost`` (the SURVEY §8(d) table) over packed instructions, vectorised."""
    global _OP_LUT
    if _OP_LUT is None:
        lut = np.zeros((256, 1024), dtype=np.int64)
        for op in range(256):
            for w in range(1, MAX_WIDTH + 1):
                try:
                    lut[op, w] = op_cost(op, w)
                except Exception:  # noqa: BLE001 - opcodes outside the table cost 0
                    pass
        _OP_LUT = lut
    words = np.asarray(words, dtype=np.uint32).reshape(-1, 4)
    return int(_OP_LUT[words[:, 0] & 0xFF, (words[:, 0] >> 8) & 0x3FF].sum())


def _reach_cost_words(words: np.ndarray) -> np.ndarray:
    """reach_cost of packed instructions, vectorised: a (op, width) lookup table."""
    op = words[:, 0] & 0xFF
    w = (words[:, 0] >> 8) & 0x3FF
    return reach_lut()[op, w]


def pack_assignments(prog: Program, cands: Sequence[Sequence[int]]) -> np.ndarray:
    """Explicit candidates -> SoA limbs [var][limb][cand] (coalesced on the GPU)."""
    n = len(cands)
    out = np.zeros((max(1, len(prog.vars)), LIMBS, n), dtype=np.uint32)
    for c, vals in enumerate(cands):
        for v, val in enumerate(vals):
            val = int(val) & mask(prog.vars[v].width)
            for l in range(LIMBS):
                out[v, l, c] = (val >> (32 * l)) & 0xFFFFFFFF
    return out


def pack_assignments_np(limbs: np.ndarray) -> np.ndarray:
    """[cand][var][limb] uint32 -> [var][limb][cand]."""
    return np.ascontiguousarray(np.transpose(limbs, (1, 2, 0)))


def u32_bytes(words: Sequence[int]) -> bytes:
    return struct.pack(f"<{len(words)}I", *words)
