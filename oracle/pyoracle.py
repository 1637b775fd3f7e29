"""ORACLE — test infrastructure only.  CPU restatement of the reference's hot-path arithmetic.

Nothing in the product (mythril_amd/) imports this module; only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg use it, as the checker.

What it restates
----------------
* z3 ``model.eval(expr, model_completion=True)`` for the SMT-LIB2 FixedSizeBitVectors ops that
  Mythril's SMT facade builds: mythril/laser/smt/bitvec.py:63-246 (``+ - *``, ``/`` = bvsdiv,
  signed ``< > <= >=``, ``>>`` = bvashr, ``<<``, ``& | ^``, padded ``==``),
  mythril/laser/smt/bitvec_helper.py:31-245 (UDiv/URem/SRem/LShR/If/Concat/Extract/ULT/UGT/
  ULE/UGE/BVAddNoOverflow/BVMulNoOverflow/BVSubNoUnderflow), mythril/laser/smt/bool.py:98-134
  (And/Or/Not/Xor).  z3 itself is the third-party dependency (z3-solver pinned
  ">=4.8.8.0,<=4.13.0.0", requirements.txt:25); it is not installed here, so this file restates
  the published SMT-LIB2 semantics with z3's total-division conventions:
  bvudiv x 0 = 2^w-1, bvurem x 0 = x, bvsdiv x 0 = (x<0 ? 1 : 2^w-1), bvsrem x 0 = x,
  bvsmod x 0 = x, shifts >= w -> 0 or the sign fill.
* The SAT criterion of ``ModelCache.check_quick_sat`` (mythril/support/support_utils.py:57-71):
  a candidate is a witness iff the conjunction evaluates to true under it.
* Keccak-256 as used by ``sha3`` (mythril/support/support_utils.py:93-101 via eth-hash,
  ``eth-hash>=0.3.1,<0.8.0`` requirements.txt:9, not installed): restated from the Keccak
  specification (pad10*1 with domain byte 0x01, NOT FIPS-202's 0x06).  Pinned against the
  reference's vmSha3Test digests (tests/golden/vmsha3.json) and the empty-input constant at
  mythril/laser/ethereum/function_managers/keccak_function_manager.py:87-93.
* The candidate-generator contract of include/pf_bytecode.h (our own design, restated here
  independently so the GPU's candidates can be regenerated and checked).

Parity pinning: EIP-145 shift vectors (reference tests/instructions/{sar,shl,shr}_test.py),
vmArithmeticTest / vmBitwiseLogicOperation fixtures (tests/golden/vmtests.json, evaluated through
tests/evm_to_ir.py) and vmSha3Test digests.  z3-only corner cases (division by zero at a symbolic
divisor, noovfl predicates) are not pinned by any reference test: "parity unpinned" for those,
covered by this restatement's own fixtures (tests/golden/ops.json).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

# --------------------------------------------------------------------------------------
# bit-vector semantics (SMT-LIB2 / z3), width-generic over Python ints
# --------------------------------------------------------------------------------------


def M(w: int) -> int:
    return (1 << w) - 1


def to_signed(x: int, w: int) -> int:
    return x - (1 << w) if (x >> (w - 1)) & 1 else x


def bvadd(a, b, w):
    return (a + b) & M(w)


def bvsub(a, b, w):
    return (a - b) & M(w)


def bvmul(a, b, w):
    return (a * b) & M(w)


def bvudiv(a, b, w):
    return M(w) if b == 0 else a // b


def bvurem(a, b, w):
    return a if b == 0 else a % b


def bvneg(a, w):
    return (-a) & M(w)


def bvnot(a, w):
    return (~a) & M(w)


def bvsdiv(a, b, w):
    # SMT-LIB2: defined through bvudiv on magnitudes (z3 follows it, incl. b == 0)
    sa, sb = (a >> (w - 1)) & 1, (b >> (w - 1)) & 1
    if not sa and not sb:
        return bvudiv(a, b, w)
    if sa and not sb:
        return bvneg(bvudiv(bvneg(a, w), b, w), w)
    if not sa and sb:
        return bvneg(bvudiv(a, bvneg(b, w), w), w)
    return bvudiv(bvneg(a, w), bvneg(b, w), w)


def bvsrem(a, b, w):
    sa, sb = (a >> (w - 1)) & 1, (b >> (w - 1)) & 1
    if not sa and not sb:
        return bvurem(a, b, w)
    if sa and not sb:
        return bvneg(bvurem(bvneg(a, w), b, w), w)
    if not sa and sb:
        return bvurem(a, bvneg(b, w), w)
    return bvneg(bvurem(bvneg(a, w), bvneg(b, w), w), w)


def bvsmod(a, b, w):
    sa, sb = (a >> (w - 1)) & 1, (b >> (w - 1)) & 1
    abs_a = bvneg(a, w) if sa else a
    abs_b = bvneg(b, w) if sb else b
    u = bvurem(abs_a, abs_b, w)
    if u == 0:
        return u
    if not sa and not sb:
        return u
    if sa and not sb:
        return bvadd(bvneg(u, w), b, w)
    if not sa and sb:
        return bvadd(u, b, w)
    return bvneg(u, w)


def bvshl(a, b, w):
    return 0 if b >= w else (a << b) & M(w)


def bvlshr(a, b, w):
    return 0 if b >= w else a >> b


def bvashr(a, b, w):
    if b >= w:
        return M(w) if (a >> (w - 1)) & 1 else 0
    return (to_signed(a, w) >> b) & M(w)


def bvexp(a, b, w):
    return pow(a, b, 1 << w)


def extract(a, lo, width):
    return (a >> lo) & M(width)


def concat(a, b, wb):
    return (a << wb) | b


def sign_extend(a, w_src, w):
    return to_signed(a, w_src) & M(w)


def ult(a, b, w):
    return a < b


def ule(a, b, w):
    return a <= b


def slt(a, b, w):
    return to_signed(a, w) < to_signed(b, w)


def sle(a, b, w):
    return to_signed(a, w) <= to_signed(b, w)


def uadd_noovf(a, b, w):
    return a + b <= M(w)


def umul_noovf(a, b, w):
    return a * b <= M(w)


# --------------------------------------------------------------------------------------
# Keccak-256 (original Keccak padding), from the specification
# --------------------------------------------------------------------------------------
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
        [27, 20, 39, 8, 14]]
_W64 = (1 << 64) - 1


def _rol(x, n):
    return ((x << n) | (x >> (64 - n))) & _W64 if n else x


def keccak_f1600(A: List[List[int]]) -> None:
    for rnd in range(24):
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        D = [C[(x - 1) % 5] ^ _rol(C[(x + 1) % 5], 1) for x in range(5)]
        for x in range(5):
            for y in range(5):
                A[x][y] ^= D[x]
        B = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                B[y][(2 * x + 3 * y) % 5] = _rol(A[x][y], _ROT[x][y])
        for x in range(5):
            for y in range(5):
                A[x][y] = B[x][y] ^ ((~B[(x + 1) % 5][y]) & B[(x + 2) % 5][y])
        A[0][0] ^= _RC[rnd]


def keccak256(data: bytes) -> bytes:
    rate = 136
    msg = bytearray(data)
    msg.append(0x01)
    while len(msg) % rate:
        msg.append(0)
    msg[-1] |= 0x80
    A = [[0] * 5 for _ in range(5)]
    for off in range(0, len(msg), rate):
        blk = msg[off:off + rate]
        for i in range(rate // 8):
            lane = int.from_bytes(blk[8 * i:8 * i + 8], "little")
            A[i % 5][i // 5] ^= lane
        keccak_f1600(A)
    out = b"".join(A[i % 5][i // 5].to_bytes(8, "little") for i in range(4))
    return out


# --------------------------------------------------------------------------------------
# candidate generator (include/pf_bytecode.h contract), vectorised over candidates
# --------------------------------------------------------------------------------------
PH_M0, PH_M1, PH_W0, PH_W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox4x32(ctr: Sequence[np.ndarray], key: Sequence[int]):
    c0, c1, c2, c3 = [np.asarray(x, dtype=np.uint64) & 0xFFFFFFFF for x in ctr]
    n = max(np.size(c0), np.size(c1), np.size(c2), np.size(c3))
    c0, c1, c2, c3 = [np.broadcast_to(x, (n,)).astype(np.uint64) for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(key[0] & 0xFFFFFFFF), np.uint64(key[1] & 0xFFFFFFFF)
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(PH_M0) * c0
        p1 = np.uint64(PH_M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & mask, lo1, (hi0 ^ c3 ^ k1) & mask, lo0
        k0 = (k0 + np.uint64(PH_W0)) & mask
        k1 = (k1 + np.uint64(PH_W1)) & mask
    return [x.astype(np.uint32) for x in (c0, c1, c2, c3)]


VK_GENERIC, VK_ACTOR, VK_KECCAK, VK_SMALL, VK_BOOL, VK_CDBYTE, VK_VALUE = 0, 1, 2, 3, 4, 5, 6


def mix32(x: int) -> int:
    """include/pf_bytecode.h mix32 (the calldata-byte arm's per-word hash)."""
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def uf_hash(x: int, salt: int) -> int:
    """PF_W_HASH (include/pf_bytecode.h): keyed 256-bit mix of x (restated)."""
    xs = [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
    h = [int(v[0]) for v in philox4x32([[xs[0]], [xs[1]], [xs[2]], [xs[3]]], (salt, 0x5BD1E995))]
    g = [int(v[0]) for v in philox4x32([[xs[4] ^ h[0]], [xs[5] ^ h[1]], [xs[6] ^ h[2]], [xs[7] ^ h[3]]],
                                       (salt, 0x27D4EB2F))]
    return sum(v << (32 * i) for i, v in enumerate(h + g))


def _boundary(j: int, k: int, w: int) -> int:
    m = M(w)
    table = (0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1,
             1 << k, (1 << k) - 1, (1 << k) + 1, (1 << 160) - 1)
    return table[j] & m


def gen_values(cands: np.ndarray, var_index: int, schema: Sequence[int], consts: Sequence[int],
               parent: Optional[int], set_seed: int, global_seed: int) -> List[int]:
    """Values of variable ``var_index`` for the candidate indices ``cands``."""
    cands = np.asarray(cands, dtype=np.uint64)
    kind, width = schema[0] & 0xFF, (schema[0] >> 8) & 0x3FF
    hint0, hint1 = schema[1], schema[2]
    key = ((global_seed & 0xFFFFFFFF) ^ (set_seed & 0xFFFFFFFF), (global_seed >> 32) & 0xFFFFFFFF)
    blocks = [philox4x32((cands, var_index, b, 0), key) for b in range(3)]
    r = blocks[0] + blocks[1]
    m = blocks[2]
    w = width
    out = []
    for i, c in enumerate(cands.tolist()):
        ri = [int(x[i]) for x in r]
        mi = [int(x[i]) for x in m]
        if c == 0 and parent is not None:
            out.append(parent & M(w))
            continue
        if parent is not None and (c & 1) and (mi[3] & ((4 << ((c >> 1) & 3)) - 1)) != 0:
            out.append(parent & M(w))  # neighbourhood candidate of the parent model
            continue
        rv = sum(x << (32 * j) for j, x in enumerate(ri))
        if kind == VK_KECCAK:
            lo = consts[hint0]
            k = (rv & M(128)) & M(117)
            out.append((lo + (k << 6)) & M(w))
            continue
        if kind == VK_SMALL:
            if (mi[0] & 16) and 4 <= hint0 < 0xFFFFFFFF:
                out.append((4 + 32 * (ri[1] % ((hint0 - 4) // 32 + 1))) & M(w))
            else:
                out.append((ri[0] % (hint0 + 1)) & M(w))
            continue
        if kind == VK_VALUE and (mi[0] & 16):
            out.append(0)
            continue
        if kind == VK_BOOL:
            out.append(ri[0] & 1)
            continue
        if kind == VK_ACTOR and (mi[1] % 4) < hint1:
            out.append(consts[hint0 + mi[1] % 4] & M(w))
            continue
        wk, ws = (hint0 >> 8) & 0xFFF, hint0 >> 20
        if wk == 0:
            wk, ws = len(consts), 0
        if kind == VK_CDBYTE and wk:
            u = mix32(c ^ key[0] ^ (hint1 * 0x9E3779B9))
            if u & 1:
                word = (consts[ws + (u >> 1) % wk] + (0, 1, -1, 0)[u >> 30]) & M(256)
                out.append((word >> (hint0 & 0xFF)) & 0xFF & M(w))
                continue
        sel = mi[0] & 15
        if sel <= 4:
            v = rv
        elif sel <= 8:
            v = _boundary(mi[1] % 12, mi[2] % w, w)
        elif sel <= 11:
            if consts:
                v = consts[mi[1] % len(consts)] + (0, 1, -1)[mi[2] % 3]
            else:
                v = rv
        elif sel <= 13:
            if parent is not None:
                v = parent
                if (mi[1] & 3) == 0:
                    v ^= 1 << (mi[2] % w)
            else:
                v = ri[0] & 0xFF
        else:
            v = ri[0] & ((1 << (1 + mi[1] % 16)) - 1)
        out.append(v & M(w))
    return out


# --------------------------------------------------------------------------------------
# bytecode evaluator (decodes the raw arrays of mythril_amd.ir.Batch independently)
# --------------------------------------------------------------------------------------
OP = dict(END=0, W_CONST=1, W_VAR=2, W_MOV=3, W_ADD=4, W_SUB=5, W_MUL=6, W_UDIV=7, W_UREM=8,
          W_SDIV=9, W_SREM=10, W_SMOD=11, W_AND=12, W_OR=13, W_XOR=14, W_NOT=15, W_NEG=16,
          W_SHL=17, W_LSHR=18, W_ASHR=19, W_EXP=20, W_EXTRACT=21, W_CONCAT=22, W_SEXT=23,
          W_ITE=24, W_HASH=25, W_SPILL=26, W_FILL=27, B_CONST=40, B_VAR=41, B_EQ=42, B_ULT=43, B_ULE=44, B_SLT=45, B_SLE=46,
          B_AND=47, B_OR=48, B_XOR=49, B_NOT=50, B_ITE=51, B_UADD_NOOVF=52, B_UMUL_NOOVF=53,
          B_FILL=54, B_SPILL=55, ASSERT=60)

_WBIN = {
    OP["W_ADD"]: bvadd, OP["W_SUB"]: bvsub, OP["W_MUL"]: bvmul, OP["W_UDIV"]: bvudiv,
    OP["W_UREM"]: bvurem, OP["W_SDIV"]: bvsdiv, OP["W_SREM"]: bvsrem, OP["W_SMOD"]: bvsmod,
    OP["W_AND"]: lambda a, b, w: a & b, OP["W_OR"]: lambda a, b, w: a | b,
    OP["W_XOR"]: lambda a, b, w: a ^ b, OP["W_SHL"]: bvshl, OP["W_LSHR"]: bvlshr,
    OP["W_ASHR"]: bvashr, OP["W_EXP"]: bvexp,
}
_BCMP = {
    OP["B_EQ"]: lambda a, b, w: a == b, OP["B_ULT"]: ult, OP["B_ULE"]: ule,
    OP["B_SLT"]: slt, OP["B_SLE"]: sle, OP["B_UADD_NOOVF"]: uadd_noovf,
    OP["B_UMUL_NOOVF"]: umul_noovf,
}


def limbs_to_int(row) -> int:
    v = 0
    for i, x in enumerate(row):
        v |= int(x) << (32 * i)
    return v


class SetView:
    """One set of a packed batch, decoded from the raw C-ABI arrays."""

    def __init__(self, code, consts, schema, parents, desc):
        d = [int(x) for x in desc]
        self.code = [tuple(int(x) for x in row) for row in code[d[0]:d[0] + d[1]]]
        self.consts = [limbs_to_int(row) for row in consts[d[2]:d[2] + d[3]]]
        self.schema = [tuple(int(x) for x in row) for row in schema[d[4]:d[4] + d[5]]]
        self.seed = d[6]
        self.parents: List[Optional[int]] = []
        for s in self.schema:
            slot = s[3]
            self.parents.append(None if slot == 0xFFFFFFFF else limbs_to_int(parents[slot]))

    @classmethod
    def from_batch(cls, batch, i):
        return cls(batch.code, batch.consts, batch.schema, batch.parents, batch.descs[i])

    def var_width(self, v):
        return (self.schema[v][0] >> 8) & 0x3FF

    def gen_assignments(self, cands, global_seed) -> List[List[int]]:
        cols = [gen_values(cands, v, self.schema[v], self.consts, self.parents[v], self.seed,
                           global_seed) for v in range(len(self.schema))]
        return [list(x) for x in zip(*cols)] if cols else [[] for _ in range(len(cands))]

    def evaluate(self, values: Sequence[int]) -> bool:
        """Evaluate the conjunction under one assignment (values indexed by variable)."""
        W: Dict[int, int] = {}
        B: Dict[int, bool] = {}
        S: Dict[int, int] = {}   # spill slots
        root = True
        for (w0, w1, aux0, aux1) in self.code:
            op, w = w0 & 0xFF, (w0 >> 8) & 0x3FF
            d, a, b, c = w1 & 0xFF, (w1 >> 8) & 0xFF, (w1 >> 16) & 0xFF, (w1 >> 24) & 0xFF
            if op == OP["END"]:
                break
            elif op == OP["W_CONST"]:
                W[d] = self.consts[aux0] & M(w)
            elif op == OP["W_VAR"]:
                W[d] = int(values[aux0]) & M(w)
            elif op == OP["W_MOV"]:
                W[d] = W[a] & M(w)
            elif op in _WBIN:
                W[d] = _WBIN[op](W[a], W[b], w)
            elif op == OP["W_NOT"]:
                W[d] = bvnot(W[a], w)
            elif op == OP["W_NEG"]:
                W[d] = bvneg(W[a], w)
            elif op == OP["W_EXTRACT"]:
                W[d] = extract(W[a], aux0, w)
            elif op == OP["W_CONCAT"]:
                W[d] = concat(W[a], W[b], aux0) & M(w)
            elif op == OP["W_SEXT"]:
                W[d] = sign_extend(W[a], aux0, w)
            elif op == OP["W_ITE"]:
                W[d] = W[a] if B[c] else W[b]
            elif op == OP["W_HASH"]:
                W[d] = uf_hash(W[a], aux0) & M(w)
            elif op == OP["W_SPILL"]:
                S[aux0] = W[a]
            elif op == OP["W_FILL"]:
                W[d] = S[aux0] & M(w)
            elif op == OP["B_SPILL"]:
                S[aux0] = int(B[a])
            elif op == OP["B_FILL"]:
                B[d] = bool(S[aux0] & 1)
            elif op == OP["B_CONST"]:
                B[d] = bool(aux0 & 1)
            elif op == OP["B_VAR"]:
                B[d] = bool(int(values[aux0]) & 1)
            elif op in _BCMP:
                B[d] = bool(_BCMP[op](W[a], W[b], w))
            elif op == OP["B_AND"]:
                B[d] = B[a] and B[b]
            elif op == OP["B_OR"]:
                B[d] = B[a] or B[b]
            elif op == OP["B_XOR"]:
                B[d] = B[a] != B[b]
            elif op == OP["B_NOT"]:
                B[d] = not B[a]
            elif op == OP["B_ITE"]:
                B[d] = B[a] if B[c] else B[b]
            elif op == OP["ASSERT"]:
                root = root and B[a]
            else:
                raise ValueError(f"oracle: unknown opcode {op}")
        return root

    def check(self, n_cand: int, global_seed: int):
        """First satisfying candidate index in [0, n_cand) (or None) and the SAT mask."""
        cands = np.arange(n_cand, dtype=np.uint64)
        assigns = self.gen_assignments(cands, global_seed)
        sat = [self.evaluate(a) for a in assigns]
        first = next((i for i, s in enumerate(sat) if s), None)
        return first, sat
