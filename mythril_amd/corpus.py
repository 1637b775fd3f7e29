"""LASER-shaped feasibility queries with planted models (BASELINE config 2 substitute).

Config 2 of BASELINE.json asks for the constraint sets Mythril dumps (``--solver-log``,
mythril/support/model.py:46-57) while analysing rubixi.sol / etherstore.sol at ``-t 2``.
Those dumps need z3 + solc, neither of which exists in this image, so this module builds the
same *kind* of queries directly with the engine's SMT facade, term for term the way LASER
builds them:

* message-call transactions (transaction/symbolic.py:103-147,207-216): ``sender_<tx>``,
  ``call_value<tx>``, ``<tx>_calldatasize``, ``<tx>_calldata``; the actor disjunction
  ``Or(caller == a)``; the value transfer ``UGE(balance[sender], value)`` and the balance
  stores (transaction_models.py:135-152);
* CALLDATALOAD words as 32 ``If(i <s size, calldata[i], 0)`` bytes (state/calldata.py:233-246);
* the solc dispatcher (``calldatasize < 4``, selector by SHR (solc >= 0.5) or by DIV+AND
  (solc 0.4)), the non-payable ``iszero(callvalue)`` check, the ABI argument-size check,
  address masking;
* JUMPI exactly as instructions.py:1589-1660 forks: a Bool condition is asserted as is /
  negated, a BitVec one as ``!= 0`` / ``== 0``; EQ / ISZERO / LT / GT push what
  instructions.py:672-765 push;
* storage as ``K(0)`` plus stores (account.py:18-29, concrete storage of a contract created
  in the analysis), mapping slots through the keccak function manager
  (instructions.py:1014-1048, keccak_function_manager.py:95-114), whose conditions are
  appended to every query (constraints.py:132-133).

Contracts: the logic of the solidity_examples the BASELINE names (token, BECToken-style
batch transfer, EtherStore, Rubixi, KillBilly, a wallet with owner indices), re-described,
not copied.

Every scenario fixes a *planted model* first (actors, call values, calldata bytes, the
balance array) and follows, at every JUMPI, the branch the planted model takes.  Queries are
issued where LASER issues them: both successors of every fork (svm.py:351-358) and every
open state at a transaction boundary (svm.py:266-286).  A query on the planted side is SAT
by construction (the planted model satisfies it under the engine's keccak interpretation,
checked here when the corpus is built); the other side is unlabelled (z3 would decide it).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .keccak_manager import KeccakFunctionManager
from .smt import (UGE, UGT, ULT, And, BitVec, Bool, Concat, If, Not, Or,  # noqa: F401
                  UDiv, symbol_factory)
from .smt import terms as T
from .smt.expr import BVAddNoOverflow, LShR
from .smt.interp import Witness
from .smt.to_dag import ACTORS, UFRegistry

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym
CONTRACT = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F
M160 = (1 << 160) - 1
ETHER = 10 ** 18


@dataclass
class Query:
    constraints: List[T.Term]
    label: str          # "sat" (planted side / tx boundary) or "open" (other fork side)
    origin: str         # contract.function:site
    planted: Optional["Planted"] = None


@dataclass
class Planted:
    """The planted model: values of free symbols and base-array contents."""

    vars: Dict[str, int] = field(default_factory=dict)
    arrays: Dict[str, Dict[int, int]] = field(default_factory=dict)


class _PlantedEval(Witness):
    """Term evaluation under a planted model with the engine's interpretation of arrays
    and keccak (mythril_amd/smt/interp.py) — what the GPU would compute for it."""

    def __init__(self, planted: Planted, registry: UFRegistry):
        self.reg = registry
        self.vars = planted.vars
        self.bools = {}
        self.reads = {}
        self.array_reads = {}
        self.uf_apps = []
        self._memo = {}
        self._tables = planted.arrays
        self._pos = None
        self._keccak_tables = {}


class Path:
    """One LASER execution path under a planted model."""

    def __init__(self, corpus: "Corpus", planted: Planted, name: str):
        self.c = corpus
        self.p = planted
        self.name = name
        self.cs: List[T.Term] = []
        self.storage = T.const_array(256, T.const(0, 256))
        self.balance = T.array("balance", 256, 256)
        self.tx = 0
        self.alive = True
        self.site = ""

    # ---- evaluation under the planted model --------------------------------------------
    def truth(self, b: T.Term) -> bool:
        return bool(_PlantedEval(self.p, self.c.kfm.registry).ev(b))

    def value(self, t: T.Term) -> int:
        return int(_PlantedEval(self.p, self.c.kfm.registry).ev(t))

    def _all(self) -> List[T.Term]:
        return self.cs + [self.c.kfm.create_conditions().raw]

    # ---- transactions ---------------------------------------------------------------------
    def begin_tx(self, actor: int, value: int, calldata: bytes):
        self.tx += 1
        tx = self.tx
        self.sender = BV(f"sender_{tx}", 256)
        self.value_sym = BV(f"call_value{tx}", 256)
        self.size = BV(f"{tx}_calldatasize", 256)
        self.cd = T.array(f"{tx}_calldata", 256, 8)
        self.p.vars[f"sender_{tx}"] = actor
        self.p.vars[f"call_value{tx}"] = value
        self.p.vars[f"{tx}_calldatasize"] = len(calldata)
        self.p.arrays[f"{tx}_calldata"] = {i: b for i, b in enumerate(calldata)}
        self.cs.append(Or(*[self.sender == BVV(a, 256) for a in ACTORS]).raw)
        bal = BitVec(T.select(self.balance, self.sender.raw))
        self.cs.append(UGE(bal, self.value_sym).raw)
        recv = T.const(CONTRACT, 256)
        self.balance = T.store(self.balance, recv, T.binop("bvadd", T.select(self.balance, recv), self.value_sym.raw))
        self.balance = T.store(self.balance, self.sender.raw,
                               T.binop("bvsub", T.select(self.balance, self.sender.raw), self.value_sym.raw))
        self.alive = True

    def end_tx(self):
        """Tx boundary: LASER re-checks every open state (svm.py:279-283)."""
        if self.alive:
            self.c.issue(self._all(), "sat", f"{self.name}:tx{self.tx}-boundary", self.p)

    # ---- EVM values as LASER builds them --------------------------------------------------
    def calldataload(self, off) -> BitVec:
        if isinstance(off, int):
            idx = [BVV(off + i, 256) for i in range(32)]
        else:
            idx = [off + BVV(i, 256) for i in range(32)]
        size = self.size
        parts = [If(i < size, BitVec(T.select(self.cd, i.raw)), BVV(0, 8)) for i in idx]
        return Concat(parts)

    def sload(self, slot: BitVec) -> BitVec:
        return BitVec(T.select(self.storage, slot.raw))

    def sstore(self, slot: BitVec, v: BitVec):
        self.storage = T.store(self.storage, slot.raw, v.raw)

    def mapping(self, key: BitVec, slot: int) -> BitVec:
        return self.c.kfm.create_keccak(Concat(key, BVV(slot, 256)))

    def timestamp(self) -> BitVec:
        sym = BV(f"{self.tx}_timestamp", 256)
        self.p.vars.setdefault(f"{self.tx}_timestamp", 1_700_000_000 + 86400 * 10 * self.tx)
        return sym

    def retval(self, pc: int) -> BitVec:
        name = f"{self.tx}_retval_{pc}"
        self.p.vars.setdefault(name, 1)
        return BV(name, 256)

    # ---- control flow -----------------------------------------------------------------------
    def jumpi(self, cond, site: str) -> bool:
        """Fork as instructions.py:1589-1660 does; returns the planted branch (True = jump)."""
        if not self.alive:
            return False
        if isinstance(cond, Bool):
            condi, negated = cond, Not(cond)
        else:
            condi, negated = cond != 0, cond == 0
        taken = self.truth(condi.raw)
        for side, c in ((True, condi), (False, negated)):
            if c.raw is T.FALSE:
                continue
            self.c.issue(self._all() + [c.raw], "sat" if side == taken else "open",
                         f"{self.name}:tx{self.tx}:{site}:{'T' if side else 'F'}", self.p)
        self.cs.append((condi if taken else negated).raw)
        return taken

    def require(self, cond, site: str) -> bool:
        ok = self.jumpi(cond, site)
        if not ok:
            self.alive = False
        return ok


def iszero(x) -> BitVec:
    """ISZERO (instructions.py:748-765)."""
    e = Not(x) if isinstance(x, Bool) else (x == 0)
    return If(e, BVV(1, 256), BVV(0, 256))


def addr(word: BitVec) -> BitVec:
    return word & BVV(M160, 256)


# ---- contracts --------------------------------------------------------------------------
@dataclass
class Fn:
    name: str
    selector: int
    n_args: int
    payable: bool
    body: Callable[[Path, List[BitVec]], None]


@dataclass
class Contract:
    name: str
    fns: List[Fn]
    solc_div: bool = False                         # solc 0.4 DIV/AND dispatcher
    ctor: Optional[Callable[[Path], None]] = None


def _dispatch(path: Path, k: Contract, fn: Fn) -> Optional[List[BitVec]]:
    """Dispatcher + prologue (calldatasize / selector / callvalue / ABI size checks)."""
    if path.jumpi(ULT(path.size, BVV(4, 256)), "calldatasize<4"):
        path.alive = False                         # fallback path (not modelled further)
        return None
    w0 = path.calldataload(0)
    sel = (UDiv(w0, BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)) if k.solc_div else LShR(w0, BVV(224, 256))
    for f in k.fns:
        if path.jumpi(sel == BVV(f.selector, 256), f"dispatch-{f.name}"):
            if f is not fn:
                path.alive = False
                return None
            break
    else:
        path.alive = False
        return None
    if not fn.payable and not path.require(iszero(path.value_sym), "nonpayable"):
        return None
    if fn.n_args and not k.solc_div:
        need = BVV(32 * fn.n_args, 256)
        if not path.require(iszero(ULT(path.size - BVV(4, 256), need)), "abi-size"):
            return None
    return [path.calldataload(4 + 32 * i) for i in range(fn.n_args)]


def _token(sel_base: int, batch: bool) -> Contract:
    BAL = 1

    def ctor(p: Path):
        p.sstore(BVV(0, 256), BVV(10 ** 27, 256))                      # totalSupply
        p.sstore(p.mapping(BVV(ACTORS[0], 256), BAL), BVV(10 ** 27, 256))

    def transfer(p: Path, a):
        to, val = addr(a[0]), a[1]
        me = p.mapping(addr(p.sender), BAL)
        bs = p.sload(me)
        if not p.require(iszero(ULT(bs, val)), "balance>=value"):
            return
        dst = p.mapping(to, BAL)
        bt = p.sload(dst)
        p.c.issue(p._all() + [Not(BVAddNoOverflow(bt, val, False)).raw], "open", f"{p.name}:integer-add")
        if not p.require(iszero(ULT(bt + val, bt)), "no-overflow"):
            return
        p.sstore(me, bs - val)
        p.sstore(dst, p.sload(dst) + val)

    def batch_transfer(p: Path, a):
        # BECToken batchTransfer(address[] receivers, uint256 value): the ABI head holds the
        # array offset; the length is read at 4 + offset (a calldata read at a symbolic index)
        off, val = a[0], a[1]
        cnt = p.calldataload(off + BVV(4, 256))
        amount = cnt * val
        if not p.require(UGT(cnt, BVV(0, 256)), "cnt>0"):
            return
        if not p.require(iszero(UGT(cnt, BVV(20, 256))), "cnt<=20"):
            return
        if not p.require(UGT(val, BVV(0, 256)), "value>0"):
            return
        me = p.mapping(addr(p.sender), BAL)
        if not p.require(iszero(ULT(p.sload(me), amount)), "balance>=amount"):
            return
        p.sstore(me, p.sload(me) - amount)

    def approve(p: Path, a):
        spender, val = addr(a[0]), a[1]
        inner = p.mapping(addr(p.sender), 2)
        slot = p.c.kfm.create_keccak(Concat(spender, inner))
        p.sstore(slot, val)

    fns = [Fn("transfer", sel_base + 1, 2, False, transfer), Fn("approve", sel_base + 2, 2, False, approve)]
    if batch:
        fns.append(Fn("batchTransfer", sel_base + 3, 2, False, batch_transfer))
    return Contract("BECToken" if batch else "token", fns, ctor=ctor)


def _etherstore() -> Contract:
    LIMIT, LAST, BAL = 0, 1, 2

    def ctor(p: Path):
        p.sstore(BVV(LIMIT, 256), BVV(ETHER, 256))

    def deposit(p: Path, a):
        me = p.mapping(addr(p.sender), BAL)
        p.sstore(me, p.sload(me) + p.value_sym)

    def withdraw(p: Path, a):
        amt = a[0]
        me = p.mapping(addr(p.sender), BAL)
        if not p.require(iszero(ULT(p.sload(me), amt)), "balance>=amount"):
            return
        if not p.require(iszero(UGT(amt, p.sload(BVV(LIMIT, 256)))), "amount<=limit"):
            return
        last = p.mapping(addr(p.sender), LAST)
        now = p.timestamp()
        if not p.require(iszero(ULT(now, p.sload(last) + BVV(7 * 86400, 256))), "time-lock"):
            return
        if not p.require(p.retval(301) == 1, "call-success"):
            return
        p.sstore(me, p.sload(me) - amt)
        p.sstore(last, now)

    return Contract("EtherStore", [Fn("depositFunds", 0xE2C41DBC, 0, True, deposit),
                                   Fn("withdrawFunds", 0x155DD5EE, 1, False, withdraw)], solc_div=True, ctor=ctor)


def _rubixi() -> Contract:
    CREATOR, FEE, FEES = 0, 1, 2

    def ctor(p: Path):
        p.sstore(BVV(FEE, 256), BVV(10, 256))

    def dynamic_pyramid(p: Path, a):    # the misnamed "constructor": anyone becomes creator
        p.sstore(BVV(CREATOR, 256), addr(p.sender))

    def only_owner(p: Path) -> bool:
        return p.require(addr(p.sender) == addr(p.sload(BVV(CREATOR, 256))), "onlyowner")

    def collect_all(p: Path, a):
        if not only_owner(p):
            return
        if not p.require(UGT(p.sload(BVV(FEES, 256)), BVV(0, 256)), "fees>0"):
            return
        p.sstore(BVV(FEES, 256), BVV(0, 256))

    def change_fee(p: Path, a):
        fee = a[0]
        if not only_owner(p):
            return
        if not p.require(iszero(UGT(fee, BVV(10, 256))), "fee<=10"):
            return
        p.sstore(BVV(FEE, 256), fee)

    def enter(p: Path, a):
        if not p.require(iszero(ULT(p.value_sym, BVV(ETHER, 256))), "value>=1ether"):
            return
        fees = p.sload(BVV(FEES, 256))
        p.sstore(BVV(FEES, 256), fees + UDiv(p.value_sym * p.sload(BVV(FEE, 256)), BVV(100, 256)))

    return Contract("Rubixi", [Fn("DynamicPyramid", 0x57D4021B, 0, False, dynamic_pyramid),
                               Fn("collectAllFees", 0xB4022950, 0, False, collect_all),
                               Fn("changeFeePercentage", 0x8A5FB3CA, 1, False, change_fee),
                               Fn("enter", 0xE97DCB62, 0, True, enter)], solc_div=True, ctor=ctor)


def _killbilly() -> Contract:
    KILLABLE, APPROVED = 0, 1

    def killerize(p: Path, a):
        p.sstore(p.mapping(addr(a[0]), APPROVED), BVV(1, 256))

    def activate(p: Path, a):
        ok = p.sload(p.mapping(addr(p.sender), APPROVED))
        if not p.require(ok == BVV(1, 256), "approved[msg.sender]"):
            return
        p.sstore(BVV(KILLABLE, 256), BVV(1, 256))

    def commence(p: Path, a):
        if not p.require(p.sload(BVV(KILLABLE, 256)) != BVV(0, 256), "is_killable"):
            return

    return Contract("KillBilly", [Fn("killerize", 0x9FE4E0C2, 1, False, killerize),
                                  Fn("activatekillability", 0x84057065, 0, False, activate),
                                  Fn("commencekilling", 0x7C11DA20, 0, False, commence)])


def _wallet() -> Contract:
    NUM, REQ, IDX = 0, 1, 2

    def init_wallet(p: Path, a):
        if not p.require(p.sload(BVV(NUM, 256)) == BVV(0, 256), "only_uninitialized"):
            return
        req = a[0]
        if not p.require(iszero(UGT(req, BVV(8, 256))), "required<=8"):
            return
        p.sstore(BVV(NUM, 256), BVV(1, 256))
        p.sstore(BVV(REQ, 256), req)
        p.sstore(p.mapping(addr(p.sender), IDX), BVV(1, 256))

    def kill(p: Path, a):
        idx = p.sload(p.mapping(addr(p.sender), IDX))
        if not p.require(idx != BVV(0, 256), "onlyowner"):
            return
        if not p.require(iszero(UGT(p.sload(BVV(REQ, 256)), BVV(1, 256))), "onlymanyowners"):
            return

    def execute(p: Path, a):
        to, val = addr(a[0]), a[1]
        idx = p.sload(p.mapping(addr(p.sender), IDX))
        if not p.require(idx != BVV(0, 256), "onlyowner"):
            return
        if not p.require(iszero(ULT(p.sload(BVV(NUM, 256)) * BVV(ETHER, 256), val)), "daylimit"):
            return
        del to

    return Contract("WalletLibrary", [Fn("initWallet", 0xE46DCFEB, 1, False, init_wallet),
                                      Fn("kill", 0xCBF0B0C0, 1, False, kill),
                                      Fn("execute", 0xB61D27F6, 2, False, execute)])


CONTRACTS: Dict[str, Callable[[], Contract]] = {
    "token": lambda: _token(0xA9059CB0, False),
    "BECToken": lambda: _token(0x83F12FC0, True),
    "EtherStore": _etherstore,
    "Rubixi": _rubixi,
    "KillBilly": _killbilly,
    "WalletLibrary": _wallet,
}


class Corpus:
    def __init__(self, kfm: Optional[KeccakFunctionManager] = None):
        self.kfm = kfm or KeccakFunctionManager(UFRegistry())
        self.queries: List[Query] = []

    def issue(self, constraints: List[T.Term], label: str, origin: str, planted=None):
        cs = [c for c in constraints if c is not T.TRUE]
        self.queries.append(Query(cs, label, origin, planted))


def _calldata(rng, fn: Fn, actors_used: List[int], k: Contract) -> bytes:
    out = fn.selector.to_bytes(4, "big")
    for i in range(fn.n_args):
        kind = int(rng.integers(0, 4))
        if kind == 0 and actors_used:
            v = actors_used[int(rng.integers(0, len(actors_used)))]
        elif kind == 1:
            v = int(rng.integers(0, 2))
        elif kind == 2:
            v = int(rng.integers(1, 64))
        else:
            v = int(rng.integers(1, 1 << 62)) * int(rng.integers(1, 1 << 40))
        if fn.name == "batchTransfer" and i == 0:
            v = 64                                   # array offset
        out += v.to_bytes(32, "big")
    if fn.name == "batchTransfer":
        out += int(rng.integers(1, 25)).to_bytes(32, "big")   # receivers.length
    return out


def live_order_groups(queries: Sequence[Query]) -> List[List[Query]]:
    """The queries as a live analysis poses them, in issue order: both successors of a fork
    together (svm.py:351-358 checks a fork's pair back to back) and each tx-boundary query
    on its own (svm.py:279-283)."""
    out: List[List[Query]] = []
    cur: List[Query] = []
    key = None
    for q in queries:
        k = q.origin.rsplit(":", 1)[0] if q.origin.endswith((":T", ":F")) else q.origin
        if k != key and cur:
            out.append(cur)
            cur = []
        key = k
        cur.append(q)
    if cur:
        out.append(cur)
    return out


def build(n_scenarios: int = 24, txs: int = 2, seed: int = 2024,
          contracts: Optional[Sequence[str]] = None,
          kfm: Optional[KeccakFunctionManager] = None) -> Corpus:
    """``n_scenarios`` planted transaction sequences of ``txs`` message calls each, spread
    over the contracts; returns every query LASER would issue along them."""
    rng = np.random.default_rng(seed)
    names = list(contracts or CONTRACTS)
    corpus = Corpus(kfm)
    for s in range(n_scenarios):
        k = CONTRACTS[names[s % len(names)]]()
        planted = Planted(arrays={"balance": {a: 10 ** 21 for a in ACTORS}})
        path = Path(corpus, planted, f"{k.name}#{s}")
        if k.ctor:
            k.ctor(path)
        actors_used: List[int] = []
        for _ in range(txs):
            fn = k.fns[int(rng.integers(0, len(k.fns)))]
            actor = ACTORS[int(rng.integers(0, len(ACTORS)))]
            actors_used.append(actor)
            value = int(rng.integers(1, 5)) * ETHER if fn.payable and rng.random() < 0.7 else 0
            saved = (list(path.cs), path.storage, path.balance)
            path.begin_tx(actor, value, _calldata(rng, fn, actors_used, k))
            args = _dispatch(path, k, fn)
            if args is not None and path.alive:
                fn.body(path, args)
            path.end_tx()
            if not path.alive:          # reverted: the next tx starts from the last open state
                path.cs, path.storage, path.balance = saved
    return corpus


def validate(corpus: Corpus) -> int:
    """Check every "sat" label against its planted model (engine interpretation of arrays
    and keccak); returns the number of SAT-labelled queries.  Raises on a wrong label."""
    n = 0
    for q in corpus.queries:
        if q.label != "sat":
            continue
        ev = _PlantedEval(q.planted, corpus.kfm.registry)
        bad = [c for c in q.constraints if not ev.ev(c)]
        if bad:
            raise AssertionError(f"{q.origin}: planted model violates {T.to_sexpr(bad[0])[:200]}")
        n += 1
    return n


# ---- queries that are UNSAT by construction (the soundness half of "% discharged") ------
def _symbol_terms(cs: List[T.Term]) -> List[T.Term]:
    seen, out, stack = set(), [], list(cs)
    while stack:
        t = stack.pop()
        if t in seen:
            continue
        seen.add(t)
        if t.op == "var":
            out.append(t)
        stack.extend(t.args)
    return sorted(out, key=lambda t: t.val)


def _reference_unsat_kats() -> List[Tuple[List[T.Term], str, UFRegistry]]:
    """The UNSAT labels of the reference's own SMT tests, rebuilt with the facade:
    tests/laser/keccak_tests.py (keccak equality of different values / widths, a symbol
    pinned to another value, keccak(keccak(a)*2) collisions with a != b, keccak == 10) and
    tests/laser/state/calldata_test.py (a read past calldatasize, equal indices with
    different bytes)."""
    from .smt import Array, If

    out = []

    def kat(name, build):
        kfm = KeccakFunctionManager(UFRegistry())
        cs = build(kfm)
        out.append(([c.raw if isinstance(c, Bool) else c for c in cs], f"kat:{name}", kfm.registry))

    def basic(i1, i2):
        def b(kfm):
            o1, o2 = kfm.create_keccak(i1), kfm.create_keccak(i2)
            return [kfm.create_conditions(), o1 == o2]
        return b

    kat("keccak_100_101", basic(BVV(100, 8), BVV(101, 8)))
    kat("keccak_w8_w16", basic(BVV(100, 8), BVV(100, 16)))
    kat("keccak_val8_sym256", basic(BVV(100, 8), BV("N1", 256)))

    def sym_and_val(kfm):
        n = BV("n", 256)
        o1, o2 = kfm.create_keccak(BVV(100, 256)), kfm.create_keccak(n)
        return [kfm.create_conditions(), o1 == o2, n == BVV(10, 256)]

    def complex_eq(kfm):
        a, b = BV("a", 160), BV("b", 160)
        o1 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(a))
        o2 = kfm.create_keccak(BVV(2, 256) * kfm.create_keccak(b))
        return [kfm.create_conditions(), o1 == o2, a != b]

    def simple_number(kfm):
        o = kfm.create_keccak(BV("a", 160))
        return [kfm.create_conditions(), BVV(10, 256) == o]

    def calldata_past_size(kfm):
        cd, size = Array("1_calldata", 256, 8), BV("1_calldatasize", 256)
        read = If(BVV(51, 256) < size, cd[BVV(51, 256)], BVV(0, 8))
        return [read == BVV(1, 8), size == BVV(50, 256)]

    def calldata_equal_indices(kfm):
        cd = Array("0_calldata", 256, 8)
        ia, ib = BV("index_a", 256), BV("index_b", 256)
        return [ia == ib, cd[ia] != cd[ib]]

    for name, fn in (("keccak_symbol_and_val", sym_and_val), ("keccak_complex_eq", complex_eq),
                     ("keccak_simple_number", simple_number), ("calldata_past_size", calldata_past_size),
                     ("calldata_equal_indices", calldata_equal_indices)):
        kat(name, fn)
    return out


def labelled_unsat(corpus: Corpus, n: int = 256, seed: int = 99) -> List[Tuple[List[T.Term], str, UFRegistry]]:
    """Queries whose label is UNSAT by construction: the reference's UNSAT KATs plus ``n``
    planted contradictions over the corpus' SAT queries — half add ``not c`` for one of the
    query's own conjuncts, half pin one of its symbols to two different values (its planted
    value and that value + 1, so the hint pass meets a near-miss).  A GPU "sat" on any of
    them would be a soundness bug."""
    rng = np.random.default_rng(seed)
    out = _reference_unsat_kats()
    sat_qs = [q for q in corpus.queries if q.label == "sat"]
    for i in range(n if sat_qs else 0):
        q = sat_qs[int(rng.integers(0, len(sat_qs)))]
        cs = list(q.constraints)
        syms = [v for v in _symbol_terms(cs) if v.val in q.planted.vars]
        if i % 2 == 0 or not syms:
            c = cs[int(rng.integers(0, len(cs)))]
            extra = [T.not_(c)]
            kind = "negated-conjunct"
        else:
            v = syms[int(rng.integers(0, len(syms)))]
            pv = q.planted.vars[v.val]
            extra = [T.eq(v, T.const(pv, v.width)), T.eq(v, T.const(pv + 1, v.width))]
            kind = "two-values"
        out.append((cs + extra, f"contra:{kind}:{q.origin}", corpus.kfm.registry))
    return out
