"""Batched GPU feasibility for constraint sets given as terms.

``check_sets`` is the batched form of the reference's objective-free query path: every set
(one LASER state's ``Constraints.get_all_constraints()``) is lowered, all sets go to the GPU
in one ``pf_check_batch`` launch, and each witness is materialised into a model whose
``eval`` agrees bit for bit with the kernel.  Sets that cannot be lowered, or have no
witness among the candidates, return ``None`` — the caller then asks z3, unchanged.
"""

from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from .. import ir
from ..lower import LoweringError, lower
from .interp import Witness
from .model import WitnessModel
from . import terms as T
from .to_dag import DEFAULT_REGISTRY, TermLowering, UFRegistry


@dataclass
class GpuConfig:
    budget: int = 65536          # candidates per set
    seed: int = 0x4D595448       # global candidate seed
    flags: int = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT
    timeout_ms: int = 0
    enabled: bool = True


CONFIG = GpuConfig()


@dataclass
class GpuStats:
    sets: int = 0            # sets offered to the GPU
    lowered: int = 0         # sets that lowered to bytecode
    sat: int = 0             # sets discharged with a GPU witness
    lowering_failures: Dict[str, int] = field(default_factory=dict)
    kernel_ms: float = 0.0
    evals: int = 0


STATS = GpuStats()
_lock = threading.Lock()


def _set_seed(constraints: Sequence[T.Term]) -> int:
    h = 0
    for c in constraints:
        h = (h * 1000003) ^ (hash(T.to_sexpr(c)) & 0xFFFFFFFF)
    return h & 0xFFFFFFFF


def check_sets(sets: Sequence[Sequence[T.Term]], registry: Optional[UFRegistry] = None,
               parents: Optional[Sequence[Optional[dict]]] = None,
               config: Optional[GpuConfig] = None) -> List[Optional[WitnessModel]]:
    from ..engine import get_engine  # the GPU is required from here on: no host fallback

    cfg = config or CONFIG
    reg = registry or DEFAULT_REGISTRY
    out: List[Optional[WitnessModel]] = [None] * len(sets)
    progs, lows, idx = [], [], []
    for i, cs in enumerate(sets):
        cs = list(cs)
        if any(c is T.FALSE for c in cs):
            continue
        try:
            tl = TermLowering(reg, parents[i] if parents else None)
            lo = tl.lower(cs)
            prog = lower(lo.dag, seed=_set_seed(cs))
        except LoweringError as e:
            key = str(e).split(":")[0][:60]
            with _lock:
                STATS.lowering_failures[key] = STATS.lowering_failures.get(key, 0) + 1
            continue
        progs.append(prog)
        lows.append(lo)
        idx.append(i)
    with _lock:
        STATS.sets += len(sets)
        STATS.lowered += len(progs)
    if not progs:
        return out
    eng = get_engine()
    db = eng.upload(progs)
    res = eng.check(db, budget=cfg.budget, seed=cfg.seed, flags=cfg.flags, timeout_ms=cfg.timeout_ms)
    sat = [k for k in range(len(progs)) if res.found[k] != 0xFFFFFFFF]
    if sat:
        vals = eng.materialize(db, sat, [int(res.found[k]) for k in sat], seed=cfg.seed)
        for k, v in zip(sat, vals):
            i = idx[k]
            w = Witness(lows[k], v, reg)
            # re-check on the host under the same interpretation before handing it out
            if all(w.ev(c) for c in sets[i]):
                out[i] = WitnessModel(w, list(sets[i]))
    db.free()
    with _lock:
        STATS.sat += sum(1 for m in out if m is not None)
        STATS.kernel_ms += res.kernel_ms
        STATS.evals += res.cands_decided
    return out
