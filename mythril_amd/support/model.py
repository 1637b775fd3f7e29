"""Query funnel — mirror of mythril/support/model.py:23-125 (``get_model``), plus its
batched form ``get_models`` used at the transaction boundary.

Semantics kept from the reference:
* ``lru_cache`` on (constraints, minimize, maximize, solver_timeout) (:63);
* timeout clamp against the global budget, <= 0 -> SolverTimeOutException (:79-82);
* a literal ``False`` -> UnsatError (:83-85); python bools dropped (:87-93);
* no objectives -> fast path first (reference: ``ModelCache.check_quick_sat``, :95-98; here:
  the GPU batched search, which evaluates 65,536 generated candidates instead of <= 100
  cached models); sat -> model, unknown -> SolverTimeOutException, unsat -> UnsatError
  (:119-125).
"""

from __future__ import annotations

import logging
from functools import lru_cache
from typing import List, Optional, Sequence

from ..exceptions import SolverTimeOutException, UnsatError
from ..smt import Bool, Model, Optimize, sat, unknown
from ..smt import terms as T
from ..smt.gpu_check import check_sets
from ..smt.model import Model as _Model
from ..smt.solver import SolverStatistics

log = logging.getLogger(__name__)

DEFAULT_SOLVER_TIMEOUT_MS = 10000   # support_args.py:6-31 default solver_timeout


def _raw_list(constraints) -> List[T.Term]:
    if hasattr(constraints, "get_all_constraints"):
        constraints = constraints.get_all_constraints()
    out = []
    for c in constraints:
        if isinstance(c, bool):
            if not c:
                raise UnsatError
            continue
        out.append(c.raw if isinstance(c, Bool) else c)
    return out


def solver_worker(constraints, minimize=(), maximize=(), solver_timeout=None):
    s = Optimize()
    s.set_timeout(solver_timeout)
    for c in constraints:
        s.add(c)
    for e in minimize:
        s.minimize(e)
    for e in maximize:
        s.maximize(e)
    return s.check(), s


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), solver_timeout=None):
    solver_timeout = solver_timeout or DEFAULT_SOLVER_TIMEOUT_MS
    if solver_timeout <= 0:
        raise SolverTimeOutException
    for c in constraints:
        if isinstance(c, bool) and not c:
            raise UnsatError
    cs = [c for c in constraints if not isinstance(c, bool)]
    result, s = solver_worker(cs, minimize, maximize, solver_timeout)
    if result == sat:
        return s.model()
    if result == unknown:
        log.debug("no witness and no z3 verdict")
        raise SolverTimeOutException
    raise UnsatError


def get_models(constraint_sets: Sequence, parents: Optional[Sequence[Optional[dict]]] = None,
               registry=None) -> List[Optional[Model]]:
    """Objective-free feasibility of many sets in ONE GPU batch (tx-boundary pruning,
    svm.py:279-283).  ``None`` = no GPU witness (ask z3 / treat as the reference would).
    ``registry``: the keccak interpretation (defaults to the global keccak manager's)."""
    raws = []
    for cs in constraint_sets:
        try:
            raws.append(_raw_list(cs))
        except UnsatError:
            raws.append([T.FALSE])
    stats = SolverStatistics()
    stats.gpu_attempts += len(raws)
    internals = check_sets(raws, registry=registry, parents=parents)
    out = []
    for m in internals:
        if m is None:
            out.append(None)
        else:
            stats.gpu_sat += 1
            out.append(_Model([m]))
    return out
