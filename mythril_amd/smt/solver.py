"""Solver / Optimize / SolverStatistics — mirror of mythril/laser/smt/solver/{solver,solver_statistics}.py.

``check()`` keeps the reference contract (solver.py:81-97): it never raises, returns
sat / unsat / unknown, and is counted by ``@stat_smt_query`` (solver_statistics.py:7-24).
The difference is where the answer comes from:

1. a constraint folded to ``False`` -> unsat;
2. no objectives -> the GPU search (mythril_amd.smt.gpu_check); a witness -> sat and the
   model is the witness;
3. otherwise (objectives present, set not lowerable, no witness) -> z3 unchanged when it is
   importable, else ``unknown`` (what the reference reports when z3 gives up).
"""

from __future__ import annotations

import logging
from time import time
from typing import Callable, List, Optional

from . import terms as T
from . import z3_bridge
from .expr import Bool, Expression
from .model import Model

log = logging.getLogger(__name__)


class CheckSatResult:
    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return self.name

    def __eq__(self, other):
        return getattr(other, "name", None) == self.name or (
            z3_bridge.HAVE_Z3 and repr(other) == self.name)

    def __hash__(self):
        return hash(self.name)


if z3_bridge.HAVE_Z3:  # pragma: no cover - z3 hosts return z3's own constants
    sat, unsat, unknown = z3_bridge.z3.sat, z3_bridge.z3.unsat, z3_bridge.z3.unknown
else:
    sat, unsat, unknown = CheckSatResult("sat"), CheckSatResult("unsat"), CheckSatResult("unknown")


class Singleton(type):
    _instances: dict = {}

    def __call__(cls, *args, **kwargs):
        if cls not in cls._instances:
            cls._instances[cls] = super().__call__(*args, **kwargs)
        return cls._instances[cls]


class SolverStatistics(metaclass=Singleton):
    """Query counting (solver_statistics.py:27-42) plus the GPU discharge counters."""

    def __init__(self):
        self.enabled = False
        self.query_count = 0
        self.solver_time = 0.0
        self.gpu_sat = 0          # queries answered sat by a GPU witness (the numerator)
        self.gpu_attempts = 0     # objective-free queries offered to the GPU
        self.z3_fallbacks = 0

    def __repr__(self):
        return (f"Query count: {self.query_count} \nSolver time: {self.solver_time}"
                f"\nGPU discharged: {self.gpu_sat}/{self.gpu_attempts}")


def stat_smt_query(func: Callable):
    stat_store = SolverStatistics()

    def function_wrapper(*args, **kwargs):
        if not stat_store.enabled:
            return func(*args, **kwargs)
        stat_store.query_count += 1
        begin = time()
        result = func(*args, **kwargs)
        stat_store.solver_time += time() - begin
        return result

    return function_wrapper


class BaseSolver:
    _optimize = False

    def __init__(self) -> None:
        self.constraints: List[T.Term] = []
        self.timeout: Optional[int] = None
        self._minimize: List[T.Term] = []
        self._maximize: List[T.Term] = []
        self._model: Model = Model()
        self._z3_solver = None

    @property
    def raw(self):
        return self

    def set_timeout(self, timeout: int) -> None:
        self.timeout = timeout

    def set_unsat_core(self) -> None:
        pass

    def add(self, *constraints: Bool) -> None:
        for c in constraints:
            if isinstance(c, (list, tuple)):
                self.add(*c)
            elif isinstance(c, Expression):
                self.constraints.append(c.raw)
            elif isinstance(c, bool):
                self.constraints.append(T.boolval(c))
            else:
                self.constraints.append(c)

    def assert_and_track(self, constraints: Bool, name: str) -> None:
        self.add(constraints)

    def append(self, *constraints: Bool) -> None:
        self.add(*constraints)

    @stat_smt_query
    def check(self, *args) -> object:
        stats = SolverStatistics()
        extra = [a.raw if isinstance(a, Expression) else a for a in args]
        cs = self.constraints + extra
        if any(c is T.FALSE for c in cs):
            return unsat
        if not self._minimize and not self._maximize:
            from . import gpu_check

            if gpu_check.CONFIG.enabled:
                stats.gpu_attempts += 1
                try:
                    m = gpu_check.check_sets([cs])[0]
                except Exception as e:  # the engine never answers on the host
                    log.info("GPU check failed: %s", e)
                    m = None
                if m is not None:
                    stats.gpu_sat += 1
                    self._model = Model([m])
                    return sat
        if z3_bridge.available():  # pragma: no cover - z3 hosts
            stats.z3_fallbacks += 1
            r, internal, s = z3_bridge.check(cs, self._minimize, self._maximize, self.timeout,
                                             optimize=self._optimize)
            self._z3_solver = s
            self._model = Model([internal]) if internal is not None else Model()
            return r
        return unknown

    def model(self) -> Model:
        return self._model

    def sexpr(self) -> str:
        lines = T.declarations(self.constraints + self._minimize + self._maximize)
        for c in self.constraints:
            lines.append(f"(assert {T.to_sexpr(c)})")
        for e in self._minimize:
            lines.append(f"(minimize {T.to_sexpr(e)})")
        for e in self._maximize:
            lines.append(f"(maximize {T.to_sexpr(e)})")
        return "\n".join(lines) + "\n(check-sat)\n"


class Solver(BaseSolver):
    def reset(self) -> None:
        self.constraints = []

    def pop(self, num: int) -> None:
        del self.constraints[len(self.constraints) - num:]


class Optimize(BaseSolver):
    _optimize = True

    def minimize(self, element: Expression) -> None:
        self._minimize.append(element.raw)

    def maximize(self, element: Expression) -> None:
        self._maximize.append(element.raw)
