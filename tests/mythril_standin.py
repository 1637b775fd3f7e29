"""Stand-ins for the Mythril modules the engine's seams touch (Mythril is not importable in
this image: z3, eth_abi and eth_hash are missing — SURVEY.md §8c).

Each piece restates the behaviour of the reference module it stands for, so the drop-in
``Optimize``, the witness model and the tx-boundary hook run inside the same control flow a
real analysis would give them:

* ``mythril.laser.smt`` — ``BaseSolver``/``Optimize`` over ``z3.Optimize`` (raw assertions,
  ``set_timeout`` -> ``raw.set(timeout=)``, ``model()`` -> ``Model([raw.model()])`` or an
  empty ``Model()`` on a z3 exception; mythril/laser/smt/solver/solver.py:20-143), ``Bool``,
  ``And``, ``simplify``;
* ``mythril.laser.smt.model.Model`` — the relevance rule of ``eval``: the first internal
  model whose ``decls()`` contains ``expression.decl()``, else the last one
  (mythril/laser/smt/model.py:45-59);
* ``mythril.support.support_utils.ModelCache`` — ``check_quick_sat`` deep-copies every
  cached model and evaluates the query with ``model_completion=True``
  (support_utils.py:57-71);
* ``mythril.support.model.get_model`` — the funnel: bools, quick-sat, ``solver_worker`` on a
  ``ThreadPool(1)``, sat -> ``model_cache.put(s.model(), 1)``, unknown ->
  ``SolverTimeOutException``, unsat -> ``UnsatError`` (support/model.py:23-125);
* ``Constraints.is_possible`` (constraints.py:31-46), ``WorldState.constraints``
  (world_state.py:39), the keccak manager singleton, the plugin interfaces.

Test infrastructure only.
"""

from __future__ import annotations

import sys
import types
from collections import OrderedDict
from copy import deepcopy
from functools import lru_cache
from multiprocessing import TimeoutError
from multiprocessing.pool import ThreadPool


def build(z3):
    """Module objects keyed by their Mythril names, bound to the given z3 module."""
    mods = {n: types.ModuleType(n) for n in (
        "mythril", "mythril.exceptions", "mythril.laser", "mythril.laser.smt",
        "mythril.laser.smt.model", "mythril.support", "mythril.support.model",
        "mythril.support.support_utils", "mythril.laser.ethereum",
        "mythril.laser.ethereum.function_managers", "mythril.laser.ethereum.state",
        "mythril.laser.ethereum.state.constraints", "mythril.laser.plugin",
        "mythril.laser.plugin.builder", "mythril.laser.plugin.interface", "mythril.plugin",
        "mythril.plugin.interface")}

    # ---- exceptions (mythril/exceptions.py:16-28) -------------------------------------
    class UnsatError(Exception):
        pass

    class SolverTimeOutException(UnsatError):
        pass

    mods["mythril.exceptions"].UnsatError = UnsatError
    mods["mythril.exceptions"].SolverTimeOutException = SolverTimeOutException

    # ---- facade ------------------------------------------------------------------------
    class Bool:
        def __init__(self, raw):
            self.raw = raw

        def simplify(self):
            self.raw = z3.simplify(self.raw)

        def __hash__(self):
            return hash(self.raw)

    def And(*args):
        return Bool(z3.And([a.raw for a in args]))

    def simplify(expression):
        expression.simplify()
        return expression

    class Model:
        def __init__(self, models=None):
            self.raw = models or []

        def decls(self):
            out = []
            for m in self.raw:
                out.extend(m.decls())
            return out

        def __getitem__(self, item):
            for i, m in enumerate(self.raw):
                try:
                    r = m[item]
                    if r is not None:
                        return r
                except IndexError:
                    if i == len(self.raw) - 1:
                        raise
            return None

        def eval(self, expression, model_completion=False):
            for i, m in enumerate(self.raw):
                is_last = i == len(self.raw) - 1
                relevant = expression.decl() in list(m.decls())
                if relevant or is_last:
                    return m.eval(expression, model_completion)
            return None

    class BaseSolver:
        def __init__(self, raw):
            self.raw = raw

        def set_timeout(self, timeout):
            self.raw.set(timeout=timeout)

        def add(self, *constraints):
            self.raw.add([c.raw for c in constraints])

        def append(self, *constraints):
            self.add(*constraints)

        def check(self, *args):
            try:
                return self.raw.check(args)
            except z3.z3types.Z3Exception:
                return z3.unknown

        def model(self):
            try:
                return Model([self.raw.model()])
            except z3.z3types.Z3Exception:
                return Model()

        def sexpr(self):
            return self.raw.sexpr()

    class Optimize(BaseSolver):
        def __init__(self):
            super().__init__(z3.Optimize())

        def minimize(self, element):
            self.raw.minimize(element.raw)

        def maximize(self, element):
            self.raw.maximize(element.raw)

    smt = mods["mythril.laser.smt"]
    smt.Bool, smt.And, smt.simplify, smt.Optimize, smt.BaseSolver = Bool, And, simplify, Optimize, BaseSolver
    smt.Model = Model
    mods["mythril.laser.smt.model"].Model = Model

    # ---- keccak manager singleton -----------------------------------------------------
    kfm = types.SimpleNamespace(interval_hook_for_size={}, concrete_hashes={},
                                create_conditions=lambda: Bool(z3.BoolVal(True)))
    mods["mythril.laser.ethereum.function_managers"].keccak_function_manager = kfm

    # ---- ModelCache (support_utils.py:35-71) -------------------------------------------
    class LRUCache:
        def __init__(self, size):
            self.size = size
            self.lru_cache = OrderedDict()

        def get(self, key):
            try:
                value = self.lru_cache.pop(key)
                self.lru_cache[key] = value
                return value
            except KeyError:
                return -1

        def put(self, key, value):
            try:
                self.lru_cache.pop(key)
            except KeyError:
                if len(self.lru_cache) >= self.size:
                    self.lru_cache.popitem(last=False)
            self.lru_cache[key] = value

    class ModelCache:
        def __init__(self):
            self.model_cache = LRUCache(size=100)

        @lru_cache(maxsize=2 ** 10)
        def check_quick_sat(self, constraints):
            for model in reversed(self.model_cache.lru_cache.keys()):
                model_copy = deepcopy(model)
                if z3.is_true(model_copy.eval(constraints, model_completion=True)):
                    self.model_cache.put(model, self.model_cache.get(model) + 1)
                    return model
            return False

        def put(self, key, value):
            self.model_cache.put(key, value)

    mods["mythril.support.support_utils"].ModelCache = ModelCache

    # ---- the funnel (support/model.py:23-125) ------------------------------------------
    funnel = mods["mythril.support.model"]
    funnel.Optimize = Optimize
    funnel.model_cache = ModelCache()
    funnel.solver_timeout_default = 10000

    def solver_worker(constraints, minimize=(), maximize=(), solver_timeout=None):
        s = funnel.Optimize()  # resolved at call time: the name install() rebinds
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
        solver_timeout = solver_timeout or funnel.solver_timeout_default
        if solver_timeout <= 0:
            raise SolverTimeOutException
        for c in constraints:
            if isinstance(c, bool) and not c:
                raise UnsatError
        if isinstance(constraints, tuple) is False:
            constraints = constraints.get_all_constraints()
        constraints = [c for c in constraints if isinstance(c, bool) is False]
        if len(maximize) + len(minimize) == 0:
            ret = funnel.model_cache.check_quick_sat(simplify(And(*constraints)).raw)
            if ret:
                return ret
        pool = ThreadPool(1)
        try:
            res = pool.apply_async(solver_worker, args=(constraints, minimize, maximize, solver_timeout))
            try:
                result, s = res.get(solver_timeout)
            except TimeoutError:
                result = z3.unknown
        finally:
            pool.terminate()
        if result == z3.sat:
            funnel.model_cache.model_cache.put(s.model(), 1)
            return s.model()
        if result == z3.unknown:
            raise SolverTimeOutException
        raise UnsatError

    funnel.solver_worker, funnel.get_model = solver_worker, get_model

    # ---- Constraints / WorldState --------------------------------------------------------
    class Constraints(list):
        def is_possible(self, solver_timeout=None):
            try:
                funnel.get_model(self, solver_timeout=solver_timeout)
            except SolverTimeOutException:
                return solver_timeout is not None
            except UnsatError:
                return False
            return True

        def get_all_constraints(self):
            return self[:] + [kfm.create_conditions()]

        def __hash__(self):
            return tuple(self[:]).__hash__()

    class WorldState:
        def __init__(self, constraints=None):
            self.constraints = Constraints(constraints or [])

    mods["mythril.laser.ethereum.state.constraints"].Constraints = Constraints
    mods["mythril.laser.ethereum.state"].WorldState = WorldState

    # ---- plugin interfaces (laser/plugin/interface.py, builder.py; plugin/interface.py) --
    class LaserPlugin:
        def initialize(self, symbolic_vm):
            raise NotImplementedError

    class PluginBuilder:
        name = "default"

        def __init__(self):
            self.enabled = True

    class MythrilPlugin:
        author = "Default Author"
        name = "Plugin Name"
        plugin_description = "This is an example plugin description"

    class MythrilLaserPlugin(MythrilPlugin):
        def __call__(self, *args, **kwargs):
            raise NotImplementedError

    mods["mythril.laser.plugin.builder"].PluginBuilder = PluginBuilder
    mods["mythril.laser.plugin.interface"].LaserPlugin = LaserPlugin
    mods["mythril.plugin.interface"].MythrilLaserPlugin = MythrilLaserPlugin
    return mods, types.SimpleNamespace(
        Bool=Bool, Model=Model, Optimize=Optimize, Constraints=Constraints, WorldState=WorldState,
        ModelCache=ModelCache, UnsatError=UnsatError, SolverTimeOutException=SolverTimeOutException,
        LaserPlugin=LaserPlugin, PluginBuilder=PluginBuilder, MythrilLaserPlugin=MythrilLaserPlugin,
        funnel=funnel, kfm=kfm)


def install(monkeypatch, z3):
    """Register the stand-ins (and z3) in sys.modules for one test."""
    mods, ns = build(z3)
    monkeypatch.setitem(sys.modules, "z3", z3)
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    return ns
