"""Stand-ins for the Mythril modules the engine's seams touch (Mythril is not importable in
this image: z3, eth_abi and eth_hash are missing — SURVEY.md §8c).

Each piece restates the reference module it stands for LINE FOR LINE where the engine's code
meets it (class bases, ``__init__`` signatures, decorators, the loader's construction
sequence), so the drop-in ``Optimize``, the witness model and the plugin run inside exactly
the control flow a real analysis gives them.  A stand-in that simplifies the reference at a
seam hides the very bugs these tests exist to find (round-2 review: a ``check`` without
``@stat_smt_query``, a ``MythrilPlugin`` without ``__init__(**kwargs)``).

* ``mythril.support.support_utils`` — ``Singleton`` (support_utils.py:15-34), ``LRUCache``,
  ``ModelCache.check_quick_sat`` (:35-71: deep copy + ``eval(..., model_completion=True)``);
* ``mythril.laser.smt.solver.solver_statistics`` — ``stat_smt_query`` / ``SolverStatistics``
  (solver_statistics.py:7-42);
* ``mythril.laser.smt`` — ``BaseSolver``/``Solver``/``Optimize`` over ``z3.Optimize`` with the
  decorated ``check`` that silences stdout and maps a ``Z3Exception`` to ``unknown``
  (solver/solver.py:20-143), ``Model`` (model.py:6-59), ``Bool``, ``And``, ``simplify``;
* ``mythril.support.model`` — ``solver_worker`` / ``get_model`` (support/model.py:23-125),
  including the ``except Exception`` -> ``unknown`` around the worker's result;
* ``Constraints.is_possible`` (constraints.py:31-46), ``WorldState.constraints``
  (world_state.py:39), the keccak manager singleton;
* the plugin stack: ``LaserPlugin`` (laser/plugin/interface.py), ``PluginBuilder``
  (laser/plugin/builder.py:6-21), ``MythrilPlugin`` / ``MythrilLaserPlugin``
  (plugin/interface.py:6-46), ``LaserPluginLoader`` (laser/plugin/loader.py:12-75),
  ``PluginDiscovery`` (plugin/discovery.py:11-73; the installed entry points are injected,
  since nothing is pip-installed here) and ``MythrilPluginLoader`` (plugin/loader.py:19-79).

Test infrastructure only.
"""

from __future__ import annotations

import os
import sys
import types
from abc import ABC, abstractmethod
from collections import OrderedDict
from copy import deepcopy
from functools import lru_cache
from multiprocessing import TimeoutError
from multiprocessing.pool import ThreadPool
from time import time
from typing import Dict

MODULES = (
    "mythril", "mythril.exceptions", "mythril.laser", "mythril.laser.smt",
    "mythril.laser.smt.model", "mythril.laser.smt.solver", "mythril.laser.smt.solver.solver",
    "mythril.laser.smt.solver.solver_statistics", "mythril.support", "mythril.support.model",
    "mythril.support.support_utils", "mythril.laser.ethereum",
    "mythril.laser.ethereum.function_managers", "mythril.laser.ethereum.state",
    "mythril.laser.ethereum.state.constraints", "mythril.laser.plugin",
    "mythril.laser.plugin.builder", "mythril.laser.plugin.interface",
    "mythril.laser.plugin.loader", "mythril.plugin", "mythril.plugin.interface",
    "mythril.plugin.discovery", "mythril.plugin.loader", "mythril.analysis", "mythril.analysis.solver")


def host_sha3(value):
    """support_utils.sha3 (eth_hash) stand-in: the oracle's Keccak-256 (test infrastructure)."""
    import pyoracle

    return pyoracle.keccak256(bytes(value))


def build(z3, installed_plugins=None):
    """Module objects keyed by their Mythril names, bound to the given z3 module.
    ``installed_plugins`` = {entry-point name: "module:attr"}, the ``"mythril.plugins"``
    entry points ``PluginDiscovery`` loads (discovery.py:22-36) — nothing is pip-installed
    here, so the test passes the value the package metadata declares (pyproject.toml)."""
    mods = {n: types.ModuleType(n) for n in MODULES}

    # ---- support_utils.py:15-34 -----------------------------------------------------------
    class Singleton(type):
        _instances: Dict = {}

        def __call__(cls, *args, **kwargs):
            if cls not in cls._instances:
                cls._instances[cls] = super(Singleton, cls).__call__(*args, **kwargs)
            return cls._instances[cls]

    mods["mythril.support.support_utils"].Singleton = Singleton

    # ---- exceptions (mythril/exceptions.py:16-28) -------------------------------------
    class UnsatError(Exception):
        pass

    class SolverTimeOutException(UnsatError):
        pass

    mods["mythril.exceptions"].UnsatError = UnsatError
    mods["mythril.exceptions"].SolverTimeOutException = SolverTimeOutException

    # ---- solver_statistics.py:7-42 --------------------------------------------------------
    def stat_smt_query(func):
        stat_store = SolverStatistics()

        def function_wrapper(*args, **kwargs):
            if not stat_store.enabled:
                return func(*args, **kwargs)

            stat_store.query_count += 1
            begin = time()

            result = func(*args, **kwargs)

            end = time()
            stat_store.solver_time += end - begin

            return result

        return function_wrapper

    class SolverStatistics(object, metaclass=Singleton):
        def __init__(self):
            self.enabled = False
            self.query_count = 0
            self.solver_time = 0

        def __repr__(self):
            return "Query count: {} \nSolver time: {}".format(self.query_count, self.solver_time)

    stats_mod = mods["mythril.laser.smt.solver.solver_statistics"]
    stats_mod.stat_smt_query, stats_mod.SolverStatistics = stat_smt_query, SolverStatistics

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

    # ---- model.py:6-59 -----------------------------------------------------------------------
    class Model:
        def __init__(self, models=None):
            self.raw = models or []

        def decls(self):
            result = []
            for internal_model in self.raw:
                result.extend(internal_model.decls())
            return result

        def __getitem__(self, item):
            for internal_model in self.raw:
                is_last_model = self.raw.index(internal_model) == len(self.raw) - 1
                try:
                    result = internal_model[item]
                    if result is not None:
                        return result
                except IndexError:
                    if is_last_model:
                        raise
                    continue
            return None

        def eval(self, expression, model_completion=False):
            for internal_model in self.raw:
                is_last_model = self.raw.index(internal_model) == len(self.raw) - 1
                is_relevant_model = expression.decl() in list(internal_model.decls())
                if is_relevant_model or is_last_model:
                    return internal_model.eval(expression, model_completion)
            return None

    # ---- solver/solver.py:20-143 ------------------------------------------------------------
    class BaseSolver:
        def __init__(self, raw):
            self.raw = raw

        def set_timeout(self, timeout):
            self.raw.set(timeout=timeout)

        def set_unsat_core(self):
            self.raw.set(unsat_core=True)

        def add(self, *constraints):
            z3_constraints = [c.raw for c in constraints]
            self.raw.add(z3_constraints)

        def assert_and_track(self, constraints, name):
            self.raw.assert_and_track(constraints.raw, name)

        def append(self, *constraints):
            self.add(*constraints)

        @stat_smt_query
        def check(self, *args):
            old_stdout = sys.stdout
            with open(os.devnull, "w") as dev_null_fd:
                sys.stdout = dev_null_fd
                try:
                    evaluate = self.raw.check(args)
                except z3.z3types.Z3Exception:
                    evaluate = z3.unknown
            sys.stdout = old_stdout
            return evaluate

        def model(self):
            try:
                return Model([self.raw.model()])
            except z3.z3types.Z3Exception:
                return Model()

        def sexpr(self):
            return self.raw.sexpr()

    class Solver(BaseSolver):
        def __init__(self):
            super().__init__(z3.Solver())

        def reset(self):
            self.raw.reset()

        def pop(self, num):
            self.raw.pop(num)

    class Optimize(BaseSolver):
        def __init__(self):
            super().__init__(z3.Optimize())

        def minimize(self, element):
            self.raw.minimize(element.raw)

        def maximize(self, element):
            self.raw.maximize(element.raw)

    smt = mods["mythril.laser.smt"]
    smt.Bool, smt.And, smt.simplify, smt.Optimize, smt.Solver = Bool, And, simplify, Optimize, Solver
    smt.BaseSolver, smt.Model, smt.SolverStatistics = BaseSolver, Model, SolverStatistics
    mods["mythril.laser.smt.model"].Model = Model
    for name in ("mythril.laser.smt.solver", "mythril.laser.smt.solver.solver"):
        mods[name].BaseSolver, mods[name].Solver, mods[name].Optimize = BaseSolver, Solver, Optimize
    mods["mythril.laser.smt.solver"].SolverStatistics = SolverStatistics

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

    mods["mythril.support.support_utils"].LRUCache = LRUCache
    mods["mythril.support.support_utils"].ModelCache = ModelCache

    # ---- the funnel (support/model.py:23-125) ------------------------------------------
    funnel = mods["mythril.support.model"]
    funnel.Optimize = Optimize
    funnel.model_cache = ModelCache()
    funnel.solver_timeout_default = 10000

    def solver_worker(constraints, minimize=(), maximize=(), solver_timeout=None):
        s = funnel.Optimize()  # resolved at call time: the name install() rebinds
        s.set_timeout(solver_timeout)
        for constraint in constraints:
            s.add(constraint)
        for e in minimize:
            s.minimize(e)
        for e in maximize:
            s.maximize(e)
        result = s.check()
        return result, s

    @lru_cache(maxsize=2 ** 23)
    def get_model(constraints, minimize=(), maximize=(), solver_timeout=None):
        solver_timeout = solver_timeout or funnel.solver_timeout_default
        if solver_timeout <= 0:
            raise SolverTimeOutException
        for constraint in constraints:
            if isinstance(constraint, bool) and not constraint:
                raise UnsatError
        if isinstance(constraints, tuple) is False:
            constraints = constraints.get_all_constraints()
        constraints = [c for c in constraints if isinstance(c, bool) is False]
        if len(maximize) + len(minimize) == 0:
            ret_model = funnel.model_cache.check_quick_sat(simplify(And(*constraints)).raw)
            if ret_model:
                return ret_model
        pool = ThreadPool(1)
        try:
            thread_result = pool.apply_async(
                solver_worker, args=(constraints, minimize, maximize, solver_timeout))
            try:
                result, s = thread_result.get(solver_timeout)
            except TimeoutError:
                result = z3.unknown
            except Exception:
                result = z3.unknown
        finally:
            pool.terminate()
        if result == z3.sat:
            funnel.model_cache.model_cache.put(s.model(), 1)
            return s.model()
        elif result == z3.unknown:
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

    # ---- laser/plugin/interface.py ---------------------------------------------------------
    class LaserPlugin:
        def initialize(self, symbolic_vm):
            raise NotImplementedError

    # ---- laser/plugin/builder.py:6-21 -------------------------------------------------------
    class PluginBuilder(ABC):
        name = "Default Plugin Name"

        def __init__(self):
            self.enabled = True

        @abstractmethod
        def __call__(self, *args, **kwargs):
            pass

    # ---- plugin/interface.py:6-46 -----------------------------------------------------------
    class MythrilPlugin:
        author = "Default Author"
        name = "Plugin Name"
        plugin_license = "All rights reserved."
        plugin_type = "Mythril Plugin"
        plugin_version = "0.0.1 "
        plugin_description = "This is an example plugin description"

        def __init__(self, **kwargs):
            pass

        def __repr__(self):
            plugin_name = type(self).__name__
            return f"{plugin_name} - {self.plugin_version} - {self.author}"

    class MythrilCLIPlugin(MythrilPlugin):
        pass

    class MythrilLaserPlugin(MythrilPlugin, PluginBuilder, ABC):
        pass

    # ---- laser/plugin/loader.py:12-75 -------------------------------------------------------
    class LaserPluginLoader(object, metaclass=Singleton):
        def __init__(self):
            self.laser_plugin_builders = {}
            self.plugin_args = {}
            self.plugin_list = {}

        def add_args(self, plugin_name, **kwargs):
            self.plugin_args[plugin_name] = kwargs

        def load(self, plugin_builder):
            if plugin_builder.name in self.laser_plugin_builders:
                return
            self.laser_plugin_builders[plugin_builder.name] = plugin_builder

        def is_enabled(self, plugin_name):
            if plugin_name not in self.laser_plugin_builders:
                return False
            else:
                return self.laser_plugin_builders[plugin_name].enabled

        def enable(self, plugin_name):
            if plugin_name not in self.laser_plugin_builders:
                return ValueError(f"Plugin with name: {plugin_name} was not loaded")
            self.laser_plugin_builders[plugin_name].enabled = True

        def instrument_virtual_machine(self, symbolic_vm, with_plugins):
            for plugin_name, plugin_builder in self.laser_plugin_builders.items():
                enabled = (plugin_builder.enabled if not with_plugins
                           else plugin_name in with_plugins)

                if not enabled:
                    continue

                plugin = plugin_builder(**self.plugin_args.get(plugin_name, {}))
                plugin.initialize(symbolic_vm)
                self.plugin_list[plugin_name] = plugin

    # ---- plugin/discovery.py:11-73 (entry points injected) ---------------------------------
    class PluginDiscovery(object, metaclass=Singleton):
        _installed_plugins = None

        def init_installed_plugins(self):
            from importlib.metadata import EntryPoint

            self._installed_plugins = {
                name: EntryPoint(name, value, "mythril.plugins").load()
                for name, value in (installed_plugins or {}).items()}

        @property
        def installed_plugins(self):
            if self._installed_plugins is None:
                self.init_installed_plugins()
            return self._installed_plugins

        def is_installed(self, plugin_name):
            return plugin_name in self.installed_plugins.keys()

        def build_plugin(self, plugin_name, plugin_args):
            if not self.is_installed(plugin_name):
                raise ValueError(f"Plugin with name: `{plugin_name}` is not installed")

            plugin = self.installed_plugins.get(plugin_name)
            if plugin is None or not issubclass(plugin, MythrilPlugin):
                raise ValueError(f"No valid plugin was found for {plugin_name}")

            return plugin(**plugin_args)

        def get_plugins(self, default_enabled=None):
            if default_enabled is None:
                return list(self.installed_plugins.keys())

            return [plugin_name
                    for plugin_name, plugin_class in self.installed_plugins.items()
                    if plugin_class.plugin_default_enabled == default_enabled]

    # ---- plugin/loader.py:19-79 -------------------------------------------------------------
    class UnsupportedPluginType(Exception):
        pass

    class MythrilPluginLoader(object, metaclass=Singleton):
        def __init__(self):
            self.loaded_plugins = []
            self.plugin_args = dict()
            self._load_default_enabled()

        def set_args(self, plugin_name, **kwargs):
            self.plugin_args[plugin_name] = kwargs

        def load(self, plugin):
            if not isinstance(plugin, MythrilPlugin):
                raise ValueError("Passed plugin is not of type MythrilPlugin")
            if isinstance(plugin, MythrilLaserPlugin):
                self._load_laser_plugin(plugin)
            else:
                raise UnsupportedPluginType("Passed plugin type is not yet supported")

            self.loaded_plugins.append(plugin)

        @staticmethod
        def _load_laser_plugin(plugin):
            LaserPluginLoader().load(plugin)

        def _load_default_enabled(self):
            for plugin_name in PluginDiscovery().get_plugins(default_enabled=True):
                plugin = PluginDiscovery().build_plugin(
                    plugin_name, self.plugin_args.get(plugin_name, {}))
                self.load(plugin)

    # ---- analysis/solver.py:129-165 (_replace_with_actual_sha), resolving the keccak
    # manager and symbol_factory through their modules at call time like the reference's
    # module globals; get_transaction_sequence calls it by its module-global name ----------
    def _replace_with_actual_sha(concrete_transactions, model, code=None):
        keccak_function_manager = mods["mythril.laser.ethereum.function_managers"].keccak_function_manager
        symbol_factory = mods["mythril.laser.smt"].symbol_factory
        concrete_hashes = keccak_function_manager.get_concrete_hash_data(model)
        for tx in concrete_transactions:
            if keccak_function_manager.hash_matcher not in tx["input"]:
                continue
            if code is not None and code.bytecode in tx["input"]:
                s_index = len(code.bytecode) + 2
            else:
                s_index = 10
            for i in range(s_index, len(tx["input"])):
                data_slice = tx["input"][i: i + 64]
                if keccak_function_manager.hash_matcher not in data_slice or len(data_slice) != 64:
                    continue
                find_input = symbol_factory.BitVecVal(int(data_slice, 16), 256)
                input_ = None
                for size in concrete_hashes:
                    _, inverse = keccak_function_manager.store_function[size]
                    if find_input.value not in concrete_hashes[size]:
                        continue
                    input_ = symbol_factory.BitVecVal(model.eval(inverse(find_input).raw).as_long(), size)
                if input_ is None:
                    continue
                keccak = keccak_function_manager.find_concrete_keccak(input_)
                hex_keccak = hex(keccak.value)[2:]
                if len(hex_keccak) != 64:
                    hex_keccak = "0" * (64 - len(hex_keccak)) + hex_keccak
                tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(
                    tx["input"][i: 64 + i], hex_keccak)

    def get_transaction_sequence_tail(concrete_transactions, model, code=None):
        """The concretisation step of get_transaction_sequence (analysis/solver.py:96-99)."""
        mods["mythril.analysis.solver"]._replace_with_actual_sha(concrete_transactions, model, code)
        return concrete_transactions

    mods["mythril.analysis.solver"]._replace_with_actual_sha = _replace_with_actual_sha
    mods["mythril.analysis.solver"].get_transaction_sequence_tail = get_transaction_sequence_tail
    mods["mythril.support.support_utils"].sha3 = host_sha3

    mods["mythril.laser.plugin.builder"].PluginBuilder = PluginBuilder
    mods["mythril.laser.plugin.interface"].LaserPlugin = LaserPlugin
    mods["mythril.laser.plugin.loader"].LaserPluginLoader = LaserPluginLoader
    pi = mods["mythril.plugin.interface"]
    pi.MythrilPlugin, pi.MythrilCLIPlugin, pi.MythrilLaserPlugin = MythrilPlugin, MythrilCLIPlugin, MythrilLaserPlugin
    mods["mythril.plugin.discovery"].PluginDiscovery = PluginDiscovery
    mods["mythril.plugin.loader"].MythrilPluginLoader = MythrilPluginLoader
    mods["mythril.plugin.loader"].UnsupportedPluginType = UnsupportedPluginType
    return mods, types.SimpleNamespace(
        Bool=Bool, Model=Model, Optimize=Optimize, Solver=Solver, Constraints=Constraints,
        WorldState=WorldState, ModelCache=ModelCache, UnsatError=UnsatError,
        SolverTimeOutException=SolverTimeOutException, SolverStatistics=SolverStatistics,
        LaserPlugin=LaserPlugin, PluginBuilder=PluginBuilder, MythrilPlugin=MythrilPlugin,
        MythrilLaserPlugin=MythrilLaserPlugin, LaserPluginLoader=LaserPluginLoader,
        PluginDiscovery=PluginDiscovery, MythrilPluginLoader=MythrilPluginLoader,
        Singleton=Singleton, funnel=funnel, kfm=kfm)


def install(monkeypatch, z3, installed_plugins=None):
    """Register the stand-ins (and z3) in sys.modules for one test."""
    mods, ns = build(z3, installed_plugins)
    # integration.install() sets process defaults (PF_TORCH, PF_DEVICES): undo them with the test
    for var in ("PF_TORCH", "PF_DEVICES", "LOCAL_RANK"):
        if var in os.environ:
            monkeypatch.setenv(var, os.environ[var])
        else:
            monkeypatch.setenv(var, "")
            monkeypatch.delenv(var)
    monkeypatch.setitem(sys.modules, "z3", z3)
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    return ns
