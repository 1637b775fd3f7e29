"""A test harness in the shape of the Mythril modules the engine's seams touch (Mythril itself
is not importable in this image: z3, eth_abi and eth_hash are missing — SURVEY.md §8c).

What the harness keeps from Mythril is the *interface contract* at each seam, not Mythril's
code: the module names the drop-in rebinds, the class bases it subclasses, the constructor
signatures, which names are resolved at call time and which are bound at import, the call
order of the query funnel, the LRU semantics of the model cache and the plugin construction
sequence.  Every piece below is written from that contract; the behaviour each one must have
is pinned by ``tests/test_standin_contract.py`` with the reference line it follows.

Seams (reference file:line of the contract):

* ``mythril.support.support_utils`` — a per-class singleton metaclass (support_utils.py:15-25),
  the size-100 LRU of cached models and ``ModelCache.check_quick_sat`` (:35-71: newest model
  first, evaluated on a private deep copy with ``model_completion=True``, the hit bumped,
  memoised by ``functools.lru_cache(2**10)``);
* ``mythril.laser.smt.solver.solver_statistics`` — ``stat_smt_query`` counts one query and its
  time while statistics are enabled (solver_statistics.py:7-25);
* ``mythril.laser.smt`` — ``BaseSolver``/``Solver``/``Optimize`` over the z3 objects, ``check``
  decorated, stdout silenced, a ``Z3Exception`` reported as ``unknown``
  (solver/solver.py:20-143); ``Model`` over a list of z3 models (model.py:6-59); the ``Bool``
  / ``BitVec`` wrappers and ``symbol_factory`` the call sites use;
* ``mythril.support.model`` — ``get_model`` / ``solver_worker`` (support/model.py:23-125):
  quick-sat first for objective-free queries, then a ``ThreadPool(1)`` worker that builds
  ``Optimize()`` through the module global, a timeout or any worker error is ``unknown``;
* ``Constraints.is_possible`` (constraints.py:31-46) and ``WorldState.constraints``;
* the ``Solver()`` call sites outside the funnel: the calldata slice loop
  (laser/ethereum/state/calldata.py:64-93, one query per byte) and the summary plugin's
  condition checks (plugins/summary/summary.py:114-117, summary/core.py:222-227) — each module
  binds ``Solver`` at import, which is what ``install()`` rebinds;
* the plugin stack: ``LaserPlugin``, ``PluginBuilder`` (laser/plugin/builder.py:6-21),
  ``MythrilPlugin`` / ``MythrilLaserPlugin`` (plugin/interface.py:6-46), ``LaserPluginLoader``
  (laser/plugin/loader.py:12-75), ``PluginDiscovery`` (plugin/discovery.py:11-73, the installed
  entry points injected) and ``MythrilPluginLoader`` (plugin/loader.py:19-79);
* the report's keccak concretisation step (analysis/solver.py:96-99 -> :129-165).

Test infrastructure only.
"""

from __future__ import annotations

import contextlib
import functools
import itertools
import os
import sys
import time
import types
from abc import ABC, abstractmethod
from collections import OrderedDict
from copy import deepcopy
from multiprocessing import TimeoutError as PoolTimeout
from multiprocessing.pool import ThreadPool

MODULES = (
    "mythril", "mythril.exceptions", "mythril.laser", "mythril.laser.smt",
    "mythril.laser.smt.model", "mythril.laser.smt.solver", "mythril.laser.smt.solver.solver",
    "mythril.laser.smt.solver.solver_statistics", "mythril.support", "mythril.support.model",
    "mythril.support.support_utils", "mythril.laser.ethereum",
    "mythril.laser.ethereum.function_managers", "mythril.laser.ethereum.state",
    "mythril.laser.ethereum.state.constraints", "mythril.laser.ethereum.state.calldata",
    "mythril.laser.plugin", "mythril.laser.plugin.builder", "mythril.laser.plugin.interface",
    "mythril.laser.plugin.loader", "mythril.laser.plugin.plugins",
    "mythril.laser.plugin.plugins.summary", "mythril.laser.plugin.plugins.summary.summary",
    "mythril.laser.plugin.plugins.summary.core", "mythril.plugin", "mythril.plugin.interface",
    "mythril.plugin.discovery", "mythril.plugin.loader", "mythril.analysis",
    "mythril.analysis.solver")


def host_sha3(value):
    """support_utils.sha3 (eth_hash) stand-in: the oracle's Keccak-256 (test infrastructure)."""
    import pyoracle

    return pyoracle.keccak256(bytes(value))


@contextlib.contextmanager
def _stdout_silenced():
    """The solver's stdout guard: libz3 may print while checking."""
    saved = sys.stdout
    with open(os.devnull, "w") as sink:
        sys.stdout = sink
        try:
            yield
        finally:
            sys.stdout = saved


# ---- singletons, statistics ----------------------------------------------------------------

def _singleton_meta():
    """A fresh per-class singleton metaclass: ``Cls()`` builds the instance once and hands
    the same object back ever after, whatever arguments later calls pass."""
    registry = {}

    class Singleton(type):
        _instances = registry

        def __call__(cls, *args, **kwargs):
            if cls not in registry:
                registry[cls] = type.__call__(cls, *args, **kwargs)
            return registry[cls]

    return Singleton


def _statistics(Singleton):
    class SolverStatistics(metaclass=Singleton):
        """Query count and solver time, recorded only while ``enabled`` (the analyzer turns
        it on, mythril_analyzer.py:147)."""

        def __init__(self):
            self.enabled = False
            self.query_count = 0
            self.solver_time = 0

        def __repr__(self):
            return f"Query count: {self.query_count} \nSolver time: {self.solver_time}"

    def stat_smt_query(check):
        @functools.wraps(check)
        def counted(*args, **kwargs):
            stats = SolverStatistics()
            if not stats.enabled:
                return check(*args, **kwargs)
            stats.query_count += 1
            started = time.time()
            answer = check(*args, **kwargs)
            stats.solver_time += time.time() - started
            return answer

        return counted

    return SolverStatistics, stat_smt_query


# ---- the smt facade --------------------------------------------------------------------------

def _facade(z3, stat_smt_query):
    def unwrap(x):
        return x.raw if hasattr(x, "raw") else x

    class Bool:
        def __init__(self, raw):
            self.raw = raw

        def simplify(self):
            self.raw = z3.simplify(self.raw)

        def __hash__(self):
            return hash(self.raw)

    class BitVec:
        def __init__(self, raw):
            self.raw = raw

        def simplify(self):
            self.raw = z3.simplify(self.raw)

        @property
        def symbolic(self):
            return not z3.is_bv_value(self.raw)

        @property
        def value(self):
            return self.raw.as_long() if z3.is_bv_value(self.raw) else None

        def size(self):
            return self.raw.size()

        def __add__(self, other):
            if isinstance(other, int):
                other = z3.BitVecVal(other, self.raw.size())
            return BitVec(self.raw + unwrap(other))

        def __eq__(self, other):  # noqa: D105 - a constraint, like z3's
            return Bool(self.raw == unwrap(other))

        def __ne__(self, other):
            return Bool(self.raw != unwrap(other))

        def __hash__(self):
            return hash(self.raw)

    class SymbolFactory:
        @staticmethod
        def BitVecVal(value, size, annotations=None):
            return BitVec(z3.BitVecVal(value, size))

        @staticmethod
        def BitVecSym(name, size, annotations=None):
            return BitVec(z3.BitVec(name, size))

    def And(*args):
        return Bool(z3.And([unwrap(a) for a in args]))

    def simplify(expression):
        expression.simplify()
        return expression

    class Model:
        """Several z3 models seen as one (``raw`` is the list)."""

        def __init__(self, models=None):
            self.raw = models or []

        def decls(self):
            return [d for internal in self.raw for d in internal.decls()]

        def __getitem__(self, item):
            last = len(self.raw) - 1
            for pos, internal in enumerate(self.raw):
                try:
                    found = internal[item]
                except IndexError:
                    if pos == last:
                        raise
                    continue
                if found is not None:
                    return found
            return None

        def eval(self, expression, model_completion=False):
            # the first model that declares the expression's head, else the last one
            head = expression.decl()
            last = len(self.raw) - 1
            for pos, internal in enumerate(self.raw):
                if pos == last or head in list(internal.decls()):
                    return internal.eval(expression, model_completion)
            return None

    class BaseSolver:
        def __init__(self, raw):
            self.raw = raw

        def set_timeout(self, timeout):
            self.raw.set(timeout=timeout)

        def set_unsat_core(self):
            self.raw.set(unsat_core=True)

        def add(self, *constraints):
            self.raw.add([unwrap(c) for c in constraints])

        def append(self, *constraints):
            return self.add(*constraints)   # through add, so an override sees appends too

        def assert_and_track(self, constraints, name):
            self.raw.assert_and_track(unwrap(constraints), name)

        @stat_smt_query
        def check(self, *args):
            with _stdout_silenced():
                try:
                    return self.raw.check(args)
                except z3.z3types.Z3Exception:
                    return z3.unknown

        def model(self):
            try:
                inner = self.raw.model()
            except z3.z3types.Z3Exception:
                return Model()
            return Model([inner])

        def sexpr(self):
            return self.raw.sexpr()

    class Solver(BaseSolver):
        def __init__(self):
            BaseSolver.__init__(self, z3.Solver())

        def reset(self):
            self.raw.reset()

        def pop(self, num):
            self.raw.pop(num)

    class Optimize(BaseSolver):
        def __init__(self):
            BaseSolver.__init__(self, z3.Optimize())

        def minimize(self, element):
            self.raw.minimize(unwrap(element))

        def maximize(self, element):
            self.raw.maximize(unwrap(element))

    return types.SimpleNamespace(Bool=Bool, BitVec=BitVec, symbol_factory=SymbolFactory(), And=And,
                                 simplify=simplify, Model=Model, BaseSolver=BaseSolver, Solver=Solver,
                                 Optimize=Optimize)


# ---- model cache ------------------------------------------------------------------------------

def _model_cache(z3):
    class LRUCache:
        """``get`` -> value (the key becomes the newest) or -1; ``put`` -> the key becomes the
        newest, the oldest key leaves when a new key would exceed ``size``."""

        def __init__(self, size):
            self.size = size
            self.lru_cache = OrderedDict()

        def get(self, key):
            if key not in self.lru_cache:
                return -1
            self.lru_cache.move_to_end(key)
            return self.lru_cache[key]

        def put(self, key, value):
            if key in self.lru_cache:
                self.lru_cache.move_to_end(key)
            elif len(self.lru_cache) >= self.size:
                self.lru_cache.popitem(last=False)
            self.lru_cache[key] = value

    class ModelCache:
        def __init__(self):
            self.model_cache = LRUCache(size=100)

        @functools.lru_cache(maxsize=2 ** 10)
        def check_quick_sat(self, constraints):
            newest_first = list(self.model_cache.lru_cache)[::-1]
            for model in newest_first:
                # completion adds interpretations to the model it runs on: a private copy
                if z3.is_true(deepcopy(model).eval(constraints, model_completion=True)):
                    self.model_cache.put(model, self.model_cache.get(model) + 1)
                    return model
            return False

        def put(self, key, value):
            self.model_cache.put(key, value)

    return LRUCache, ModelCache


# ---- the query funnel ---------------------------------------------------------------------------

def _funnel(z3, funnel, smt, UnsatError, SolverTimeOutException):
    def solver_worker(constraints, minimize=(), maximize=(), solver_timeout=None):
        solver = funnel.Optimize()   # the module global, read per call: what install() rebinds
        solver.set_timeout(solver_timeout)
        solver.add(*constraints)
        for kind, objectives in (("minimize", minimize), ("maximize", maximize)):
            for objective in objectives:
                getattr(solver, kind)(objective)
        return solver.check(), solver

    def run_worker(constraints, minimize, maximize, timeout):
        pool = ThreadPool(1)
        try:
            pending = pool.apply_async(solver_worker, args=(constraints, minimize, maximize, timeout))
            try:
                return pending.get(timeout)
            except PoolTimeout:
                return z3.unknown, None
            except Exception:  # noqa: BLE001 - any worker failure reads as unknown
                return z3.unknown, None
        finally:
            pool.terminate()

    @functools.lru_cache(maxsize=2 ** 23)
    def get_model(constraints, minimize=(), maximize=(), solver_timeout=None):
        timeout = solver_timeout or funnel.solver_timeout_default
        if timeout <= 0:
            raise SolverTimeOutException
        if any(isinstance(c, bool) and not c for c in constraints):
            raise UnsatError
        if not isinstance(constraints, tuple):
            constraints = constraints.get_all_constraints()
        smt_constraints = [c for c in constraints if not isinstance(c, bool)]
        if not minimize and not maximize:
            hit = funnel.model_cache.check_quick_sat(smt.simplify(smt.And(*smt_constraints)).raw)
            if hit:
                return hit
        verdict, solver = run_worker(smt_constraints, minimize, maximize, timeout)
        if verdict == z3.unknown:
            raise SolverTimeOutException
        if verdict != z3.sat:
            raise UnsatError
        # the cache receives one model() result and the caller another (two calls)
        funnel.model_cache.model_cache.put(solver.model(), 1)
        return solver.model()

    return solver_worker, get_model


def _state(funnel, kfm, UnsatError, SolverTimeOutException):
    class Constraints(list):
        def is_possible(self, solver_timeout=None):
            try:
                funnel.get_model(self, solver_timeout=solver_timeout)
            except UnsatError as e:
                # a timeout (an UnsatError subclass) under a short custom timeout is "maybe"
                return isinstance(e, SolverTimeOutException) and solver_timeout is not None
            return True

        def get_all_constraints(self):
            return list(self) + [kfm.create_conditions()]

        def __hash__(self):
            return hash(tuple(self))

    class WorldState:
        def __init__(self, constraints=None):
            self.constraints = Constraints(constraints or [])

    return Constraints, WorldState


# ---- Solver() call sites outside the funnel ---------------------------------------------------

def _calldata_module(mod, smt, z3):
    """The calldata slice loop: from ``start``, one ``Solver()`` query per index (timeout 1 s)
    asking whether the index can still differ from ``stop``; an ``unsat`` or ``unknown``
    verdict ends the slice.  ``Solver`` is this module's global (bound at import)."""
    mod.Solver = smt.Solver

    class Calldata:
        def __init__(self, tx_id, values):
            self.tx_id = tx_id
            self.values = list(values)   # concrete bytes; symbolic beyond them

        @property
        def size(self):
            return len(self.values)

        def _load(self, index):
            i = index.value if isinstance(index, smt.BitVec) else index
            if i is not None and i < len(self.values):
                return self.values[i]
            array = z3.Array(f"{self.tx_id}_calldata", z3.BitVecSort(256), z3.BitVecSort(8))
            return smt.BitVec(z3.Select(array, index.raw))

        def __getitem__(self, item):
            if not isinstance(item, slice):
                return self._load(item)
            first = 0 if item.start is None else item.start
            stride = 1 if item.step is None else item.step
            stop = self.size if item.stop is None else item.stop
            cursor = first if isinstance(first, smt.BitVec) else smt.symbol_factory.BitVecVal(first, 256)
            parts = []
            for _ in itertools.count():
                query = mod.Solver()
                query.set_timeout(1000)
                query.add(cursor != stop)
                if query.check() in (z3.unsat, z3.unknown):
                    return parts
                byte = self._load(cursor)
                parts.append(byte if isinstance(byte, smt.BitVec) else smt.symbol_factory.BitVecVal(byte, 8))
                cursor = smt.simplify(cursor + stride)

    mod.Calldata = Calldata


def _summary_modules(summary_mod, core_mod, smt, z3, kfm):
    """The summary plugin's two condition checks, each over its module's ``Solver``."""
    summary_mod.Solver = smt.Solver
    core_mod.Solver = smt.Solver

    def summary_applies(constraints, solver_timeout):
        # summary.py:114-117: the state's constraints after the summary's conditions
        query = summary_mod.Solver()
        query.set_timeout(solver_timeout)
        query.add(*constraints)
        return query.check() == z3.sat

    def keys_may_alias(state_key, key):
        # core.py:222-227: one storage key against another, with the keccak conditions
        query = core_mod.Solver()
        query.set_timeout(3000)
        query.add(state_key == key)
        query.add(kfm.create_conditions())
        return query.check() == z3.sat

    summary_mod.summary_applies = summary_applies
    core_mod.keys_may_alias = keys_may_alias


# ---- plugins ---------------------------------------------------------------------------------------

def _plugins(Singleton, installed_plugins):
    class LaserPlugin:
        def initialize(self, symbolic_vm):
            raise NotImplementedError

    class PluginBuilder(ABC):
        name = "Default Plugin Name"

        def __init__(self):
            self.enabled = True

        @abstractmethod
        def __call__(self, *args, **kwargs):
            ...

    class MythrilPlugin:
        author = "Default Author"
        name = "Plugin Name"
        plugin_license = "All rights reserved."
        plugin_type = "Mythril Plugin"
        plugin_version = "0.0.1 "
        plugin_description = "This is an example plugin description"

        def __init__(self, **kwargs):   # takes the plugin args, sets nothing (no `enabled`)
            pass

        def __repr__(self):
            return f"{type(self).__name__} - {self.plugin_version} - {self.author}"

    class MythrilCLIPlugin(MythrilPlugin):
        pass

    class MythrilLaserPlugin(MythrilPlugin, PluginBuilder, ABC):
        pass

    class LaserPluginLoader(metaclass=Singleton):
        def __init__(self):
            self.laser_plugin_builders = {}
            self.plugin_args = {}
            self.plugin_list = {}

        def add_args(self, plugin_name, **kwargs):
            self.plugin_args[plugin_name] = kwargs

        def load(self, plugin_builder):
            self.laser_plugin_builders.setdefault(plugin_builder.name, plugin_builder)

        def is_enabled(self, plugin_name):
            builder = self.laser_plugin_builders.get(plugin_name)
            return builder is not None and builder.enabled

        def enable(self, plugin_name):
            builder = self.laser_plugin_builders.get(plugin_name)
            if builder is None:
                return ValueError(f"Plugin with name: {plugin_name} was not loaded")
            builder.enabled = True

        def instrument_virtual_machine(self, symbolic_vm, with_plugins):
            for name, builder in self.laser_plugin_builders.items():
                wanted = name in with_plugins if with_plugins else builder.enabled
                if wanted:
                    plugin = builder(**self.plugin_args.get(name, {}))
                    plugin.initialize(symbolic_vm)
                    self.plugin_list[name] = plugin

    class PluginDiscovery(metaclass=Singleton):
        _installed_plugins = None

        def init_installed_plugins(self):
            from importlib.metadata import EntryPoint

            self._installed_plugins = {}
            for name, target in (installed_plugins or {}).items():
                self._installed_plugins[name] = EntryPoint(name, target, "mythril.plugins").load()

        @property
        def installed_plugins(self):
            if self._installed_plugins is None:
                self.init_installed_plugins()
            return self._installed_plugins

        def is_installed(self, plugin_name):
            return plugin_name in self.installed_plugins

        def build_plugin(self, plugin_name, plugin_args):
            if not self.is_installed(plugin_name):
                raise ValueError(f"Plugin with name: `{plugin_name}` is not installed")
            cls = self.installed_plugins.get(plugin_name)
            if cls is None or not issubclass(cls, MythrilPlugin):
                raise ValueError(f"No valid plugin was found for {plugin_name}")
            return cls(**plugin_args)

        def get_plugins(self, default_enabled=None):
            plugins = self.installed_plugins
            if default_enabled is None:
                return list(plugins)
            return [n for n, cls in plugins.items() if cls.plugin_default_enabled == default_enabled]

    class UnsupportedPluginType(Exception):
        pass

    class MythrilPluginLoader(metaclass=Singleton):
        def __init__(self):
            self.loaded_plugins = []
            self.plugin_args = {}
            self._load_default_enabled()

        def set_args(self, plugin_name, **kwargs):
            self.plugin_args[plugin_name] = kwargs

        def load(self, plugin):
            if not isinstance(plugin, MythrilPlugin):
                raise ValueError("Passed plugin is not of type MythrilPlugin")
            if not isinstance(plugin, MythrilLaserPlugin):
                raise UnsupportedPluginType("Passed plugin type is not yet supported")
            LaserPluginLoader().load(plugin)
            self.loaded_plugins.append(plugin)

        def _load_default_enabled(self):
            discovery = PluginDiscovery()
            for name in discovery.get_plugins(default_enabled=True):
                self.load(discovery.build_plugin(name, self.plugin_args.get(name, {})))

    return types.SimpleNamespace(
        LaserPlugin=LaserPlugin, PluginBuilder=PluginBuilder, MythrilPlugin=MythrilPlugin,
        MythrilCLIPlugin=MythrilCLIPlugin, MythrilLaserPlugin=MythrilLaserPlugin,
        LaserPluginLoader=LaserPluginLoader, PluginDiscovery=PluginDiscovery,
        UnsupportedPluginType=UnsupportedPluginType, MythrilPluginLoader=MythrilPluginLoader)


# ---- the report's keccak concretisation ---------------------------------------------------------

def _report_module(mod, mods):
    """Each 64-hex-digit window of a transaction's calldata (after the selector, or after the
    creation code when the input carries it) that contains the keccak manager's hash marker
    and is a concrete hash the model knows is replaced by the keccak of its preimage, the
    preimage read from the model through the width's inverse function."""

    def preimage_of(kfm, sf, known, model, digest):
        found = None
        for width, digests in known.items():   # the last width that knows it wins
            if digest in digests:
                _, inverse = kfm.store_function[width]
                raw = model.eval(inverse(sf.BitVecVal(digest, 256)).raw)
                found = sf.BitVecVal(raw.as_long(), width)
        return found

    def _replace_with_actual_sha(concrete_transactions, model, code=None):
        # the manager and factory are read through their modules at call time
        kfm = mods["mythril.laser.ethereum.function_managers"].keccak_function_manager
        sf = mods["mythril.laser.smt"].symbol_factory
        known = kfm.get_concrete_hash_data(model)
        for tx in concrete_transactions:
            original = tx["input"]
            if kfm.hash_matcher not in original:
                continue
            with_code = code is not None and code.bytecode in original
            head = len(code.bytecode) + 2 if with_code else 10
            for pos in range(head, len(original)):
                window = tx["input"][pos:pos + 64]
                if len(window) != 64 or kfm.hash_matcher not in window:
                    continue
                pre = preimage_of(kfm, sf, known, model, int(window, 16))
                if pre is None:
                    continue
                digest = "%064x" % kfm.find_concrete_keccak(pre).value
                current = tx["input"]
                tx["input"] = current[:head] + current[head:].replace(window, digest)

    def get_transaction_sequence_tail(concrete_transactions, model, code=None):
        """The concretisation step of get_transaction_sequence (analysis/solver.py:96-99),
        calling the step by its module-global name."""
        mod._replace_with_actual_sha(concrete_transactions, model, code)
        return concrete_transactions

    mod._replace_with_actual_sha = _replace_with_actual_sha
    mod.get_transaction_sequence_tail = get_transaction_sequence_tail


# ---- assembly -------------------------------------------------------------------------------------

def build(z3, installed_plugins=None):
    """Module objects keyed by their Mythril names, bound to the given z3 module.
    ``installed_plugins`` = {entry-point name: "module:attr"}, the ``"mythril.plugins"``
    entry points discovery loads — nothing is pip-installed here, so the test passes the value
    the package metadata declares (pyproject.toml)."""
    mods = {n: types.ModuleType(n) for n in MODULES}
    Singleton = _singleton_meta()

    class UnsatError(Exception):
        pass

    class SolverTimeOutException(UnsatError):
        pass

    SolverStatistics, stat_smt_query = _statistics(Singleton)
    smt = _facade(z3, stat_smt_query)
    LRUCache, ModelCache = _model_cache(z3)

    exc = mods["mythril.exceptions"]
    exc.UnsatError, exc.SolverTimeOutException = UnsatError, SolverTimeOutException
    stats_mod = mods["mythril.laser.smt.solver.solver_statistics"]
    stats_mod.stat_smt_query, stats_mod.SolverStatistics = stat_smt_query, SolverStatistics
    smt_mod = mods["mythril.laser.smt"]
    for name in ("Bool", "BitVec", "symbol_factory", "And", "simplify", "Optimize", "Solver",
                 "BaseSolver", "Model"):
        setattr(smt_mod, name, getattr(smt, name))
    smt_mod.SolverStatistics = SolverStatistics
    mods["mythril.laser.smt.model"].Model = smt.Model
    for name in ("mythril.laser.smt.solver", "mythril.laser.smt.solver.solver"):
        m = mods[name]
        m.BaseSolver, m.Solver, m.Optimize = smt.BaseSolver, smt.Solver, smt.Optimize
    mods["mythril.laser.smt.solver"].SolverStatistics = SolverStatistics

    kfm = types.SimpleNamespace(interval_hook_for_size={}, concrete_hashes={},
                                create_conditions=lambda: smt.Bool(z3.BoolVal(True)))
    mods["mythril.laser.ethereum.function_managers"].keccak_function_manager = kfm

    utils = mods["mythril.support.support_utils"]
    utils.Singleton, utils.LRUCache, utils.ModelCache, utils.sha3 = Singleton, LRUCache, ModelCache, host_sha3

    funnel = mods["mythril.support.model"]
    funnel.Optimize = smt.Optimize        # bound at import (support/model.py:13)
    funnel.model_cache = ModelCache()
    funnel.solver_timeout_default = 10000
    funnel.solver_worker, funnel.get_model = _funnel(z3, funnel, smt, UnsatError, SolverTimeOutException)

    Constraints, WorldState = _state(funnel, kfm, UnsatError, SolverTimeOutException)
    mods["mythril.laser.ethereum.state.constraints"].Constraints = Constraints
    mods["mythril.laser.ethereum.state"].WorldState = WorldState

    _calldata_module(mods["mythril.laser.ethereum.state.calldata"], smt, z3)
    _summary_modules(mods["mythril.laser.plugin.plugins.summary.summary"],
                     mods["mythril.laser.plugin.plugins.summary.core"], smt, z3, kfm)

    pl = _plugins(Singleton, installed_plugins)
    mods["mythril.laser.plugin.builder"].PluginBuilder = pl.PluginBuilder
    mods["mythril.laser.plugin.interface"].LaserPlugin = pl.LaserPlugin
    mods["mythril.laser.plugin.loader"].LaserPluginLoader = pl.LaserPluginLoader
    pi = mods["mythril.plugin.interface"]
    pi.MythrilPlugin, pi.MythrilCLIPlugin, pi.MythrilLaserPlugin = (pl.MythrilPlugin, pl.MythrilCLIPlugin,
                                                                    pl.MythrilLaserPlugin)
    mods["mythril.plugin.discovery"].PluginDiscovery = pl.PluginDiscovery
    mods["mythril.plugin.loader"].MythrilPluginLoader = pl.MythrilPluginLoader
    mods["mythril.plugin.loader"].UnsupportedPluginType = pl.UnsupportedPluginType

    _report_module(mods["mythril.analysis.solver"], mods)

    return mods, types.SimpleNamespace(
        Bool=smt.Bool, BitVec=smt.BitVec, symbol_factory=smt.symbol_factory, Model=smt.Model,
        Optimize=smt.Optimize, Solver=smt.Solver, Constraints=Constraints, WorldState=WorldState,
        LRUCache=LRUCache, ModelCache=ModelCache, UnsatError=UnsatError,
        SolverTimeOutException=SolverTimeOutException, SolverStatistics=SolverStatistics,
        stat_smt_query=stat_smt_query, LaserPlugin=pl.LaserPlugin, PluginBuilder=pl.PluginBuilder,
        MythrilPlugin=pl.MythrilPlugin, MythrilLaserPlugin=pl.MythrilLaserPlugin,
        LaserPluginLoader=pl.LaserPluginLoader, PluginDiscovery=pl.PluginDiscovery,
        MythrilPluginLoader=pl.MythrilPluginLoader, Singleton=Singleton, funnel=funnel, kfm=kfm,
        calldata=mods["mythril.laser.ethereum.state.calldata"],
        summary=mods["mythril.laser.plugin.plugins.summary.summary"],
        summary_core=mods["mythril.laser.plugin.plugins.summary.core"])


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
