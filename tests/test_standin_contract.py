"""Pins of the Mythril behaviour the stand-in harness (tests/mythril_standin.py) must have, each
against the reference line it follows.  The harness is written from these contracts rather
than from Mythril's code; these tests are what makes it a faithful place to run the drop-in.
"""

import sys

import pytest

import fake_z3 as z3
import mythril_standin


@pytest.fixture
def ns(monkeypatch):
    return mythril_standin.install(monkeypatch, z3)


# ---- support_utils.py:15-34 (Singleton) ------------------------------------------------------
def test_singleton_one_instance_per_class(ns):
    class A(metaclass=ns.Singleton):
        def __init__(self, v=0):
            self.v = v

    class B(metaclass=ns.Singleton):
        pass

    a = A(1)
    assert A(2) is a and a.v == 1          # later arguments are ignored
    assert B() is B() and B() is not a


# ---- support_utils.py:35-55 (LRUCache) --------------------------------------------------------
def test_lru_get_put_order_and_eviction(ns):
    c = ns.LRUCache(3)
    assert c.get("x") == -1                      # a miss is -1 (:42-47)
    for k in "abc":
        c.put(k, k.upper())
    assert list(c.lru_cache) == ["a", "b", "c"]
    assert c.get("a") == "A"                     # a hit becomes the newest (:43-45)
    assert list(c.lru_cache) == ["b", "c", "a"]
    c.put("b", "B2")                             # an existing key: no eviction, newest (:50-51)
    assert list(c.lru_cache) == ["c", "a", "b"] and c.lru_cache["b"] == "B2"
    c.put("d", "D")                              # a new key at capacity evicts the oldest (:52-54)
    assert list(c.lru_cache) == ["a", "b", "d"]


# ---- support_utils.py:57-71 (ModelCache.check_quick_sat) ------------------------------------
class _CountingModel:
    """A model whose eval says True iff the constraint is in ``truths``; completion mutates it
    (like z3's), so the cache must hand eval a copy."""

    def __init__(self, name, truths):
        self.name, self.truths, self.completed, self.evals = name, set(truths), False, []

    def __deepcopy__(self, memo):
        twin = _CountingModel(self.name, self.truths)
        twin.evals = self.evals                  # shared log of evaluations
        return twin

    def eval(self, constraints, model_completion=False):
        assert model_completion is True          # (:63)
        self.completed = True
        self.evals.append(self.name)
        return z3.BoolVal(constraints in self.truths)


def test_quick_sat_newest_first_copy_and_bump(ns):
    mc = ns.ModelCache()
    log = []
    models = [_CountingModel(n, t) for n, t in (("old", {"q1", "q2"}), ("mid", {"q2"}), ("new", set()))]
    for m in models:
        m.evals = log
        mc.put(m, 1)
    assert mc.check_quick_sat("q2") is models[1]          # newest first: new, then mid (:61)
    assert log == ["new", "mid"]
    assert not any(m.completed for m in models)           # evaluated on deep copies (:62)
    assert mc.model_cache.lru_cache[models[1]] == 2       # hit bumped by get + 1 (:64)
    assert list(mc.model_cache.lru_cache)[-1] is models[1]
    assert mc.check_quick_sat("nothing") is False         # no model holds (:66)
    n = len(log)
    assert mc.check_quick_sat("q2") is models[1] and len(log) == n   # lru_cache memo (:59)


# ---- solver_statistics.py:7-25 (stat_smt_query) --------------------------------------------
def test_stat_smt_query_counts_once_when_enabled(ns):
    calls = []

    class S:
        @ns.stat_smt_query
        def check(self, *a):
            calls.append(a)
            return "sat"

    st = ns.SolverStatistics()
    assert st is ns.SolverStatistics()
    assert S().check() == "sat" and st.query_count == 0   # disabled: not counted (:13-14)
    st.enabled = True
    assert S().check(1) == "sat" and st.query_count == 1 and st.solver_time >= 0
    assert calls == [(), (1,)]
    s = ns.Solver()
    s.check()
    assert st.query_count == 2                           # BaseSolver.check is decorated (solver.py:72)


# ---- laser/smt/model.py:6-59 (Model) -----------------------------------------------------------
def test_model_eval_picks_the_declaring_model_or_the_last(ns):
    x, y = z3.BitVec("x", 8), z3.BitVec("y", 8)
    m1 = z3.ModelRef({x.decl(): 3})
    m2 = z3.ModelRef({y.decl(): 4})
    m = ns.Model([m1, m2])
    assert m.eval(x).as_long() == 3 and m.eval(y).as_long() == 4
    assert [d.name() for d in m.decls()] == ["x", "y"]
    assert m[x.decl()].as_long() == 3 and m[y.decl()].as_long() == 4
    assert ns.Model().eval(x) is None and ns.Model().raw == []


# ---- support/model.py:23-125 (get_model / solver_worker) -------------------------------------
def test_funnel_order_and_exceptions(ns, monkeypatch):
    funnel = ns.funnel
    made = []

    class FakeOptimize:
        def __init__(self):
            self.calls = []
            made.append(self)

        def set_timeout(self, t):
            self.calls.append(("timeout", t))

        def add(self, *cs):
            self.calls.append(("add", len(cs)))

        def minimize(self, e):
            self.calls.append(("min", e))

        def maximize(self, e):
            self.calls.append(("max", e))

        def check(self):
            self.calls.append(("check",))
            return z3.sat

        def model(self):
            return ("model", len(made))

    monkeypatch.setattr(funnel, "Optimize", FakeOptimize)   # resolved at call time (:37)
    B = ns.Bool
    c = (B(z3.BoolVal(True)), B(z3.Bool("p")))
    m = funnel.get_model(c, minimize=("o",), solver_timeout=7)
    assert made[0].calls == [("timeout", 7), ("add", 2), ("min", "o"), ("check",)]
    assert m == ("model", 1)
    assert list(funnel.model_cache.model_cache.lru_cache) == [("model", 1)]   # sat is cached (:120)
    assert funnel.get_model(c, minimize=("o",), solver_timeout=7) is m and len(made) == 1  # lru (:63)
    with pytest.raises(ns.SolverTimeOutException):
        funnel.get_model((B(z3.Bool("q")),), solver_timeout=-1)           # (:81-82)
    with pytest.raises(ns.UnsatError):
        funnel.get_model((False, B(z3.Bool("q"))), solver_timeout=5)      # (:83-85)

    class Boom(FakeOptimize):
        def check(self):
            raise RuntimeError("worker failure")

    monkeypatch.setattr(funnel, "Optimize", Boom)
    with pytest.raises(ns.SolverTimeOutException):                        # error -> unknown (:108-110)
        funnel.get_model((B(z3.Bool("r")),), minimize=("o",), solver_timeout=5)


def test_funnel_quick_sat_only_without_objectives(ns, monkeypatch):
    funnel = ns.funnel
    seen = []
    monkeypatch.setattr(funnel.model_cache, "check_quick_sat", lambda c: seen.append(c) or "cached")
    B = ns.Bool
    assert funnel.get_model((B(z3.Bool("a")),), solver_timeout=5) == "cached"   # (:95-98)
    assert len(seen) == 1
    with pytest.raises(ns.SolverTimeOutException):       # stand-in z3 answers unknown
        funnel.get_model((B(z3.Bool("a")),), maximize=("m",), solver_timeout=5)
    assert len(seen) == 1


# ---- constraints.py:31-46 (is_possible) ------------------------------------------------------
def test_is_possible_timeout_semantics(ns, monkeypatch):
    def raise_(exc):
        def f(*a, **k):
            raise exc
        return f

    monkeypatch.setattr(ns.funnel, "get_model", raise_(ns.SolverTimeOutException()))
    c = ns.Constraints([])
    assert c.is_possible() is False and c.is_possible(solver_timeout=100) is True
    monkeypatch.setattr(ns.funnel, "get_model", raise_(ns.UnsatError()))
    assert c.is_possible() is False and c.is_possible(solver_timeout=100) is False
    monkeypatch.setattr(ns.funnel, "get_model", lambda *a, **k: "m")
    assert c.is_possible() is True
    assert hash(ns.Constraints([1, 2])) == hash((1, 2))


# ---- the plugin construction sequence (plugin/loader.py:19-79, discovery.py:11-73,
# laser/plugin/loader.py:12-75, plugin/interface.py:6-46, laser/plugin/builder.py:6-21) -----
def test_plugin_construction_sequence(monkeypatch):
    events = []

    class Plugin:
        pass

    import types

    mod = types.ModuleType("standin_plugin_mod")
    monkeypatch.setitem(sys.modules, "standin_plugin_mod", mod)
    ns = mythril_standin.install(monkeypatch, z3, installed_plugins={"p": "standin_plugin_mod:Builder",
                                                                     "off": "standin_plugin_mod:Off"})

    class LP(ns.LaserPlugin):
        def __init__(self, **kw):
            events.append(("plugin", kw))

        def initialize(self, vm):
            events.append(("initialize", vm))

    class Builder(ns.MythrilLaserPlugin):
        name = "p"
        plugin_default_enabled = True

        def __init__(self, **kwargs):
            ns.MythrilLaserPlugin.__init__(self, **kwargs)
            assert not hasattr(self, "enabled")      # MythrilPlugin.__init__ shadows the builder's
            ns.PluginBuilder.__init__(self)
            events.append(("builder", kwargs))

        def __call__(self, *args, **kwargs):
            return LP(**kwargs)

    class Off(Builder):
        name = "off"
        plugin_default_enabled = False

    mod.Builder, mod.Off = Builder, Off
    loader = ns.MythrilPluginLoader()               # loads every default-enabled entry point
    assert events == [("builder", {})]
    assert [type(p) for p in loader.loaded_plugins] == [Builder]
    laser = ns.LaserPluginLoader()
    assert list(laser.laser_plugin_builders) == ["p"] and laser.is_enabled("p")
    laser.add_args("p", depth=3)
    laser.instrument_virtual_machine("vm", None)
    assert events[1:] == [("plugin", {"depth": 3}), ("initialize", "vm")]
    assert set(laser.plugin_list) == {"p"}
    with pytest.raises(ValueError):
        loader.load(object())
    assert ns.PluginDiscovery().get_plugins() == ["p", "off"]
    assert ns.PluginDiscovery().get_plugins(default_enabled=False) == ["off"]
