"""Seam #2: the LASER plugin and the tx-boundary batch
(mythril_amd/integration.py).

Mythril itself is not importable here (z3, eth_abi, eth_hash missing — SURVEY §8c), so the
plugin classes are exercised against minimal stand-ins of the three Mythril interfaces they
subclass (mythril/laser/plugin/interface.py, mythril/laser/plugin/builder.py,
mythril/plugin/interface.py:40-46) and a stand-in symbolic VM exposing ``laser_hook`` and
``open_states`` (svm.py:133-145, 726-741).  The batch itself runs on the GPU over states
whose constraints are mythril_amd.smt terms (the drop-in facade); with z3 present the same
function reads z3 ASTs through SMT-LIB2.
"""

import sys
import types

import pytest

from mythril_amd import integration
from mythril_amd.smt import ULT, symbol_factory
from mythril_amd.smt.to_dag import UFRegistry


@pytest.fixture
def stub_mythril(monkeypatch):
    """Register stand-ins for the Mythril plugin interfaces in sys.modules."""

    class LaserPlugin:  # mythril/laser/plugin/interface.py
        def initialize(self, symbolic_vm):
            raise NotImplementedError

    class PluginBuilder:  # mythril/laser/plugin/builder.py
        name = "default"

        def __init__(self):
            self.enabled = True

    class MythrilPlugin:  # mythril/plugin/interface.py
        author = "Default Author"
        name = "Plugin Name"
        plugin_license = "All rights reserved."
        plugin_type = "Mythril Plugin"
        plugin_version = "0.0.1 "
        plugin_description = "This is an example plugin description"

    class MythrilLaserPlugin(MythrilPlugin):  # mythril/plugin/interface.py:40-46
        def __call__(self, *args, **kwargs):
            raise NotImplementedError

    mods = {
        "mythril": types.ModuleType("mythril"),
        "mythril.laser": types.ModuleType("mythril.laser"),
        "mythril.laser.plugin": types.ModuleType("mythril.laser.plugin"),
        "mythril.laser.plugin.builder": types.ModuleType("mythril.laser.plugin.builder"),
        "mythril.laser.plugin.interface": types.ModuleType("mythril.laser.plugin.interface"),
        "mythril.plugin": types.ModuleType("mythril.plugin"),
        "mythril.plugin.interface": types.ModuleType("mythril.plugin.interface"),
    }
    mods["mythril.laser.plugin.builder"].PluginBuilder = PluginBuilder
    mods["mythril.laser.plugin.interface"].LaserPlugin = LaserPlugin
    mods["mythril.plugin.interface"].MythrilLaserPlugin = MythrilLaserPlugin
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    return types.SimpleNamespace(LaserPlugin=LaserPlugin, PluginBuilder=PluginBuilder,
                                 MythrilLaserPlugin=MythrilLaserPlugin)


class FakeSVM:
    """The part of LaserEVM the plugin touches: laser_hook registration, open_states."""

    def __init__(self, open_states=()):
        self.hooks = {}
        self.open_states = list(open_states)

    def laser_hook(self, name):
        def deco(fn):
            self.hooks.setdefault(name, []).append(fn)
            return fn
        return deco


def test_plugin_builder_contract(stub_mythril):
    """discovery.py:71 reads plugin_default_enabled; SymExecWrapper calls the builder and
    initialize(symbolic_vm) (analysis/symbolic.py:169, laser/plugin/loader.py:55-75)."""
    laser_cls, builder_cls = integration._plugin_classes()
    assert issubclass(builder_cls, stub_mythril.MythrilLaserPlugin)
    assert issubclass(builder_cls, stub_mythril.PluginBuilder)
    assert builder_cls.plugin_default_enabled is True
    assert builder_cls.name == "mythril-amd-path-feasibility"
    plugin = builder_cls()()
    assert isinstance(plugin, stub_mythril.LaserPlugin)


def test_plugin_initialize_registers_tx_boundary_hook(stub_mythril, monkeypatch):
    """initialize() rebinds the funnel's Optimize once and registers a stop_sym_trans hook
    that batches every open state (svm.py:307-308 runs it right before the next
    iteration's is_possible() pass, svm.py:279-283)."""
    calls = {"install": 0, "batch": []}
    monkeypatch.setattr(integration, "install", lambda: calls.__setitem__("install", calls["install"] + 1))
    monkeypatch.setattr(integration, "batch_open_states",
                        lambda states: calls["batch"].append(list(states)) or len(states))
    _, builder_cls = integration._plugin_classes()
    svm = FakeSVM(open_states=["s0", "s1", "s2"])
    builder_cls()().initialize(svm)
    assert calls["install"] == 1
    assert list(svm.hooks) == ["stop_sym_trans"]
    svm.hooks["stop_sym_trans"][0]()
    assert calls["batch"] == [["s0", "s1", "s2"]]


class _BV:
    def __init__(self, value, size):
        self.value, self._size = value, size

    def size(self):
        return self._size


def test_sync_keccak_registry_mirrors_manager():
    """Intervals (keccak_function_manager.py:158-163: index * PART) and concrete hashes
    (:57-69) are mirrored into the lowering's UF registry."""
    kfm = types.SimpleNamespace(interval_hook_for_size={512: 0, 256: 1},
                                concrete_hashes={_BV(7, 256): _BV(0xABC, 256)})
    reg = UFRegistry()
    integration.sync_keccak_registry(kfm, reg)
    assert reg.keccak[512].lo == 0
    assert reg.keccak[256].lo == integration.PART
    assert reg.keccak[256].concrete == {7: 0xABC}


class _Constraints(list):
    """constraints.py:132-133: get_all_constraints() = the list + the keccak conditions."""

    def get_all_constraints(self):
        return list(self)


class _WorldState:
    """svm.py:85,380: open_states holds WorldStates, which carry .constraints directly
    (world_state.py:39) — there is no .world_state attribute on them."""

    def __init__(self, constraints):
        self.constraints = _Constraints(constraints)


def _state(constraints):
    return _WorldState(constraints)


def test_state_terms_uses_facade_terms_directly():
    x = symbol_factory.BitVecSym("x", 256)
    c = ULT(x, symbol_factory.BitVecVal(10, 256))
    terms = integration.state_terms(_state([c, True]))
    assert terms == [c.raw]
    assert not hasattr(_state([c]), "world_state")


@pytest.mark.gpu
def test_batch_open_states_discharges_sat_states(engine):
    """Three open states at a tx boundary in one launch: two satisfiable, one contradictory;
    the witnesses are parked for the is_possible() pass and evaluate their sets to true."""
    integration._BATCH_CACHE.clear()
    cv = symbol_factory.BitVecSym("call_value1", 256)
    size = symbol_factory.BitVecSym("1_calldatasize", 256)
    v = symbol_factory.BitVecVal
    sat_a = [ULT(cv, v(1000, 256)), cv != v(0, 256)]
    sat_b = [ULT(v(3, 256), size), ULT(size, v(68, 256))]
    unsat = [ULT(cv, v(5, 256)), ULT(v(9, 256), cv)]
    states = [_state(sat_a), _state(sat_b), _state(unsat)]
    kfm = types.SimpleNamespace(interval_hook_for_size={}, concrete_hashes={})
    n = integration.batch_open_states(states, kfm=kfm, registry=UFRegistry())
    assert n == 2
    for cs in (sat_a, sat_b):
        m = integration._lookup_batch([c.raw for c in cs])
        assert m is not None
        assert all(bool(m.eval(c)) for c in cs)
    assert integration._lookup_batch([c.raw for c in unsat]) is None
