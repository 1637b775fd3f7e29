"""Seam #2: the LASER plugin and the tx-boundary batch
(mythril_amd/integration.py).

Mythril itself is not importable here (z3, eth_abi, eth_hash missing — SURVEY §8c), so the
plugin classes are exercised against the Mythril plugin stack restated line for line
(tests/mythril_standin.py: the interfaces they subclass, discovery and both loaders) and a
stand-in symbolic VM exposing ``laser_hook`` and ``open_states`` (svm.py:133-145, 726-741).  The batch itself runs on the GPU over states
whose constraints are mythril_amd.smt terms (the drop-in facade); with z3 present the same
function reads z3 ASTs through SMT-LIB2.
"""

import os
import types

import pytest

from mythril_amd import integration
from mythril_amd.smt import ULT, symbol_factory
from mythril_amd.smt.to_dag import UFRegistry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _entry_points():
    """The ``"mythril.plugins"`` entry points the package metadata declares (setup.cfg
    ``[options.entry_points]``; test_wheel_declares_the_entry_point builds the wheel)."""
    import configparser

    cfg = configparser.ConfigParser()
    cfg.read(os.path.join(ROOT, "setup.cfg"))
    out = {}
    for line in cfg["options.entry_points"]["mythril.plugins"].strip().splitlines():
        name, value = (x.strip() for x in line.split("=", 1))
        out[name] = value
    return out


@pytest.fixture
def stub_mythril(monkeypatch):
    """The Mythril plugin stack restated line for line (tests/mythril_standin.py:
    plugin/interface.py:6-46, laser/plugin/builder.py:6-21, laser/plugin/loader.py:12-75,
    plugin/discovery.py, plugin/loader.py), with the package's declared entry points as the
    installed plugins."""
    import fake_z3
    import mythril_standin

    return mythril_standin.install(monkeypatch, fake_z3, installed_plugins=_entry_points())


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
    """discovery.py:71 reads plugin_default_enabled; the builder is a MythrilLaserPlugin
    (so also a LASER PluginBuilder, plugin/interface.py:40) built with keyword arguments
    (discovery.py:57) that still carries ``enabled`` (laser/plugin/builder.py:14-15)."""
    laser_cls, builder_cls = integration._plugin_classes()
    assert issubclass(builder_cls, stub_mythril.MythrilLaserPlugin)
    assert issubclass(builder_cls, stub_mythril.PluginBuilder)
    assert issubclass(builder_cls, stub_mythril.MythrilPlugin)
    assert builder_cls.plugin_default_enabled is True
    assert builder_cls.name == "mythril-amd-path-feasibility"
    b = builder_cls(**{})
    assert b.enabled is True
    plugin = b()
    assert isinstance(plugin, stub_mythril.LaserPlugin)
    assert integration._plugin_classes() is integration._plugin_classes()   # built once


def test_reference_loader_sequence_reaches_the_hook(stub_mythril, monkeypatch):
    """The construction sequence of a real ``myth analyze`` with the package installed:
    ``MythrilPluginLoader()`` (cli.py:32) loads every default-enabled entry point —
    ``PluginDiscovery.build_plugin`` -> ``plugin(**{})`` (discovery.py:50-57) ->
    ``LaserPluginLoader().load`` (plugin/loader.py:65-68) — and ``SymExecWrapper`` then calls
    ``instrument_virtual_machine(laser, None)`` (analysis/symbolic.py:169), which reads
    ``.enabled``, builds the LASER plugin and initialises it (laser/plugin/loader.py:55-75);
    LASER fires ``stop_sym_trans`` after each transaction (svm.py:306-307)."""
    calls = {"batch": []}
    monkeypatch.setattr(integration, "batch_open_states",
                        lambda states: calls["batch"].append(list(states)) or 0)
    ml = stub_mythril.MythrilPluginLoader()
    assert [type(p).__name__ for p in ml.loaded_plugins] == ["MythrilAmdPluginBuilder"]
    laser_loader = stub_mythril.LaserPluginLoader()
    assert laser_loader.is_enabled("mythril-amd-path-feasibility")
    svm = FakeSVM(open_states=["s0", "s1"])
    laser_loader.instrument_virtual_machine(svm, None)
    assert "mythril-amd-path-feasibility" in laser_loader.plugin_list
    import sys
    assert sys.modules["mythril.support.model"].Optimize.__name__ == "GpuOptimize"
    assert os.environ.get("PF_DEVICES") == "all"     # one Mythril process drives every GPU
    for hook in svm.hooks["stop_sym_trans"]:
        hook()
    assert calls["batch"] == [["s0", "s1"]]


def test_install_keeps_an_explicit_device_choice(stub_mythril, monkeypatch):
    """PF_DEVICES (or a launcher's LOCAL_RANK) wins over the all-devices default."""
    monkeypatch.setenv("PF_DEVICES", "1")
    integration.install()
    assert os.environ["PF_DEVICES"] == "1"
    monkeypatch.delenv("PF_DEVICES")
    monkeypatch.setenv("LOCAL_RANK", "3")
    integration.install()
    assert "PF_DEVICES" not in os.environ


def test_plugin_hook_never_raises(stub_mythril, monkeypatch):
    """svm.py:306-307 runs the hook with no guard: an engine failure inside the batch must
    not end the analysis."""
    def boom(states):
        raise RuntimeError("device lost")

    monkeypatch.setattr(integration, "batch_open_states", boom)
    monkeypatch.setattr(integration, "install", lambda: None)
    svm = FakeSVM(open_states=["s0"])
    integration._plugin_classes()[1](**{})().initialize(svm)
    svm.hooks["stop_sym_trans"][0]()


def test_wheel_declares_the_entry_point(tmp_path):
    """The package builds offline into a wheel whose entry_points.txt registers the builder
    under ``mythril.plugins`` (what PluginDiscovery iterates, discovery.py:22-36)."""
    import shutil
    import subprocess
    import sys
    import zipfile

    src = tmp_path / "src"
    src.mkdir()
    for f in ("pyproject.toml", "setup.cfg"):
        shutil.copy(os.path.join(ROOT, f), src / f)
    shutil.copytree(os.path.join(ROOT, "mythril_amd"), src / "mythril_amd",
                    ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation",
                        "--no-index", "-q", str(src), "-w", str(tmp_path / "dist")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    whl, = (tmp_path / "dist").glob("mythril_amd-*.whl")
    z = zipfile.ZipFile(whl)
    ep = [n for n in z.namelist() if n.endswith("entry_points.txt")]
    text = z.read(ep[0]).decode()
    assert "[mythril.plugins]" in text
    assert "mythril_amd = mythril_amd.integration:MythrilAmdPluginBuilder" in text
    assert any(n.startswith("mythril_amd/integration.py") for n in z.namelist())


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
