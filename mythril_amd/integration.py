"""Wiring into a real Mythril (z3-bearing) process: the drop-in ``Optimize`` and the LASER plugin.

Nothing here runs in this build container (Mythril's dependencies — z3, eth_abi, eth_hash —
are not installed); it is the code path INTEGRATION.md describes, kept import-safe.

Seams:
* ``mythril.support.model.Optimize`` is the one name the query funnel resolves at call time
  (support/model.py:13, :37) — ``install()`` rebinds it to :func:`gpu_optimize_class`'s class.
  Its ``check()`` sends objective-free queries to the GPU (z3 assertions are read through
  ``z3.Optimize.sexpr()`` with :mod:`mythril_amd.smtlib`), returns ``z3.sat`` with a model
  whose ``eval`` answers z3 expressions from the GPU witness, and otherwise delegates to the
  original z3 ``check()`` unchanged (objectives, no witness, unsupported shapes).
* ``MythrilAmdPluginBuilder`` — a ``MythrilLaserPlugin`` (mythril/plugin/interface.py:40-46,
  ``plugin_default_enabled = True`` read at discovery.py:71) whose LASER plugin batches every
  open state's constraints at ``stop_sym_trans`` (svm.py:307-308) — right before the
  tx-boundary ``is_possible`` pass of the next iteration (svm.py:266-286) — in ONE GPU
  launch, so that pass is answered from the batch.
"""

from __future__ import annotations

import logging
from typing import Dict, List, Optional

from .smt import terms as T
from .smt.to_dag import DEFAULT_REGISTRY, KeccakSpec, UFRegistry
from .smtlib import Reader, read_query

log = logging.getLogger(__name__)

PART = (2 ** 256 - 1) // 10 ** 40

# precomputed verdicts of the tx-boundary batch: key = tuple of z3 AST ids of a state's
# constraints (+ keccak conditions) -> internal witness model
_BATCH_CACHE: Dict[tuple, object] = {}


def sync_keccak_registry(kfm, registry: UFRegistry = DEFAULT_REGISTRY) -> None:
    """Mirror Mythril's KeccakFunctionManager state (intervals, concrete hashes) into the
    UF registry used by the lowering (keccak_function_manager.py:38-46, :158-163)."""
    for length, index in kfm.interval_hook_for_size.items():
        spec = registry.keccak.setdefault(length, KeccakSpec(lo=None))
        spec.lo = index * PART
    for data, digest in kfm.concrete_hashes.items():
        spec = registry.keccak.setdefault(data.size(), KeccakSpec(lo=None))
        spec.concrete[data.value] = digest.value


class _Z3View:
    """Adapter: evaluates z3 expressions under a GPU witness (Model-compatible)."""

    def __init__(self, internal, reader: Reader, z3mod):
        self.internal = internal
        self.reader = reader
        self.z3 = z3mod

    def decls(self):
        return []

    def __getitem__(self, item):
        name = item.name()
        w = self.internal.w
        if name in w.vars:
            return self.z3.BitVecVal(w.vars[name], item.range().size())
        if name in w.bools:
            return self.z3.BoolVal(w.bools[name])
        return None

    def eval(self, expression, model_completion: bool = False):
        term = self.reader.term(_parse_one(expression.sexpr()), {})
        v = self.internal.w.ev(term)
        if term.is_bool:
            return self.z3.BoolVal(bool(v))
        return self.z3.BitVecVal(int(v), term.width)


def _parse_one(text: str):
    from .smtlib import parse_sexprs

    return parse_sexprs(text)[0]


def gpu_optimize_class():  # pragma: no cover - needs Mythril + z3
    """Build the drop-in subclass of mythril.laser.smt.Optimize."""
    import z3
    from mythril.laser.smt import Optimize as MythrilOptimize
    from mythril.laser.smt.model import Model
    from mythril.laser.ethereum.function_managers import keccak_function_manager

    from .smt.gpu_check import check_sets
    from .smt.solver import SolverStatistics

    class GpuOptimize(MythrilOptimize):
        def __init__(self):
            super().__init__()
            self._objectives = False
            self._gpu_model = None

        def minimize(self, element):
            self._objectives = True
            super().minimize(element)

        def maximize(self, element):
            self._objectives = True
            super().maximize(element)

        def check(self, *args):
            if not self._objectives and not args:
                stats = SolverStatistics()
                stats.gpu_attempts += 1
                try:
                    reader = Reader()
                    q = reader.read(self.raw.sexpr())
                    key = tuple(sorted(a.get_id() for a in self.raw.assertions()))
                    internal = _BATCH_CACHE.pop(key, None)
                    if internal is None:
                        sync_keccak_registry(keccak_function_manager)
                        internal = check_sets([q.assertions])[0]
                    if internal is not None:
                        stats.gpu_sat += 1
                        self._gpu_model = Model([_Z3View(internal, reader, z3)])
                        return z3.sat
                except Exception as e:
                    log.info("GPU path skipped: %s", e)
            return super().check(*args)

        def model(self):
            if self._gpu_model is not None:
                return self._gpu_model
            return super().model()

    return GpuOptimize


def install() -> None:  # pragma: no cover - needs Mythril
    """Rebind the funnel's Optimize (support/model.py:13 binds it by value at import)."""
    import mythril.support.model as funnel

    funnel.Optimize = gpu_optimize_class()


def _z3_terms(raws):  # pragma: no cover - needs z3
    """z3 ASTs -> (terms, cache key): through the assertions' SMT-LIB2 text (what
    ``z3.Optimize.sexpr()`` prints, support/model.py:46-57) and mythril_amd.smtlib."""
    import z3

    s = z3.Optimize()
    s.add(raws)
    return read_query(s.sexpr()).assertions, tuple(sorted(r.get_id() for r in raws))


def state_terms(state):
    """One open state's query, as the funnel would pose it: ``get_all_constraints()``
    (constraints.py:132-133 — path constraints + the keccak manager's conditions), python
    bools dropped (support/model.py:87-93).  Constraints that already are mythril_amd.smt
    terms (the drop-in facade) are used as they are; z3 ones go through SMT-LIB2."""
    cs = [c for c in state.world_state.constraints.get_all_constraints() if not isinstance(c, bool)]
    raws = [c.raw for c in cs]
    if all(isinstance(r, T.Term) for r in raws):
        return raws, tuple(id(r) for r in raws)
    return _z3_terms(raws)


def batch_open_states(open_states, kfm=None, registry: UFRegistry = DEFAULT_REGISTRY) -> int:
    """Tx-boundary batch (svm.py:266-286): one GPU launch over every open state's
    constraint set; each witness is parked in ``_BATCH_CACHE`` under the state's key so the
    ``is_possible()`` pass that follows is answered without z3.  Returns the number of
    states with a witness."""
    from .smt.gpu_check import check_sets

    if kfm is None:  # pragma: no cover - needs Mythril
        from mythril.laser.ethereum.function_managers import keccak_function_manager as kfm
    sync_keccak_registry(kfm, registry)
    sets, keys = [], []
    for st in open_states:
        terms, key = state_terms(st)
        sets.append(terms)
        keys.append(key)
    models = check_sets(sets, registry=registry) if sets else []
    n = 0
    for k, m in zip(keys, models):
        if m is not None:
            _BATCH_CACHE[k] = m
            n += 1
    return n


def _plugin_classes():  # pragma: no cover - needs Mythril
    from mythril.laser.plugin.builder import PluginBuilder
    from mythril.laser.plugin.interface import LaserPlugin
    from mythril.plugin.interface import MythrilLaserPlugin

    class MythrilAmdLaserPlugin(LaserPlugin):
        def initialize(self, symbolic_vm) -> None:
            install()

            @symbolic_vm.laser_hook("stop_sym_trans")
            def _batch():
                n = batch_open_states(symbolic_vm.open_states)
                log.info("GPU batch: %d/%d open states have a witness", n, len(symbolic_vm.open_states))

    class MythrilAmdPluginBuilder(MythrilLaserPlugin, PluginBuilder):
        name = "mythril-amd-path-feasibility"
        plugin_default_enabled = True
        author = "mythril_amd"
        plugin_description = "MI355X batched path-feasibility engine (GPU witnesses skip z3)"

        def __call__(self, *args, **kwargs):
            return MythrilAmdLaserPlugin()

    return MythrilAmdLaserPlugin, MythrilAmdPluginBuilder


def __getattr__(name):  # lazy: importing mythril_amd never imports mythril
    if name in ("MythrilAmdLaserPlugin", "MythrilAmdPluginBuilder"):
        return dict(zip(("MythrilAmdLaserPlugin", "MythrilAmdPluginBuilder"), _plugin_classes()))[name]
    raise AttributeError(name)
