"""Wiring into a real Mythril (z3-bearing) process: the drop-in ``Optimize`` and the LASER plugin.

Mythril's own dependencies (z3, eth_abi, eth_hash) are not installed in the build image, so
the CPU tests drive this module against faithful stand-ins of z3 (tests/fake_z3.py) and of the
Mythril interfaces it touches (tests/mythril_standin.py); the GPU tests run the same code
against the real engine.

Seams:
* ``mythril.support.model.Optimize`` is the one name the query funnel resolves at call time
  (support/model.py:13, :37) — ``install()`` rebinds it to :func:`gpu_optimize_class`'s class.
  Its ``check()`` sends objective-free queries to the GPU: the z3 assertions are converted by
  the AST-id-cached walker (mythril_amd/z3_terms.py), the search runs under the solver's own
  timeout as a device deadline (``set_timeout``, support/model.py:38), and a witness returns
  ``z3.sat`` with a model whose ``eval`` answers any z3 expression (also ones over symbols
  outside the query, completed as z3's ``model_completion`` would).  Everything else
  (objectives, no witness, unsupported shapes, engine errors) goes to the original z3
  ``check()`` unchanged.
* ``MythrilAmdPluginBuilder`` — a ``MythrilLaserPlugin`` (mythril/plugin/interface.py:40-46,
  ``plugin_default_enabled = True`` read at discovery.py:71) whose LASER plugin batches every
  open state's constraints at ``stop_sym_trans`` (svm.py:307-308) — right before the
  tx-boundary ``is_possible`` pass of the next iteration (svm.py:266-286) — in ONE GPU
  launch, so that pass is answered from the batch.
"""

from __future__ import annotations

import logging
import os
import threading
from dataclasses import replace
from typing import Dict, List, Optional, Tuple

from .smt import terms as T
from .smt.to_dag import DEFAULT_REGISTRY, KeccakSpec, UFRegistry

log = logging.getLogger(__name__)

PART = (2 ** 256 - 1) // 10 ** 40

# Witnesses of the latest tx-boundary batch: key = the state's query as a tuple of
# hash-consed terms (structural: a key can only match the same constraints, whatever z3 does
# with AST ids) -> WitnessModel.  Cleared at every batch; a hit is re-checked against the
# query before it is returned.
_BATCH_CACHE: Dict[Tuple[T.Term, ...], object] = {}
_BATCH_LOCK = threading.Lock()


def sync_keccak_registry(kfm, registry: UFRegistry = DEFAULT_REGISTRY) -> None:
    """Mirror Mythril's KeccakFunctionManager state (intervals, concrete hashes) into the
    UF registry used by the lowering (keccak_function_manager.py:38-46, :158-163)."""
    for length, index in kfm.interval_hook_for_size.items():
        spec = registry.keccak.setdefault(length, KeccakSpec(lo=None))
        spec.lo = index * PART
    for data, digest in kfm.concrete_hashes.items():
        spec = registry.keccak.setdefault(data.size(), KeccakSpec(lo=None))
        spec.concrete[data.value] = digest.value


def _z3_sort_decl(z3, d):
    """A z3 FuncDeclRef for one of the witness's declarations (mythril_amd.smt.model.Decl)."""
    name, sort = d.name(), d.sort
    if sort == T.BOOL:
        return z3.Bool(name).decl()
    if sort[0] == "bv":
        return z3.BitVec(name, sort[1]).decl()
    if sort[0] == "array":
        return z3.Array(name, z3.BitVecSort(sort[1]), z3.BitVecSort(sort[2])).decl()
    # ("fn", dom..., rng)
    doms, rng = sort[1:-1], sort[-1]
    return z3.Function(name, *[z3.BitVecSort(w) for w in doms], z3.BitVecSort(rng))


class Z3WitnessView:
    """A GPU witness seen as one internal model of ``mythril.laser.smt.Model``
    (mythril/laser/smt/model.py:6-59): ``decls()``, ``__getitem__`` and ``eval`` over z3
    expressions.

    Immutable by design: the funnel stores the model in ``ModelCache`` (support/model.py:120)
    and every later quick-sat check deep-copies it (support_utils.py:62-68), so a copy is
    the object itself.  No module or reader object is held (z3 is imported where needed).
    ``eval`` converts the expression with the process-wide AST converter and evaluates it
    under the witness; symbols the witness does not assign evaluate to z3's
    ``model_completion`` defaults (0 / false / arrays 0 everywhere), and UF applications
    outside the query take the engine's interpretation of that UF.  With
    ``model_completion=False`` the completed value is returned as well (z3 would hand back
    the symbol itself for an unassigned one).
    """

    def __init__(self, internal):
        self.internal = internal   # mythril_amd.smt.model.WitnessModel
        self._decls = None

    def __deepcopy__(self, memo):
        return self

    def __copy__(self):
        return self

    def __reduce__(self):
        return (Z3WitnessView, (self.internal,))

    def decls(self):
        if self._decls is None:
            import z3

            self._decls = [_z3_sort_decl(z3, d) for d in self.internal.decls()]
        return self._decls

    def __getitem__(self, item):
        import z3

        if isinstance(item, int):
            return self.decls()[item]
        name = item.name()
        w = self.internal.w
        if name in w.vars:
            return z3.BitVecVal(w.vars[name], item.range().size())
        if name in w.bools:
            return z3.BoolVal(w.bools[name])
        return None

    def eval(self, expression, model_completion: bool = False):
        import z3

        from .z3_terms import converter

        term = converter(z3).term(expression)
        v = self.internal.w.ev(term)
        if term.is_bool:
            return z3.BoolVal(bool(v))
        return z3.BitVecVal(int(v), term.width)


def _query_key(terms: List[T.Term]) -> Tuple[T.Term, ...]:
    return tuple(t for t in terms if t is not T.TRUE)


def _lookup_batch(terms: List[T.Term]):
    """A parked tx-boundary witness for exactly this query, re-checked before use."""
    key = _query_key(terms)
    with _BATCH_LOCK:
        m = _BATCH_CACHE.get(key)
    if m is None:
        return None
    if all(m.w.ev(c) for c in key):
        return m
    return None


def gpu_optimize_class():
    """Build the drop-in subclass of ``mythril.laser.smt.Optimize`` (needs Mythril + z3)."""
    import z3
    from mythril.laser.ethereum.function_managers import keccak_function_manager
    from mythril.laser.smt import Optimize as MythrilOptimize
    from mythril.laser.smt.model import Model

    from .smt import gpu_check
    from .smt.solver import SolverStatistics
    from .z3_terms import converter

    class GpuOptimize(MythrilOptimize):
        def __init__(self):
            super().__init__()
            self._objectives = False
            self._gpu_model = None
            self._timeout_ms: Optional[int] = None

        def set_timeout(self, timeout: int) -> None:
            self._timeout_ms = timeout
            super().set_timeout(timeout)

        def minimize(self, element):
            self._objectives = True
            super().minimize(element)

        def maximize(self, element):
            self._objectives = True
            super().maximize(element)

        def check(self, *args):
            self._gpu_model = None
            if not self._objectives and not args and gpu_check.CONFIG.enabled:
                stats = SolverStatistics()
                stats.gpu_attempts += 1
                try:
                    terms = converter(z3).terms(self.raw.assertions())
                    internal = _lookup_batch(terms)
                    if internal is None:
                        sync_keccak_registry(keccak_function_manager)
                        cfg = gpu_check.CONFIG
                        if self._timeout_ms:
                            cfg = replace(cfg, timeout_ms=int(self._timeout_ms))
                        internal = gpu_check.check_sets([terms], config=cfg)[0]
                    if internal is not None:
                        stats.gpu_sat += 1
                        self._gpu_model = Model([Z3WitnessView(internal)])
                        return z3.sat
                except Exception as e:  # the GPU never decides a query it cannot answer
                    log.info("GPU path skipped: %s", e)
            return super().check(*args)

        def model(self):
            if self._gpu_model is not None:
                return self._gpu_model
            return super().model()

    return GpuOptimize


def install() -> None:
    """Rebind the funnel's Optimize (support/model.py:13 binds it by value at import).  The
    analysis process does not use torch, so the engine is loaded without it (PF_TORCH=0,
    mythril_amd/_lib.py) unless the caller chose otherwise."""
    import mythril.support.model as funnel

    os.environ.setdefault("PF_TORCH", "0")

    funnel.Optimize = gpu_optimize_class()


def state_terms(state) -> List[T.Term]:
    """One open state's query, as the funnel would pose it: the ``WorldState``'s
    ``constraints.get_all_constraints()`` (world_state.py:39; constraints.py:132-133 — path
    constraints + the keccak manager's conditions), python bools dropped
    (support/model.py:87-93).  Facade constraints (mythril_amd.smt terms) are used as they
    are; z3 ones go through the AST converter."""
    cs = [c for c in state.constraints.get_all_constraints() if not isinstance(c, bool)]
    raws = [c.raw for c in cs]
    if all(isinstance(r, T.Term) for r in raws):
        return raws
    import z3

    from .z3_terms import converter

    return converter(z3).terms(raws)


def batch_open_states(open_states, kfm=None, registry: UFRegistry = DEFAULT_REGISTRY) -> int:
    """Tx-boundary batch (svm.py:266-286): one GPU launch over every open ``WorldState``'s
    constraint set (svm.py:85,380: ``open_states`` holds WorldStates); each witness is
    parked under the state's query so the ``is_possible()`` pass that follows is answered
    without z3.  The previous batch's witnesses are dropped first.  Returns the number of
    states with a witness."""
    from .smt.gpu_check import check_sets

    if kfm is None:  # pragma: no cover - needs Mythril
        from mythril.laser.ethereum.function_managers import keccak_function_manager as kfm
    sync_keccak_registry(kfm, registry)
    sets = [state_terms(st) for st in open_states]
    models = check_sets(sets, registry=registry) if sets else []
    n = 0
    with _BATCH_LOCK:
        _BATCH_CACHE.clear()
        for terms, m in zip(sets, models):
            if m is not None:
                _BATCH_CACHE[_query_key(terms)] = m
                n += 1
    return n


def _plugin_classes():
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
