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
  open state's constraints in ONE GPU launch right before each tx-boundary ``is_possible``
  pass (svm.py:279-283): at ``start_execute_transactions`` (svm.py:227-228) for the first
  prune and at ``stop_sym_trans`` (svm.py:306-307) for the next one — never after the last
  transaction, which no prune follows (svm.py:259) — so every prune is answered from the
  batch.
"""

from __future__ import annotations

import logging
import os
import sys
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

    ``eval`` follows z3's ``ModelRef.eval`` contract, including that it never raises on a
    well-formed expression: ``check_quick_sat`` (support_utils.py:63-67) evaluates every
    later query against every cached model with no ``try``, so an exception here would
    abort ``get_model`` (support/model.py:96) and the analysis with it.
    * The expression is converted with the process-wide AST converter and evaluated under
      the witness — the kernel's interpretation, bit for bit.  With ``model_completion=True``
      symbols the witness does not assign take z3's completion defaults (0 / false / arrays
      0 everywhere) and UF applications outside the query the engine's UF interpretation.
    * With ``model_completion=False`` an expression over a symbol the witness does not
      interpret is returned partially evaluated, as z3 does: the assigned symbols are
      substituted and the result simplified, so a bare unassigned symbol comes back as
      itself (model.py:45-59).
    * An expression the converter cannot take (an operator outside the lowering's
      vocabulary) is evaluated the same way, by substitution + ``z3.simplify``.  If that does
      not reduce a Bool to a literal, the answer is ``False``: ``is_true`` fails, quick-sat
      moves on to the next model and the query reaches z3 — never an unsound ``True``.
    """

    def __init__(self, internal):
        self.internal = internal   # mythril_amd.smt.model.WitnessModel
        self._decls = None
        self._names = None

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

    def _interpreted(self) -> set:
        """Names the witness interprets: the symbols, arrays and UFs of its query."""
        if self._names is None:
            self._names = {d.name() for d in self.internal.decls()}
        return self._names

    def eval(self, expression, model_completion: bool = False):
        import z3

        try:
            from .smt.model import _symbols
            from .z3_terms import converter

            term = converter(z3).term(expression)
            names = self._interpreted()
            if model_completion or all(
                    (s.val[0] if s.op == "apply" else s.val) in names for s in _symbols([term])):
                v = self.internal.w.ev(term)
                if term.is_bool:
                    return z3.BoolVal(bool(v))
                return z3.BitVecVal(int(v), term.width)
        except Exception as e:  # noqa: BLE001 - z3's eval does not raise; see the docstring
            log.debug("witness eval by substitution: %s", e)
        try:
            return self._eval_substituted(z3, expression, model_completion)
        except Exception as e:  # noqa: BLE001
            log.debug("witness eval failed: %s", e)
            return z3.BoolVal(False) if z3.is_bool(expression) else expression

    def _eval_substituted(self, z3, expression, model_completion: bool):
        """Substitute the witness's symbol values (completion defaults for the others when
        ``model_completion``) and let z3 simplify; a Bool that does not reduce is False under
        completion."""
        w = self.internal.w
        pairs, seen, stack = [], set(), [expression]
        while stack:
            e = stack.pop()
            if e.get_id() in seen:
                continue
            seen.add(e.get_id())
            d = e.decl()
            if e.num_args() == 0 and d.kind() == z3.Z3_OP_UNINTERPRETED:
                name, srt = d.name(), e.sort()
                if z3.is_bool(e):
                    if name in w.bools or model_completion:
                        pairs.append((e, z3.BoolVal(bool(w.bools.get(name, False)))))
                elif z3.is_bv(e):
                    if name in w.vars or model_completion:
                        pairs.append((e, z3.BitVecVal(w.vars.get(name, 0), srt.size())))
                elif z3.is_array(e):
                    tab = w.tables().get(name)
                    if tab is not None or model_completion:
                        dom, rng = srt.domain(), srt.range()
                        a = z3.K(dom, z3.BitVecVal(0, rng.size()))
                        for i, v in sorted((tab or {}).items()):
                            a = z3.Store(a, z3.BitVecVal(i, dom.size()), z3.BitVecVal(v, rng.size()))
                        pairs.append((e, a))
                continue
            stack.extend(e.arg(i) for i in range(e.num_args()))
        r = z3.simplify(z3.substitute(expression, *pairs) if pairs else expression)
        if model_completion and z3.is_bool(r) and not (z3.is_true(r) or z3.is_false(r)):
            return z3.BoolVal(False)
        return r


# A tx-boundary batch whose prune may not come (the end of a prioritised sequence: whether
# another sequence follows is only known when its first prune query arrives): the states,
# and their query keys once computed.  Run by the first funnel query that is one of them.
_DEFERRED: Dict[str, object] = {"states": None, "keys": None}


def defer_batch(open_states) -> None:
    with _BATCH_LOCK:
        _DEFERRED["states"] = list(open_states)
        _DEFERRED["keys"] = None


def drop_deferred() -> None:
    with _BATCH_LOCK:
        _DEFERRED["states"] = _DEFERRED["keys"] = None


def run_deferred(terms: List[T.Term]) -> bool:
    """Run the deferred batch if ``terms`` (a funnel query) is one of its states' queries —
    the prune it was kept for has started.  True if it ran."""
    with _BATCH_LOCK:
        states, keys = _DEFERRED["states"], _DEFERRED["keys"]
    if states is None:
        return False
    if keys is None:
        keys = set()
        for st in states:
            try:
                keys.add(_query_key(state_terms(st)))
            except Exception:  # noqa: BLE001 - such a state goes to z3 in the prune
                pass
        with _BATCH_LOCK:
            if _DEFERRED["states"] is states:
                _DEFERRED["keys"] = keys
    if _query_key(terms) not in keys:
        return False
    with _BATCH_LOCK:
        if _DEFERRED["states"] is not states:
            return False
        _DEFERRED["states"] = _DEFERRED["keys"] = None
    batch_open_states(states)
    return True


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


_GPU_CLASSES = None


def _gpu_solver_classes():
    """(GpuOptimize, GpuSolver): the drop-in subclasses of ``mythril.laser.smt.Optimize`` and
    ``mythril.laser.smt.Solver`` (need Mythril + z3), built once per Mythril binding.  Both
    take the GPU path in the same ``check`` (:class:`_GpuCheck` below); ``GpuOptimize`` adds
    the objective bookkeeping (a query with objectives always goes to z3)."""
    global _GPU_CLASSES
    from mythril.laser.smt import Optimize as MythrilOptimize
    from mythril.laser.smt import Solver as MythrilSolver

    if (_GPU_CLASSES is not None and _GPU_CLASSES[0].__bases__[1] is MythrilOptimize
            and _GPU_CLASSES[1].__bases__[1] is MythrilSolver):
        return _GPU_CLASSES
    import z3
    from mythril.laser.ethereum.function_managers import keccak_function_manager
    from mythril.laser.smt.model import Model
    from mythril.laser.smt.solver.solver_statistics import stat_smt_query

    from .smt import gpu_check
    from .smt.solver import SolverStatistics
    from .z3_terms import converter

    class _GpuCheck:
        """The shared GPU path.  Query accounting: ``check`` carries Mythril's
        own ``@stat_smt_query`` (solver_statistics.py:7-25), exactly as ``BaseSolver.check``
        does (solver.py:72), so every query — GPU-answered or sent to z3 — bumps
        ``SolverStatistics().query_count`` and ``solver_time`` once; the z3 fallback runs
        ``BaseSolver.check``'s body (``_z3_check``) rather than the decorated
        ``super().check()``, which would count the query twice.  ``gpu_sat`` /
        ``gpu_attempts`` are kept beside them (mythril_amd.smt.solver), so "% discharged" =
        ``gpu_sat / query_count`` (:func:`discharge_ratio`)."""

        def __init__(self):
            super().__init__()
            self._objectives = False
            self._gpu_model = None
            self._timeout_ms: Optional[int] = None

        def set_timeout(self, timeout: int) -> None:
            self._timeout_ms = timeout
            super().set_timeout(timeout)

        @stat_smt_query
        def check(self, *args):
            self._gpu_model = None
            if not self._objectives and not args and gpu_check.CONFIG.enabled:
                stats = SolverStatistics()
                stats.gpu_attempts += 1
                try:
                    terms = converter(z3).terms(self.raw.assertions())
                    run_deferred(terms)
                    internal = _lookup_batch(terms)
                    if internal is None:
                        sync_keccak_registry(keccak_function_manager)
                        cfg = gpu_check.CONFIG
                        if self._timeout_ms:
                            cfg = replace(cfg, timeout_ms=int(self._timeout_ms))
                        # parent models: buckets new to this query start from the newest
                        # witness / z3 model values of their symbols (gpu_check._RECENT)
                        internal = gpu_check.check_sets([terms], config=cfg)[0]
                    if internal is not None:
                        stats.gpu_sat += 1
                        self._gpu_model = Model([Z3WitnessView(internal)])
                        return z3.sat
                except Exception as e:  # the GPU never decides a query it cannot answer
                    log.info("GPU path skipped: %s", e)
            result = self._z3_check(*args)
            if result == z3.sat and gpu_check.CONFIG.enabled:
                _note_z3_model(z3, self.raw)
            return result

        def _z3_check(self, *args):
            """``BaseSolver.check``'s body without its decorator (solver.py:72-88): stdout
            silenced around libz3, a ``Z3Exception`` becomes ``unknown``."""
            old_stdout = sys.stdout
            with open(os.devnull, "w") as dev_null_fd:
                sys.stdout = dev_null_fd
                try:
                    evaluate = self.raw.check(args)
                except z3.z3types.Z3Exception as e:
                    evaluate = z3.unknown
                    log.info("Encountered Z3 exception when checking the constraints: %s", e)
                finally:
                    sys.stdout = old_stdout
            return evaluate

        def model(self):
            if self._gpu_model is not None:
                return self._gpu_model
            return super().model()

    class GpuOptimize(_GpuCheck, MythrilOptimize):
        """The funnel's solver (support/model.py:37): objective-free queries to the GPU."""

        def minimize(self, element):
            self._objectives = True
            super().minimize(element)

        def maximize(self, element):
            self._objectives = True
            super().maximize(element)

    class GpuSolver(_GpuCheck, MythrilSolver):
        """``Solver()`` built outside the funnel (calldata.py:78, summary.py:114,
        summary/core.py:223): the same GPU path; ``reset`` / ``pop`` act on the z3 solver,
        whose assertions each ``check`` converts afresh."""

    _GPU_CLASSES = (GpuOptimize, GpuSolver)
    return _GPU_CLASSES


def gpu_optimize_class():
    """The drop-in subclass of ``mythril.laser.smt.Optimize`` (see :func:`_gpu_solver_classes`)."""
    return _gpu_solver_classes()[0]


def gpu_solver_class():
    """The drop-in subclass of ``mythril.laser.smt.Solver`` (see :func:`_gpu_solver_classes`)."""
    return _gpu_solver_classes()[1]


# Modules that build ``mythril.laser.smt.Solver`` directly, bound by value at their import
# (``from mythril.laser.smt import Solver``), so each needs its own rebinding: the symbolic
# calldata slice loop (laser/ethereum/state/calldata.py:16,78 — one query per byte, SAT on
# every iteration but the last) and the summary plugin's checks (plugins/summary/summary.py:8,
# 114; summary/core.py:30,223).
SOLVER_SITES = ("mythril.laser.ethereum.state.calldata",
                "mythril.laser.plugin.plugins.summary.summary",
                "mythril.laser.plugin.plugins.summary.core")


def _rebind_solver_sites() -> List[str]:
    """Point every ``SOLVER_SITES`` module's ``Solver`` at ``GpuSolver``; a module not yet
    loaded is imported first (so a later import finds it rebound), one that cannot be
    imported is skipped.  Returns the modules rebound."""
    import importlib

    from mythril.laser.smt import Solver as MythrilSolver

    gpu_solver = gpu_solver_class()
    done = []
    for name in SOLVER_SITES:
        mod = sys.modules.get(name)
        if mod is None:
            try:
                mod = importlib.import_module(name)
            except Exception as e:  # noqa: BLE001 - an optional Mythril module
                log.debug("Solver site %s not rebound: %s", name, e)
                continue
        if getattr(mod, "Solver", None) in (MythrilSolver, gpu_solver):
            mod.Solver = gpu_solver
            done.append(name)
    return done


def _note_z3_model(z3, raw) -> None:
    """A z3-answered query's model becomes the parent model of the buckets its children add
    (a child state = the parent's constraints + one JUMPI condition, instructions.py:1638,
    1662; the reference keeps the same model in ``model_cache``, support/model.py:120)."""
    from .smt import gpu_check

    try:
        m = raw.model()
        vals = {}
        for d in m.decls():
            if d.arity() != 0:
                continue
            v = m[d]
            if z3.is_bv_value(v):
                vals[d.name()] = v.as_long()
            elif z3.is_true(v) or z3.is_false(v):
                vals[d.name()] = int(z3.is_true(v))
        gpu_check.note_values(vals)
    except Exception as e:  # noqa: BLE001 - parents are only a search seed
        log.debug("z3 model not noted: %s", e)


def discharge_ratio() -> Optional[float]:
    """SURVEY §8(d) "% discharged": GPU-answered objective-free queries over Mythril's
    ``SolverStatistics().query_count`` (solver_statistics.py:14-21; counted only while
    Mythril's statistics are enabled, mythril_analyzer.py:147).  None before any query."""
    from mythril.laser.smt.solver.solver_statistics import SolverStatistics as MythrilStats

    from .smt.solver import SolverStatistics

    n = MythrilStats().query_count
    return SolverStatistics().gpu_sat / n if n else None


def install() -> None:
    """Rebind the funnel's Optimize (support/model.py:13 binds it by value at import), the
    ``Solver`` of the modules that query outside the funnel (:data:`SOLVER_SITES`), its
    ``model_cache`` (support/model.py:20; ``PF_MODEL_CACHE=0`` keeps the reference's) and the
    report's keccak concretisation (``mythril.analysis.solver._replace_with_actual_sha``).  The
    analysis process does not use torch, so the engine is loaded without it (PF_TORCH=0,
    mythril_amd/_lib.py) unless the caller chose otherwise.

    Devices: Mythril analyses in ONE process (``myth analyze``), so unless the caller chose
    (``PF_DEVICES``) or the process is one rank of a launcher (``LOCAL_RANK``), the engine
    drives every visible gfx950 device (``PF_DEVICES=all``, engine.get_engine): a tx-boundary
    batch is split into cost-balanced shards searched concurrently."""
    import mythril.support.model as funnel

    os.environ.setdefault("PF_TORCH", "0")
    if "LOCAL_RANK" not in os.environ:
        os.environ.setdefault("PF_DEVICES", "all")

    funnel.Optimize = gpu_optimize_class()
    _rebind_solver_sites()
    try:
        # keccak concretisation of reported transaction sequences (analysis/solver.py:129-165,
        # resolved at call time by get_transaction_sequence): batched, GPU for large batches
        import mythril.analysis.solver as report_solver

        from .concretize import live_replace_with_actual_sha

        report_solver._replace_with_actual_sha = live_replace_with_actual_sha
    except ImportError:  # pragma: no cover - a Mythril without the analysis package
        pass
    if os.environ.get("PF_MODEL_CACHE", "1") != "0":
        # the quick-sat loop before every objective-free query (support/model.py:95-98) as
        # one engine call over the cached models (mythril_amd/model_cache.py)
        from . import model_cache

        model_cache.install()


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
    states with a witness.

    The batch is an optimisation only: a state whose constraints do not convert (an operator
    or sort outside the lowering) is left out — its ``is_possible()`` goes to z3 as before —
    and an engine error drops the batch, never the analysis (svm.py:306-307 runs the hook
    with no guard)."""
    from .smt.gpu_check import check_sets

    if kfm is None:  # pragma: no cover - needs Mythril
        from mythril.laser.ethereum.function_managers import keccak_function_manager as kfm
    with _BATCH_LOCK:
        _BATCH_CACHE.clear()
    sync_keccak_registry(kfm, registry)
    sets = []
    for st in open_states:
        try:
            sets.append(state_terms(st))
        except Exception as e:  # noqa: BLE001 - z3 answers this state later
            log.info("tx-boundary batch: state left to z3 (%s)", e)
    try:
        models = check_sets(sets, registry=registry) if sets else []
    except Exception as e:  # noqa: BLE001
        log.warning("tx-boundary batch skipped: %s", e)
        return 0
    n = 0
    with _BATCH_LOCK:
        for terms, m in zip(sets, models):
            if m is not None:
                _BATCH_CACHE[_query_key(terms)] = m
                n += 1
    return n


def prune_follows(svm, tx_index: int) -> bool:
    """Whether LASER runs a tx-boundary prune (svm.py:266-283) next, given ``tx_index``
    transactions started since ``start_execute_transactions`` — i.e. whether a batch now
    would be read.

    * no prune at all without ``use_reachability_check`` (svm.py:266; off e.g. for concolic
      runs, concolic_execution.py:33), and none over zero open states (the loop breaks,
      svm.py:260);
    * the ordered loop (``tx_strategy is None``, svm.py:229-234) runs only if no plugin has
      executed the transactions already, and prunes at iterations 0 … ``transaction_count``-1
      (svm.py:259): after the last transaction's ``stop_sym_trans`` nothing prunes;
    * with a tx prioritiser (svm.py:235-237) every sequence re-enters the loop at i = 0
      (svm.py:248-250), so a batch after any transaction may feed the next sequence's first
      prune (the plugin defers the one at a sequence's end until that prune's first query:
      after the last sequence none comes).
    A stand-in without these attributes counts as the default ordered loop of unknown
    length (batch)."""
    if not getattr(svm, "use_reachability_check", True) or not svm.open_states:
        return False
    if getattr(svm, "tx_strategy", None) is not None:
        return True
    if tx_index == 0 and getattr(svm, "executed_transactions", False):
        return False
    n = getattr(svm, "transaction_count", None)
    return n is None or tx_index < n


_PLUGIN_CLASSES = None


def _plugin_classes():
    """(MythrilAmdLaserPlugin, MythrilAmdPluginBuilder), built once per Mythril binding.

    The builder is constructed the way Mythril constructs installed plugins —
    ``plugin(**plugin_args)`` (plugin/discovery.py:57) — and then read as a LASER
    ``PluginBuilder`` (``.enabled``, laser/plugin/loader.py:62-64).  ``MythrilLaserPlugin``
    resolves ``__init__`` to ``MythrilPlugin.__init__(**kwargs)``, which does not set
    ``enabled`` (plugin/interface.py:23-24 shadows laser/plugin/builder.py:14-15), so the
    builder's own ``__init__`` runs both."""
    global _PLUGIN_CLASSES
    from mythril.laser.plugin.builder import PluginBuilder
    from mythril.laser.plugin.interface import LaserPlugin
    from mythril.plugin.interface import MythrilLaserPlugin

    if _PLUGIN_CLASSES is not None and _PLUGIN_CLASSES[1].__bases__[0] is MythrilLaserPlugin:
        return _PLUGIN_CLASSES

    class MythrilAmdLaserPlugin(LaserPlugin):
        """Batches the open states right before each tx-boundary prune (svm.py:279-283).

        The prune of iteration i runs at the top of the loop body, before that iteration's
        ``start_sym_trans`` (svm.py:301) — so the hook that precedes it is the previous
        iteration's ``stop_sym_trans`` (svm.py:306), and for i = 0 ``start_execute_transactions``
        (svm.py:227-228, fired after contract creation, :190-206).  The iteration count is
        ``transaction_count`` (svm.py:259): the ``stop_sym_trans`` of the last transaction is
        followed by no prune, so it launches nothing (its batch would be dropped unread)."""

        def initialize(self, symbolic_vm) -> None:
            install()
            self.tx_index = 0          # start_sym_trans calls in the current transaction loop
            self.batches = 0
            self.deferred = 0

            def _batch():
                if not prune_follows(symbolic_vm, self.tx_index):
                    return
                tc = getattr(symbolic_vm, "transaction_count", None)
                if (getattr(symbolic_vm, "tx_strategy", None) is not None and self.tx_index > 0 and tc
                        and self.tx_index % tc == 0):
                    # the end of a prioritised sequence: a prune follows only if another
                    # sequence does, which the strategy's iterator does not tell — the batch
                    # waits for that prune's first query (run_deferred)
                    defer_batch(symbolic_vm.open_states)
                    self.deferred += 1
                    return
                try:
                    n = batch_open_states(symbolic_vm.open_states)
                    self.batches += 1
                    log.info("GPU batch before prune %d: %d/%d open states have a witness",
                             self.tx_index, n, len(symbolic_vm.open_states))
                except Exception as e:  # noqa: BLE001 - the batch is only an optimisation
                    log.warning("GPU batch failed: %s", e)

            @symbolic_vm.laser_hook("start_execute_transactions")
            def _before_first_prune():
                self.tx_index = 0
                _batch()

            @symbolic_vm.laser_hook("start_sym_trans")
            def _count():
                self.tx_index += 1
                drop_deferred()        # the prune a deferred batch was kept for has passed

            @symbolic_vm.laser_hook("stop_execute_transactions")
            def _done():
                drop_deferred()

            @symbolic_vm.laser_hook("stop_sym_trans")
            def _before_next_prune():
                _batch()

    class MythrilAmdPluginBuilder(MythrilLaserPlugin):
        name = "mythril-amd-path-feasibility"
        plugin_default_enabled = True
        author = "mythril_amd"
        plugin_version = "0.3.0"
        plugin_description = "MI355X batched path-feasibility engine (GPU witnesses skip z3)"

        def __init__(self, **kwargs):
            MythrilLaserPlugin.__init__(self, **kwargs)   # MythrilPlugin.__init__
            PluginBuilder.__init__(self)                  # enabled = True

        def __call__(self, *args, **kwargs):
            return MythrilAmdLaserPlugin()

    _PLUGIN_CLASSES = (MythrilAmdLaserPlugin, MythrilAmdPluginBuilder)
    return _PLUGIN_CLASSES


def __getattr__(name):  # lazy: importing mythril_amd never imports mythril
    if name in ("MythrilAmdLaserPlugin", "MythrilAmdPluginBuilder"):
        return dict(zip(("MythrilAmdLaserPlugin", "MythrilAmdPluginBuilder"), _plugin_classes()))[name]
    raise AttributeError(name)
