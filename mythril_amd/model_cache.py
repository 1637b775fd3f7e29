"""GPU-resident ``ModelCache`` — the reference's quick-sat loop as one engine call.

Reference (mythril/support/support_utils.py:57-71, called before every objective-free query
at mythril/support/model.py:95-98)::

    @lru_cache(maxsize=2**10)
    def check_quick_sat(self, constraints):
        for model in reversed(self.model_cache.lru_cache.keys()):     # most recent first
            model_copy = deepcopy(model)
            if is_true(model_copy.eval(constraints, model_completion=True)):
                self.model_cache.put(model, self.model_cache.get(model) + 1)   # LRU bump
                return model
        return False

Up to 100 models are deep-copied and evaluated one after the other.  Here the query
``constraints`` (``simplify(And(*cs)).raw``) is converted once (the AST-id-cached walker,
z3_terms.py) and lowered once by the EXPLICIT lowering (to_dag.ExplicitLowering, or
libpflower.so's ``PFLT_EXPLICIT``): every base-array read and UF application is a leaf
variable.  Each cached model supplies its values of those leaves — a z3 model through
``eval(leaf, model_completion=True)`` on one private copy, a GPU witness through its own
interpretation (``Witness.ev``) — memoised per (model, leaf term), so a leaf is evaluated once
per model for the whole analysis (LASER's queries share almost all of their leaves).  All
models are then evaluated in ONE ``pf_eval_assignments`` launch (one lane per model) and the
answer is the first model, most recent first, whose lane is true — the model the reference
loop returns, with the same LRU bump and the same ``lru_cache`` on the method.

The newest FIRST_STAGE models go in a first launch (the loop's most frequent answers), the
others in a second one only if none of those holds.  A model whose leaves cannot be evaluated
(an empty ``Model()``, a leaf its evaluator rejects) is decided by the reference's own
statement for that query, in its place in the order; a
query the converter or the lowering cannot take runs the reference loop unchanged.  The
decision itself is never approximated: the program computes the conjunction's exact value
(SMT-LIB bit-vector semantics, GPU-parity-tested against the oracle) from exact leaf values.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from collections import OrderedDict
from collections.abc import Mapping
from copy import deepcopy
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .lower import LoweringError, lower
from .smt import terms as T
from .smt.to_dag import ExplicitLowering

log = logging.getLogger(__name__)


@dataclass
class QuickSatStats:
    queries: int = 0          # check_quick_sat calls that reached the engine path (lru misses)
    hits: int = 0             # ... that returned a model
    engine_calls: int = 0     # pf_eval_assignments launches
    models_engine: int = 0    # model evaluations done on the engine
    models_host: int = 0      # model evaluations done by the reference statement (fallback)
    reference_loops: int = 0  # queries the converter / lowering could not take (reference loop)
    leaf_evals: int = 0       # (model, leaf) values computed (the rest were memoised)
    leaf_evals_native: int = 0   # of which by the native witness evaluator (pflt_witness_values)
    verdicts_memo: int = 0       # (model, conjunct) verdicts read from a model's memo
    verdicts_native: int = 0     # ... computed by the native witness evaluator (small batches)
    verdicts_engine: int = 0     # ... computed on the engine (pf_eval_programs)
    phase_s: Dict[str, float] = field(default_factory=dict)


STATS = QuickSatStats()
_STATS_LOCK = threading.Lock()

# query term -> (leaf terms, program) or the LoweringError text; the quick-sat of a query is
# lru-cached by the caller, but the same conjunction term reaches here from distinct z3 ASTs
_PROGRAMS: "OrderedDict[T.Term, object]" = OrderedDict()
_PROGRAMS_MAX = 512
_PROG_LOCK = threading.Lock()


def explicit_program(query: T.Term):
    """(leaf terms, program) of a Bool query term under the explicit lowering; raises
    LoweringError for a query outside the lowering's vocabulary."""
    with _PROG_LOCK:
        hit = _PROGRAMS.get(query)
        if hit is not None:
            _PROGRAMS.move_to_end(query)
    if hit is None:
        conj = list(query.args) if query.op == "and" else [query]
        try:
            hit = _lower_explicit(conj)
        except (LoweringError, ValueError, OverflowError, RecursionError) as e:
            hit = f"{type(e).__name__}: {e}"
        with _PROG_LOCK:
            _PROGRAMS[query] = hit
            while len(_PROGRAMS) > _PROGRAMS_MAX:
                _PROGRAMS.popitem(last=False)
    if isinstance(hit, str):
        raise LoweringError(hit)
    return hit


def _lower_explicit(conj: List[T.Term]):
    """Native (libpflower.so PFLT_EXPLICIT) when built, else the Python reference lowering —
    the same program node for node (tests/test_model_cache.py)."""
    from .smt import native_terms

    if native_terms.store() is not None and native_terms.has_explicit():
        r = native_terms.lower_native(conj, _EMPTY_REG, None, native_terms.PROGRAM | native_terms.EXPLICIT, 0)
        # the batch is packed from the native result (ir.Batch -> pack_batch): nothing else
        # of the program is decoded
        return r.var_terms(), native_terms.NativeProgram(r, 0)
    return lower_explicit_py(conj)


def lower_explicit_py(conj: List[T.Term]):
    lo = ExplicitLowering().lower(conj)
    return lo.var_terms, lower(lo.dag, seed=0)


def n_vars(program) -> int:
    if isinstance(program, ExplicitGroups):
        return len(program.gather)
    r = getattr(program, "native_result", None)
    return int(r.info[0]) if r is not None else len(program.vars)


# ---- conjunct groups: a long query as several programs side by side ----------------------
# One quick-sat launch is a lone wave walking the whole conjunction (~0.45 us per bytecode
# instruction, §3 of DESIGN.md; LASER's queries lower to ~500 instructions).  With
# SPLIT_NODES > 0, a query whose (flattened) conjuncts add up to more than SPLIT_NODES term
# nodes is lowered as up to MAX_GROUPS programs over balanced groups of its conjuncts
# (largest first onto the lightest group), all run in one launch (pf_eval_programs: one wave
# per group and 64 models); a model satisfies the query iff it satisfies every group.
# Shared subterms are lowered once per group.  Off by default: measured on the quick-sat
# workload (profiles/r05t_quick_sat_split.md) the launches got 0.09 ms cheaper per query and
# the lowering 0.3 ms dearer (one native lowering per group, the shared keccak terms lowered
# again in each).  PF_QS_SPLIT_NODES turns it on.
MAX_GROUPS = 8
SPLIT_NODES = int(os.environ.get("PF_QS_SPLIT_NODES", "0"))


class ExplicitGroups:
    """The programs of one query's conjunct groups: ``gather`` lists, group after group,
    the position in the query's leaf list of each program variable (the SoA rows the
    programs read, in pf_eval_programs' order); ``pack`` the packed arrays, made once."""

    __slots__ = ("programs", "gather", "offsets", "conjs", "_pack")

    def __init__(self, programs, gather: np.ndarray, offsets: List[int], conjs: Optional[List[T.Term]] = None):
        self.programs, self.gather, self.offsets = programs, gather, offsets
        self.conjs = conjs      # with CONJ_PROGRAMS: the conjunct term of each program
        self._pack = None

    def spans(self) -> List[Tuple[int, int]]:
        ends = self.offsets[1:] + [len(self.gather)]
        return list(zip(self.offsets, ends))

    def subset(self, ks: Sequence[int]) -> Tuple[List[int], "ExplicitGroups"]:
        """(leaf positions, group) of programs ``ks`` alone: the group's gather renumbered
        onto the returned positions (indices into the query's leaf list)."""
        spans = self.spans()
        pos: Dict[int, int] = {}
        gather, offsets = [], []
        for k in ks:
            lo, hi = spans[k]
            offsets.append(len(gather))
            for g in self.gather[lo:hi]:
                gather.append(pos.setdefault(int(g), len(pos)))
        return list(pos), ExplicitGroups([self.programs[k] for k in ks], np.array(gather, dtype=np.int64), offsets,
                                         [self.conjs[k] for k in ks] if self.conjs is not None else None)

    def pack(self):
        if self._pack is None:
            from .ir import Batch

            b = Batch(list(self.programs))
            self._pack = tuple(np.ascontiguousarray(a, dtype=np.uint32).reshape(-1)
                               for a in (b.code, b.consts, b.schema, b.descs))
        return self._pack


def _term_nodes(t: T.Term) -> int:
    seen = set()
    stack = [t]
    while stack:
        x = stack.pop()
        if x in seen:
            continue
        seen.add(x)
        stack.extend(x.args)
    return len(seen)


def flat_conjuncts(conj: List[T.Term]) -> List[T.Term]:
    """The conjuncts with nested ``and``s opened (the keccak manager's conditions arrive as
    one conjunct of nested ands), in order."""
    out: List[T.Term] = []
    stack = list(reversed(conj))
    while stack:
        c = stack.pop()
        if c.op == "and":
            stack.extend(reversed(c.args))
        else:
            out.append(c)
    return out


def conjunct_groups(conj: List[T.Term]) -> List[List[T.Term]]:
    """The (flattened) conjuncts in balanced groups (one group when the query is short)."""
    conj = flat_conjuncts(conj)
    if len(conj) < 2:
        return [conj]
    sizes = [_term_nodes(c) for c in conj]
    total = sum(sizes)
    g = min(len(conj), MAX_GROUPS, -(-total // SPLIT_NODES))
    if g < 2:
        return [conj]
    groups: List[List[int]] = [[] for _ in range(g)]
    load = [0] * g
    for i in sorted(range(len(conj)), key=lambda i: -sizes[i]):
        k = min(range(g), key=load.__getitem__)
        groups[k].append(i)
        load[k] += sizes[i]
    # each group keeps the conjuncts' query order
    return [[conj[i] for i in sorted(gr)] for gr in groups if gr]


_GROUPS: "OrderedDict[T.Term, object]" = OrderedDict()


# Every (flattened) conjunct of a query is its own program, lowered once and cached by
# conjunct across queries — LASER's queries along a path share all but their newest
# conjuncts, so a query lowers only those — and all of a query's conjunct programs run in one
# launch (pf_eval_programs), side by side: the launch lasts as long as the longest conjunct,
# not the whole conjunction.  Measured (profiles/r05z_quick_sat_conj.md): witness cache 0.93
# -> 0.67 ms mean per query (lowering 0.26 -> 0.13, launch 0.43 -> 0.34).  PF_QS_CONJ=0 lowers
# each query whole.
CONJ_PROGRAMS = os.environ.get("PF_QS_CONJ", "1") != "0"
_CONJ: "OrderedDict[T.Term, object]" = OrderedDict()
_CONJ_MAX = 4096   # lowering results of a few KB each


def _conj_program(c: T.Term):
    with _PROG_LOCK:
        hit = _CONJ.get(c)
        if hit is not None:
            _CONJ.move_to_end(c)
    if hit is None:
        try:
            hit = _lower_explicit([c])
        except (LoweringError, ValueError, OverflowError, RecursionError) as e:
            hit = f"{type(e).__name__}: {e}"
        with _PROG_LOCK:
            _CONJ[c] = hit
            while len(_CONJ) > _CONJ_MAX:
                _CONJ.popitem(last=False)
    if isinstance(hit, str):
        raise LoweringError(hit)
    return hit


def explicit_groups(query: T.Term):
    """(leaf terms, ExplicitGroups or a single program) of a Bool query term: a long
    conjunction split by ``conjunct_groups`` (or, with CONJ_PROGRAMS, one cached program per
    conjunct), each group lowered as explicit_program does; raises LoweringError as
    explicit_program does."""
    if (SPLIT_NODES <= 0 and not CONJ_PROGRAMS) or query.op != "and":
        return explicit_program(query)
    with _PROG_LOCK:
        hit = _GROUPS.get(query)
        if hit is not None:
            _GROUPS.move_to_end(query)
    if hit is None:
        if CONJ_PROGRAMS:
            conj = [c for c in dict.fromkeys(flat_conjuncts(list(query.args))) if c is not T.TRUE]
            groups = [[c] for c in conj] or [[T.TRUE]]
        else:
            groups = conjunct_groups(list(query.args))
        try:
            if len(groups) == 1 and not CONJ_PROGRAMS:
                hit = explicit_program(query)
            else:
                lowered = [_conj_program(gr[0]) for gr in groups] if CONJ_PROGRAMS else \
                    [_lower_explicit(gr) for gr in groups]
                pos: Dict[T.Term, int] = {}
                gather, offsets = [], []
                for vt, prog in lowered:
                    if len(vt) != n_vars(prog):
                        raise LoweringError("explicit group: variables and leaves differ")
                    offsets.append(len(gather))
                    for t in vt:
                        gather.append(pos.setdefault(t, len(pos)))
                hit = (list(pos), ExplicitGroups([p for _, p in lowered], np.array(gather, dtype=np.int64),
                                                 offsets, [gr[0] for gr in groups] if CONJ_PROGRAMS else None))
        except (LoweringError, ValueError, OverflowError, RecursionError) as e:
            hit = f"{type(e).__name__}: {e}"
        with _PROG_LOCK:
            _GROUPS[query] = hit
            while len(_GROUPS) > _PROGRAMS_MAX:
                _GROUPS.popitem(last=False)
    if isinstance(hit, str):
        raise LoweringError(hit)
    return hit


class _EmptyRegistry:
    """The registry the explicit lowering reads: no actors, no keccak specs (UFs are leaves)."""

    keccak: dict = {}
    actors: tuple = ()


_EMPTY_REG = _EmptyRegistry()


# ---- per-model leaf values --------------------------------------------------------------

LEAF_VALS_MAX = 1 << 15


class LeafValues:
    """One cached model's values of leaf terms, each computed once and kept as the 32 bytes
    (little-endian) of its row in pf_eval_assignments' input.

    ``evaluate_many`` (optional) values several leaves in ONE evaluation of the model — a z3
    model evaluates the concatenation of the leaves with one ``eval``, sharing every common
    subterm (store chains, keccak applications) the way the reference's single eval of the
    whole conjunction does, where one ``eval`` per leaf re-walked them per leaf."""

    __slots__ = ("evaluate", "evaluate_many", "vals", "verdicts")

    def __init__(self, evaluate: Callable[[T.Term], int],
                 evaluate_many: Optional[Callable[[Sequence[T.Term]], List[int]]] = None):
        self.evaluate = evaluate
        self.evaluate_many = evaluate_many
        self.vals: Dict[T.Term, bytes] = {}
        # conjunct -> its truth under this model (CONJ_PROGRAMS): a model is immutable, so a
        # conjunct is evaluated under it once, whichever query it comes with
        self.verdicts: Dict[T.Term, bool] = {}

    def _put(self, t: T.Term, x: int) -> bytes:
        v = self.vals[t] = (int(x) & T.M(max(t.width, 1))).to_bytes(32, "little")
        return v

    def row(self, leaves: Sequence[T.Term]) -> Optional[bytes]:
        """The values of ``leaves`` as one byte row; None if the model's evaluator rejects
        one of them."""
        vals = self.vals
        if len(vals) > LEAF_VALS_MAX:   # bounded like the verdict memo: values are recomputable
            vals.clear()
        missing = [t for t in dict.fromkeys(leaves) if t not in vals]
        if len(missing) > 1 and self.evaluate_many is not None:
            try:
                for t, x in zip(missing, self.evaluate_many(missing)):
                    self._put(t, x)
            except Exception as e:  # noqa: BLE001 - per leaf below finds the one it rejects
                log.debug("batched leaf evaluation declined: %s", e)
        new = 0
        for t in missing:
            if t in vals:
                new += 1
                continue
            try:
                x = int(self.evaluate(t))
            except Exception as e:  # noqa: BLE001 - the reference statement decides then
                log.debug("leaf %s not evaluated: %s", t.op, e)
                return None
            self._put(t, x)
            new += 1
        if new:
            with _STATS_LOCK:
                STATS.leaf_evals += new
        return b"".join([vals[t] for t in leaves])

    def value(self, t: T.Term) -> Optional[int]:
        v = self.vals.get(t)
        return None if v is None else int.from_bytes(v, "little")


class NativeLeafValues(LeafValues):
    """LeafValues of a GPU witness held natively (native_terms.NativeWitness): ``native_rows``
    reads the rows of many such models in one native call (the values memoised in the native
    witness, not here); a model with a leaf the native evaluator declines goes to ``row`` —
    the Python witness's ``leaf_value`` — as before."""

    __slots__ = ("native", "reg")

    def __init__(self, evaluate: Callable[[T.Term], int], native, reg):
        super().__init__(evaluate)
        self.native, self.reg = native, reg


# threads of one native leaf evaluation (the witnesses split across them)
LEAF_THREADS = max(1, min(8, os.cpu_count() or 1))


def native_rows(leaf_values: Sequence[Optional[LeafValues]], leaves: Sequence[T.Term]) -> Mapping:
    """{position in ``leaf_values``: its row as (len(leaves), 8) u32 limbs} for the natively
    held models whose every leaf evaluated natively — one pflt_witness_values call per term
    store (and registry)."""
    groups: Dict[Tuple[int, int], List[int]] = {}
    for j, lv in enumerate(leaf_values):
        if isinstance(lv, NativeLeafValues):
            groups.setdefault((id(lv.native.st), id(lv.reg)), []).append(j)
    out: Mapping = {}
    if not groups or not leaves:
        return out
    from .smt import native_terms

    for js in groups.values():
        lvs = [leaf_values[j] for j in js]
        vals, ok = native_terms.witness_values_many([lv.native for lv in lvs], list(leaves), lvs[0].reg,
                                                    min(LEAF_THREADS, len(lvs)))
        full = ok.all(axis=1)
        if len(groups) == 1 and len(js) == len(leaf_values) and full.all():
            # every model native and complete (a cache of GPU witnesses): the block itself,
            # models in order — eval_rows takes it as the SoA source without restacking
            out = _NativeBlock(vals)
        else:
            for j, m in zip(js, range(len(js))):
                if full[m]:
                    out[j] = vals[m]
        with _STATS_LOCK:
            STATS.leaf_evals_native += int(full.sum()) * len(leaves)
    return out


class _NativeBlock(Mapping):
    """native_rows' answer when every model of the stage is native and complete: the rows
    as one (models, leaves, 8) array (``block``), readable per model like the dict
    native_rows returns otherwise (no per-model views made unless asked for)."""

    __slots__ = ("block",)

    def __init__(self, block: np.ndarray):
        self.block = block

    def __getitem__(self, j: int) -> np.ndarray:
        if not 0 <= j < len(self.block):
            raise KeyError(j)
        return self.block[j]

    def __iter__(self):
        return iter(range(len(self.block)))

    def __len__(self) -> int:
        return len(self.block)


def soa_of(rows: Sequence, n_vars: int) -> np.ndarray:
    """[var][limb][cand] u32 (pf_eval_assignments' layout) from per-candidate rows: byte
    strings (``n_vars`` x 32 bytes each) or (n_vars, 8) u32 limb arrays."""
    n = len(rows)
    if n_vars == 0:
        return np.zeros((1, 8, n), dtype=np.uint32)
    if isinstance(rows, np.ndarray):   # a (models, vars, 8) block (native_rows)
        return np.ascontiguousarray(rows.transpose(1, 2, 0), dtype=np.uint32)
    if all(isinstance(r, bytes) for r in rows):
        a = np.frombuffer(b"".join(rows), dtype="<u4").reshape(n, n_vars, 8)
    else:
        a = np.stack([np.frombuffer(r, dtype="<u4").reshape(n_vars, 8) if isinstance(r, bytes) else r
                      for r in rows])
    return np.ascontiguousarray(a.transpose(1, 2, 0), dtype=np.uint32)


def rows_of_ints(rows: Sequence[Sequence[int]]) -> List[bytes]:
    return [b"".join((v & T.M(256)).to_bytes(32, "little") for v in r) for r in rows]


def eval_rows(program, rows: Sequence[bytes], engine=None) -> np.ndarray:
    """SAT flag of each explicit assignment: one launch (pf_eval_program, or pf_eval_programs
    for conjunct groups; an engine without them — the tests' oracle engine — through upload +
    eval_assignments per program)."""
    if engine is None:
        from .engine import get_engine

        engine = get_engine()
    if isinstance(program, ExplicitGroups):
        t0 = time.perf_counter()
        n_leaves = int(program.gather.max()) + 1 if len(program.gather) else 0
        if not n_leaves:
            soa = soa_of(rows, 0)
        elif isinstance(rows, np.ndarray):   # (models, leaves, 8): transpose once, gather rows
            soa = soa_of(rows, n_leaves)[program.gather]
        else:
            soa = soa_of(rows, n_leaves)[program.gather]
        if hasattr(engine, "eval_programs"):
            pack = program.pack()
            dt = time.perf_counter() - t0
            with _STATS_LOCK:   # the host share of the "eval" phase: SoA gather + packing
                STATS.phase_s["eval_host"] = STATS.phase_s.get("eval_host", 0.0) + dt
            return engine.eval_programs(pack, soa).all(axis=0)
        ends = program.offsets[1:] + [len(program.gather)]
        out = np.ones(soa.shape[-1], dtype=bool)
        for prog, lo, hi in zip(program.programs, program.offsets, ends):
            out &= _eval_one(prog, np.ascontiguousarray(soa[lo:hi]) if hi > lo else soa_of(rows, 0), engine)
        return out
    return _eval_one(program, soa_of(rows, n_vars(program)), engine)


def _eval_one(program, soa: np.ndarray, engine) -> np.ndarray:
    if hasattr(engine, "eval_program"):
        return engine.eval_program(program, soa)
    db = engine.upload([program])
    try:
        return engine.eval_assignments(db, 0, soa)
    finally:
        db.free()


# Models evaluated in the first launch: the reference loop stops at the first model that
# holds, and in a live analysis that is most often one of the newest (the parent state's
# model, bumped to the front by the query before) — computing every z3 model's leaves for
# such a query would cost more than the loop it replaces.  The first launch therefore covers
# the newest models up to (not including) the (FIRST_STAGE + 1)-th whose leaves are dear —
# a z3 model, evaluated per leaf through its own eval; a natively held GPU witness costs a
# copy per leaf — and the rest go in a second launch only if none of those holds (0: one
# launch for all).  Measured (profiles/r05x_quick_sat_stages.md): a cache of GPU witnesses
# in one launch 0.98 -> 0.86 ms mean per query; z3-heavy caches keep the two stages.
# (Deciding only the newest model on the host first measured slower: it held for 24 of 121
# profile queries, profiles/r05g_quick_sat_hostfirst.jsonl.)
FIRST_STAGE = int(os.environ.get("PF_QS_FIRST_STAGE", "4"))


def first_stage_end(leaf_values: Sequence[Optional[LeafValues]], k: int) -> int:
    """End of the first launch's models: the longest prefix holding at most k models whose
    leaves are dear (everything but NativeLeafValues; an unvaluable model counts as dear —
    the reference statement decides it in its place)."""
    if k <= 0:
        return len(leaf_values)
    dear = 0
    for i, lv in enumerate(leaf_values):
        if not isinstance(lv, NativeLeafValues):
            dear += 1
            if dear > k:
                return i
    return len(leaf_values)


def choose(query: T.Term, leaf_values: Sequence[Optional[LeafValues]],
           reference: Callable[[int], bool], engine=None, first_stage: Optional[int] = None) -> Optional[int]:
    """Index (in the given most-recent-first order) of the first model under which ``query``
    is true, or None.  The models are evaluated in at most two launches: the newest up to the
    (``first_stage`` + 1)-th with dear leaves (FIRST_STAGE, ``first_stage_end``), then, if none
    of them holds, all the others.  A model whose
    ``leaf_values[i]`` is None, or that has a leaf its evaluator rejects, is decided by
    ``reference(i)`` — the reference statement — in its place in the order.  Raises
    LoweringError when the query cannot be lowered (the caller runs the reference loop)."""
    n = len(leaf_values)
    if n == 0 or query is T.FALSE:
        return None
    k1 = FIRST_STAGE if first_stage is None else first_stage
    t0 = time.perf_counter()
    phases: Dict[str, float] = {}

    def lap(name, t):
        now = time.perf_counter()
        phases[name] = phases.get(name, 0.0) + now - t
        return now

    if VERDICT_MEMO and CONJ_PROGRAMS and query is not T.TRUE:
        # conjunct by conjunct from the models' verdict memos: nothing is lowered unless some
        # (model, conjunct) pair goes to the engine
        if engine is None:
            from .engine import get_engine

            engine = get_engine()
        conjs = query_conjuncts(query)
        t = lap("lower", t0)
        choice, host, launches, on_engine_n = _choose_memo(conjs, leaf_values, reference, engine, k1, lap, t)
        _account(choice, host, launches, on_engine_n, phases)
        return choice
    if query is T.TRUE:
        leaves, program = [], None
    else:
        leaves, program = explicit_groups(query)
    t = lap("lower", t0)
    e1 = first_stage_end(leaf_values, k1)
    stages = [(0, e1), (e1, n)] if 0 < e1 < n else [(0, n)]
    if engine is None and program is not None:
        from .engine import get_engine

        engine = get_engine()
    choice, host, launches, on_engine_n, t = _stages(stages, leaves, program, leaf_values, reference,
                                                     engine, lap, t)
    _account(choice, host, launches, on_engine_n, phases)
    return choice


# Per-(model, conjunct) verdicts (CONJ_PROGRAMS): a cached model is immutable, so the truth
# of a conjunct under it is computed once and kept in the model's LeafValues; a query is then
# decided model by model, newest first, from the memo — a model with a false conjunct is out,
# one whose every conjunct is true is the answer — and only the unknown (model, conjunct) pairs
# of the models the walk reaches are evaluated.  LASER's queries along a path share all but
# their newest conjuncts, so after the first query of a path most of the work is one new
# conjunct under the few models the old conjuncts leave standing.  The unknown pairs of a
# batch of models go in one engine launch (only the programs of the unknown conjuncts, over
# only those models' rows); a batch of natively held GPU witnesses alone with at most
# HOST_VERDICT_PAIRS unknown pairs is evaluated by the native witness evaluator instead
# (csrc/pf_recheck.cpp: the interpretation Z3WitnessView.eval applies, natively) — for a few
# pairs the launch's fixed cost dominates.  PF_QS_MEMO=0 restores the all-models launches;
# PF_QS_HOST_PAIRS=0 sends every batch to the engine.
VERDICT_MEMO = os.environ.get("PF_QS_MEMO", "1") != "0"
HOST_VERDICT_PAIRS = int(os.environ.get("PF_QS_HOST_PAIRS", "256"))


# a model's verdict memo is cleared past this many conjuncts (a long analysis poses tens of
# thousands; the verdicts are recomputable, the memory of 100 models x all of them is not)
VERDICTS_MAX = 1 << 14


def _memo_status(lv: Optional[LeafValues], conjs: Sequence[T.Term]) -> Optional[bool]:
    """False if a conjunct is known false under the model, True if every one is known true,
    else None (some unknown)."""
    if lv is None:
        return None
    vd = lv.verdicts
    unknown = False
    for c in conjs:
        v = vd.get(c)
        if v is None:
            unknown = True
        elif not v:
            return False
    return None if unknown else True


def eval_rows_each(group: ExplicitGroups, rows, n_leaves: int, engine) -> np.ndarray:
    """SAT flags [program][model] of a group's programs over explicit model rows (one
    pf_eval_programs launch)."""
    soa = soa_of(rows, n_leaves)[group.gather] if n_leaves else soa_of(rows, 0)
    if hasattr(engine, "eval_programs"):
        return engine.eval_programs(group.pack(), soa)
    n = soa.shape[-1]
    out = np.ones((len(group.programs), n), dtype=bool)
    for k, (prog, (lo, hi)) in enumerate(zip(group.programs, group.spans())):
        out[k] = _eval_one(prog, np.ascontiguousarray(soa[lo:hi]) if hi > lo else soa_of(rows, 0)[:, :, :n], engine)
    return out


_QCONJ: "OrderedDict[T.Term, List[T.Term]]" = OrderedDict()
_SUBGROUPS: "OrderedDict[Tuple[T.Term, ...], object]" = OrderedDict()


def query_conjuncts(query: T.Term) -> List[T.Term]:
    """The query's flattened, de-duplicated conjuncts (explicit_groups' split), cached."""
    with _PROG_LOCK:
        hit = _QCONJ.get(query)
        if hit is not None:
            _QCONJ.move_to_end(query)
            return hit
    if query.op == "and":
        conj = [c for c in dict.fromkeys(flat_conjuncts(list(query.args))) if c is not T.TRUE]
    else:
        conj = [query]
    with _PROG_LOCK:
        _QCONJ[query] = conj
        while len(_QCONJ) > _PROGRAMS_MAX:
            _QCONJ.popitem(last=False)
    return conj


def conjunct_group(conjs: Sequence[T.Term]) -> Tuple[List[T.Term], ExplicitGroups]:
    """(leaf terms, group) of one program per conjunct, run side by side (cached by the
    conjunct tuple); raises LoweringError if a conjunct cannot be lowered."""
    key = tuple(conjs)
    with _PROG_LOCK:
        hit = _SUBGROUPS.get(key)
        if hit is not None:
            _SUBGROUPS.move_to_end(key)
            return hit
    lowered = [_conj_program(c) for c in conjs]
    pos: Dict[T.Term, int] = {}
    gather, offsets = [], []
    for vt, prog in lowered:
        if len(vt) != n_vars(prog):
            raise LoweringError("explicit group: variables and leaves differ")
        offsets.append(len(gather))
        for t in vt:
            gather.append(pos.setdefault(t, len(pos)))
    hit = (list(pos), ExplicitGroups([p for _, p in lowered], np.array(gather, dtype=np.int64), offsets, list(conjs)))
    with _PROG_LOCK:
        _SUBGROUPS[key] = hit
        while len(_SUBGROUPS) > _PROGRAMS_MAX:
            _SUBGROUPS.popitem(last=False)
    return hit


def _resolve(batch: List[int], conjs: Sequence[T.Term], leaf_values, engine, noval: set) -> Tuple[int, int]:
    """Compute the unknown conjunct verdicts of the models ``batch`` into their memos;
    (launches, models on the engine).  A model whose leaves cannot be valued goes to
    ``noval`` (the reference statement decides it)."""
    todo: Dict[int, List[int]] = {}
    for j in batch:
        vd = leaf_values[j].verdicts
        ks = [k for k, c in enumerate(conjs) if c not in vd]
        if ks:
            todo[j] = ks
    if not todo:
        return 0, 0
    for j in todo:
        if len(leaf_values[j].verdicts) > VERDICTS_MAX:
            leaf_values[j].verdicts.clear()
            todo[j] = list(range(len(conjs)))
    t_r = time.perf_counter()

    def sub_phase(name):
        nonlocal t_r
        now = time.perf_counter()
        with _STATS_LOCK:
            STATS.phase_s[name] = STATS.phase_s.get(name, 0.0) + now - t_r
        t_r = now

    natives = [j for j in todo if isinstance(leaf_values[j], NativeLeafValues)]
    # only a batch of natives alone: with dear models in it the launch is made anyway, and
    # the witnesses ride in it (measured, profiles/r06_quick_sat.md: the mixed cache's
    # slowest query 23 ms that way against 77-88 ms with the witnesses taken natively first)
    if natives and len(natives) == len(todo) and HOST_VERDICT_PAIRS > 0:
        ks = sorted({k for j in natives for k in todo[j]})
        if len(natives) * len(ks) <= HOST_VERDICT_PAIRS:
            from .smt import native_terms

            groups: Dict[Tuple[int, int], List[int]] = {}
            for j in natives:
                lv = leaf_values[j]
                groups.setdefault((id(lv.native.st), id(lv.reg)), []).append(j)
            terms = [conjs[k] for k in ks]
            n_done = 0
            for js in groups.values():
                lvs = [leaf_values[j] for j in js]
                vals, ok = native_terms.witness_values_many([lv.native for lv in lvs], terms, lvs[0].reg,
                                                            min(LEAF_THREADS, len(lvs)))
                for m, j in enumerate(js):
                    vd = leaf_values[j].verdicts
                    for q, k in enumerate(ks):
                        if ok[m, q]:
                            vd[conjs[k]] = bool(vals[m, q, 0] & 1)
                            n_done += 1
                    todo[j] = [k for k in todo[j] if conjs[k] not in vd]
                    if not todo[j]:
                        del todo[j]
            with _STATS_LOCK:
                STATS.verdicts_native += n_done
            sub_phase("eval.native_verdicts")
    if not todo:
        return 0, 0
    js = list(todo)
    ks = sorted({k for j in js for k in todo[j]})
    sub_leaves, sub = conjunct_group([conjs[k] for k in ks])
    nat = native_rows([leaf_values[j] for j in js], sub_leaves)
    block = getattr(nat, "block", None)
    if block is not None:
        rows, on = block, js
    else:
        rows, on = [], []
        for m, j in enumerate(js):
            r = nat[m] if m in nat else leaf_values[j].row(sub_leaves)
            if r is None:
                noval.add(j)
                continue
            rows.append(r)
            on.append(j)
    sub_phase("eval.rows")
    if not on:
        return 0, 0
    flags = eval_rows_each(sub, rows, len(sub_leaves), engine)
    sub_phase("eval.engine")
    for m, j in enumerate(on):
        vd = leaf_values[j].verdicts
        for q, k in enumerate(ks):
            vd[conjs[k]] = bool(flags[q, m])
    with _STATS_LOCK:
        STATS.verdicts_engine += len(on) * len(ks)
    return 1, len(on)


def _choose_memo(conjs: Sequence[T.Term], leaf_values, reference, engine, k1, lap, t):
    """choose() over the per-(model, conjunct) memo: (choice, host, launches, models on the
    engine).  Models are walked newest first; an undecided model and the next ones up to the
    (k + 1)-th with dear leaves are resolved as one batch — k = k1 the first time, four times
    as many each time after (natively held witnesses ride along), so a deep answer costs a
    few launches and at most ~4x the dear models the reference loop would evaluate — and the
    answer is the reference loop's: the first model in the order that holds."""
    n = len(leaf_values)
    host = launches = on_engine_n = 0
    noval: set = set()
    memo_hits = 0
    kk = k1
    i = 0
    choice = None
    while i < n:
        lv = leaf_values[i]
        st = _memo_status(lv, conjs) if i not in noval else None
        if st is False:
            memo_hits += 1
            i += 1
            continue
        if st is True:
            memo_hits += 1
            choice = i
            break
        if lv is None or i in noval:   # unvaluable: the reference statement, in its place
            host += 1
            if reference(i):
                choice = i
                break
            i += 1
            continue
        rest = leaf_values[i:]
        end = i + first_stage_end(rest, kk)
        kk *= 4
        batch = [j for j in range(i, max(end, i + 1))
                 if leaf_values[j] is not None and j not in noval and _memo_status(leaf_values[j], conjs) is None]
        t = lap("leaves", t)
        nl, ne = _resolve(batch, conjs, leaf_values, engine, noval)
        launches += nl
        on_engine_n += ne
        t = lap("eval", t)
    lap("host", t)
    with _STATS_LOCK:
        STATS.verdicts_memo += memo_hits
    return choice, host, launches, on_engine_n


def _account(choice, host, launches, on_engine_n, phases) -> None:
    with _STATS_LOCK:
        STATS.queries += 1
        STATS.hits += choice is not None
        STATS.engine_calls += launches
        STATS.models_engine += on_engine_n
        STATS.models_host += host
        for k, v in phases.items():
            STATS.phase_s[k] = STATS.phase_s.get(k, 0.0) + v


def _stages(stages, leaves, program, leaf_values, reference, engine, lap, t):
    """choose()'s launches, newest models first."""
    choice = None
    host = launches = on_engine_n = 0
    for lo, hi in stages:
        nat = native_rows(leaf_values[lo:hi], leaves)
        block = getattr(nat, "block", None)
        if block is not None:
            rows, on_engine = None, list(range(lo, hi))
        else:
            rows = [nat[i - lo] if i - lo in nat else leaf_values[i].row(leaves) if leaf_values[i] is not None
                    else None for i in range(lo, hi)]
            on_engine = [i for i in range(lo, hi) if rows[i - lo] is not None]
        t = lap("leaves", t)
        flags: Dict[int, bool] = {}
        if on_engine:
            if program is None:          # literal True: every model satisfies it
                flags = {i: True for i in on_engine}
            else:
                sat = eval_rows(program, block if block is not None else [rows[i - lo] for i in on_engine],
                                engine)
                flags = dict(zip(on_engine, (bool(x) for x in sat)))
                launches += 1
                on_engine_n += len(on_engine)
        t = lap("eval", t)
        for i in range(lo, hi):
            if i in flags:
                if flags[i]:
                    choice = i
                    break
            else:
                host += 1
                if reference(i):
                    choice = i
                    break
        t = lap("host", t)
        if choice is not None:
            break
    return choice, host, launches, on_engine_n, t


# ---- the Mythril seam ---------------------------------------------------------------------

def z3_literal(z3, v) -> int:
    """An evaluated leaf as an int: a bit-vector numeral or a Bool literal."""
    if z3.is_bv_value(v):
        return v.as_long()
    if z3.is_true(v):
        return 1
    if z3.is_false(v):
        return 0
    raise ValueError(f"not a literal: {v}")


def internal_for(model, expression):
    """The internal model ``mythril.laser.smt.Model.eval`` would use for ``expression``
    (laser/smt/model.py:45-59): the first whose ``decls()`` holds the expression's
    declaration, else the last; None for an empty ``Model()`` (whose ``eval`` is None)."""
    raw = getattr(model, "raw", None)
    if not raw:
        return None
    if len(raw) == 1:
        return raw[0]
    d = expression.decl()
    for im in raw:
        if d in list(im.decls()):
            return im
    return raw[-1]


def leaf_evaluator(z3, internal):
    """Term -> int under one internal model: a GPU witness (integration.Z3WitnessView)
    through its own interpretation, anything else (a z3 ``ModelRef``) through ``eval`` of the
    leaf's z3 AST with completion on a private copy (completion adds interpretations to the
    model it runs on, which is why the reference deep-copies before every eval)."""
    w = getattr(getattr(internal, "internal", None), "w", None)
    if w is not None and hasattr(w, "leaf_value"):
        return w.leaf_value
    return _z3_leaf_evaluators(z3, internal)[0]


def _z3_leaf_evaluators(z3, internal):
    """(one leaf, several leaves) evaluators of a z3 model on one private deep copy.  The
    batched form evaluates ``Concat`` of the leaves (a Bool leaf as a 1-bit ``If``) with one
    ``eval(..., model_completion=True)`` and splits the value: one evaluation per model and
    query, as the reference's ``eval`` of the whole conjunction (support_utils.py:63), so
    shared subterms are evaluated once and completion happens inside one call."""
    from .z3_terms import converter

    conv = converter(z3)
    holder: list = []

    def copy_():
        if not holder:
            holder.append(deepcopy(internal))
        return holder[0]

    def ev(t: T.Term) -> int:
        return z3_literal(z3, copy_().eval(conv.ast_of(t), model_completion=True))

    def ev_many(ts: Sequence[T.Term]) -> List[int]:
        parts, widths = [], []
        for t in ts:
            a = conv.ast_of(t)
            if z3.is_bool(a):
                a = z3.If(a, z3.BitVecVal(1, 1), z3.BitVecVal(0, 1))
            parts.append(a)
            widths.append(a.size())
        v = copy_().eval(parts[0] if len(parts) == 1 else z3.Concat(*parts), model_completion=True)
        if not z3.is_bv_value(v):
            raise ValueError("batched leaf evaluation: not a numeral")
        x = v.as_long()
        out = [0] * len(ts)
        for i in range(len(ts) - 1, -1, -1):
            out[i] = x & ((1 << widths[i]) - 1)
            x >>= widths[i]
        return out

    return ev, ev_many


def leaf_values_of(z3, internal) -> LeafValues:
    """The LeafValues of one internal model: natively held for a GPU witness whose buckets
    were lowered natively (NativeLeafValues), else over ``leaf_evaluator``."""
    wm = getattr(internal, "internal", None)
    w = getattr(wm, "w", None)
    if w is None or not hasattr(w, "leaf_value"):
        ev, ev_many = _z3_leaf_evaluators(z3, internal)
        return LeafValues(ev, ev_many)
    ev = w.leaf_value
    parts, reg = getattr(wm, "parts", None), getattr(wm, "reg", None)
    if parts and reg is not None and NATIVE_LEAVES:
        from .smt import native_terms

        nw = native_terms.NativeWitness.build(parts, reg)
        if nw is not None:
            return NativeLeafValues(ev, nw, reg)
    return LeafValues(ev)


# PF_NATIVE_LEAVES=0 evaluates witness leaves in Python (interp.Witness.leaf_value) instead
NATIVE_LEAVES = os.environ.get("PF_NATIVE_LEAVES", "1") != "0"

_GPU_MODEL_CACHE = None


def gpu_model_cache_class():
    """The drop-in subclass of ``mythril.support.support_utils.ModelCache`` (needs Mythril's
    module, or the test stand-in); built once per binding."""
    global _GPU_MODEL_CACHE
    from mythril.support.support_utils import ModelCache

    if _GPU_MODEL_CACHE is not None and _GPU_MODEL_CACHE.__bases__[0] is ModelCache:
        return _GPU_MODEL_CACHE
    import functools

    import z3

    from .z3_terms import converter

    class GpuModelCache(ModelCache):
        """``ModelCache`` whose quick-sat evaluates every cached model in one engine call
        (module docstring); ``model_cache`` (the LRU) and ``put`` are the reference's own."""

        def __init__(self, previous=None):
            super().__init__()
            if previous is not None:   # keep the process's cached models and their order
                self.model_cache.lru_cache.update(previous.model_cache.lru_cache)
            self._leaves: Dict[Tuple[int, int], Tuple[object, LeafValues]] = {}
            self._lock = threading.Lock()

        def _leaf_values(self, model, constraints) -> Optional[LeafValues]:
            im = internal_for(model, constraints)
            if im is None:
                return None
            key = (id(model), id(im))
            ent = self._leaves.get(key)
            if ent is None or ent[0] is not im:
                ent = (im, leaf_values_of(z3, im))
                self._leaves[key] = ent
            return ent[1]

        def _prune(self) -> None:
            live = {id(m) for m in self.model_cache.lru_cache.keys()}
            if len(self._leaves) > 2 * max(len(live), 1):
                self._leaves = {k: v for k, v in self._leaves.items() if k[0] in live}

        def _reference_eval(self, model, constraints) -> bool:
            model_copy = deepcopy(model)
            return z3.is_true(model_copy.eval(constraints, model_completion=True))

        @functools.lru_cache(maxsize=2 ** 10)
        def check_quick_sat(self, constraints):
            models = list(reversed(self.model_cache.lru_cache.keys()))
            choice = None
            with self._lock:
                try:
                    query = converter(z3).term(constraints)
                    lvs = [self._leaf_values(m, constraints) for m in models]
                    choice = choose(query, lvs, lambda i: self._reference_eval(models[i], constraints))
                    self._prune()
                except LoweringError as e:
                    log.debug("quick-sat by the reference loop: %s", e)
                    with _STATS_LOCK:
                        STATS.reference_loops += 1
                    choice = next((i for i, m in enumerate(models) if self._reference_eval(m, constraints)),
                                  None)
            if choice is None:
                return False
            model = models[choice]
            self.model_cache.put(model, self.model_cache.get(model) + 1)
            return model

    _GPU_MODEL_CACHE = GpuModelCache
    return GpuModelCache


def install() -> None:
    """Rebind the funnel's ``model_cache`` (support/model.py:20, read at call time at :96 and
    :120) to a GpuModelCache holding the same models; also the class name the
    ``DelayConstraintStrategy`` instantiates (strategy/constraint_strategy.py:5,13)."""
    import sys

    import mythril.support.model as funnel

    cls = gpu_model_cache_class()
    if not isinstance(funnel.model_cache, cls):
        funnel.model_cache = cls(funnel.model_cache)
    strat = sys.modules.get("mythril.laser.ethereum.strategy.constraint_strategy")
    if strat is not None and getattr(strat, "ModelCache", None) is not None:
        strat.ModelCache = cls
