"""Batched GPU feasibility for constraint sets given as terms.

``check_sets`` is the batched form of the reference's objective-free query path: every set
(one LASER state's ``Constraints.get_all_constraints()``) is split into independence
buckets (mythril/laser/smt/solver/independence_solver.py:38-83, here
mythril_amd/smt/independence.py), every distinct bucket is lowered once, given a
constraint-directed hint model (mythril_amd/seed.py) and searched in ONE ``pf_check_batch``
launch; each witness is materialised into a model whose ``eval`` agrees bit for bit with
the kernel.  A set is SAT when all its buckets are; sets that cannot be lowered, or have a
bucket without a witness among the candidates, return ``None`` — the caller then asks z3,
unchanged.

Bucket witnesses are cached by bucket (terms are hash-consed, so a bucket is its tuple of
constraint terms): LASER's sets grow by appending constraints, so the tx-boundary and fork
queries of one analysis share most buckets — the GPU-resident counterpart of the
reference's ``ModelCache`` (support/support_utils.py:57-71), keyed by structure instead of
re-evaluating up to 100 models per query.
"""

from __future__ import annotations

import os
import threading
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import ir, seed
from ..lower import LoweringError, lower
from .independence import buckets
from .interp import Witness
from .model import WitnessModel
from . import terms as T
from .to_dag import DEFAULT_REGISTRY, Lowered, TermLowering, UFRegistry


@dataclass
class GpuConfig:
    budget: int = 65536          # candidates per bucket
    seed: int = 0x4D595448       # global candidate seed
    flags: int = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT
    timeout_ms: int = 0
    enabled: bool = True
    split: bool = True           # independence buckets
    hints: bool = True           # constraint-directed parent (hint) models
    # parent models for buckets new to a query: the newest witness / z3-model value of each
    # of the bucket's symbols and array reads (note_values / _note_witness) — a child state
    # is its parent's constraints plus one JUMPI condition (instructions.py:1638,1662), so
    # the parent's model is the natural candidate 0 (mutated by the generator's
    # neighbourhood candidates, include/pf_bytecode.h) for the one bucket the condition changes
    parents: bool = True
    recent_size: int = 1 << 14   # symbol values kept for parent models
    # terms in the native store before it is retired for a fresh one (a long analysis would
    # otherwise keep every term it ever posed): ~2M terms, a few hundred MB of host memory
    store_limit: int = 1 << 21
    cache_size: int = 1 << 16    # bucket witnesses kept
    # re-evaluate every constraint of a multi-bucket set under the union of its bucket
    # witnesses.  Off by default: each bucket witness is re-checked on exactly its bucket's
    # constraints, and buckets share no symbol, array or inverse-keccak family
    # (independence.py), so the union satisfies the set by construction; the tests switch
    # it on to check that construction (tests/test_discharge.py).
    recheck_union: bool = False
    # host lowering workers (spawned processes; terms re-intern on unpickling): used for a
    # call with at least `parallel_min` new buckets — the lowering is pure Python and was
    # 95 % of the corpus' wall time on one core
    workers: int = int(os.environ.get("PF_LOWER_WORKERS", "0")) or min(16, os.cpu_count() or 1)
    parallel_min: int = 48
    # candidate 0 of a long bucket program first as the bucket's conjuncts side by side: a
    # bucket whose program has at least this many instructions and whose every variable
    # carries a parent / hint value (so candidate 0 is known on the host) is evaluated at
    # that assignment by its cached per-conjunct explicit programs in one launch, a wave per
    # conjunct (model_cache, pf_eval_programs) — the search is a lone wave walking the whole
    # program, ~0.45 us per instruction.  A bucket that holds there skips the search; the
    # host re-check runs as for any witness.  0 turns it off.
    probe_min_ins: int = int(os.environ.get("PF_PROBE_SPLIT_MIN", "400"))
    # ... for calls of at most this many programs (a single query's buckets: latency); a
    # batch's search runs its long programs side by side anyway
    probe_max_progs: int = 4


CONFIG = GpuConfig()


@dataclass
class GpuStats:
    sets: int = 0            # sets offered to the GPU
    lowered: int = 0         # sets whose every bucket lowered to bytecode
    sat: int = 0             # sets discharged with a GPU witness
    buckets: int = 0         # distinct buckets searched on the GPU
    bucket_hits: int = 0     # buckets answered from the witness cache
    lowering_failures: Dict[str, int] = field(default_factory=dict)
    bucket_origin: Dict[str, int] = field(default_factory=dict)  # witness provenance per bucket
    recheck_failures: int = 0  # GPU witnesses the host re-check rejected (must stay 0)
    probe_split: int = 0       # long buckets whose candidate 0 went through the conjunct probe
    probe_split_sat: int = 0   # ... and held there (no search launch for them)
    kernel_ms: float = 0.0
    evals: int = 0
    host_s: float = 0.0      # lowering + hints + witness re-checks
    phase_s: Dict[str, float] = field(default_factory=dict)  # wall time per check_sets phase


STATS = GpuStats()
_lock = threading.Lock()
_CACHE: "OrderedDict[tuple, Tuple[Lowered, List[int]]]" = OrderedDict()
# buckets whose search found no witness, per search configuration: the search is a pure
# function of (program, seed, budget, flags), so repeating it cannot change the answer —
# LASER re-poses a parent's buckets at every fork below it (svm.py:351-358)
_NEG: "OrderedDict[tuple, None]" = OrderedDict()


# newest values of symbols (name -> value) and of base-array reads (array name ->
# {select term -> value}) over the accepted witnesses and noted z3 models: the parent models
_RECENT_VARS: "OrderedDict[str, int]" = OrderedDict()
_RECHECK_DEBUG: list = []   # the last few re-check failures (bucket, lowered, values, program, index)
_RECENT_READS: "OrderedDict[str, OrderedDict]" = OrderedDict()


def _host_threads(cfg: GpuConfig, n_jobs: int) -> int:
    """Host threads for a native batch call over ``n_jobs`` buckets: the library's persistent
    worker pool (csrc/pf_pool.h) for 8 or more; fewer run on the caller (measured on a single
    query's ~3.5 buckets: 0.55 ms of native lowering on one thread, 0.82 ms on four)."""
    return max(1, min(cfg.workers, n_jobs)) if n_jobs >= 8 else 1


def reset_cache() -> None:
    with _lock:
        _CACHE.clear()
        _NEG.clear()
        _RECENT_VARS.clear()
        _RECENT_READS.clear()
        if _native_batch():
            from . import native_terms

            native_terms.recent_clear()


def _neg_key(key: tuple, cfg: GpuConfig) -> tuple:
    # parents only seed candidate 0 of a bucket's first search; a bucket whose complete
    # search found nothing stays negative (as the reference's lru_cache'd check_quick_sat
    # keeps its negative answers, support_utils.py:59)
    return (key, cfg.budget, cfg.seed, cfg.flags, cfg.hints)


def note_values(vals: Dict[str, int], cfg: Optional[GpuConfig] = None) -> None:
    """Record symbol values (a z3 model's, integration._note_z3_model) for parent models."""
    cfg = cfg or CONFIG
    with _lock:
        for k, v in vals.items():
            _RECENT_VARS[k] = v
            _RECENT_VARS.move_to_end(k)
        while len(_RECENT_VARS) > cfg.recent_size:
            _RECENT_VARS.popitem(last=False)
        if _native_batch():
            from . import native_terms

            native_terms.note_vars(vals, cfg.recent_size)


def _note_witness(lo: Lowered, values: List[int], cfg: GpuConfig) -> None:
    """Record an accepted bucket witness's variable values (caller holds _lock)."""
    if getattr(lo, "res", None) is not None:
        # a native witness: the store's recent tables (pflt_note_result, the same updates)
        from . import native_terms

        native_terms.note_result(lo, values, cfg.recent_size)
        return
    for term, val in zip(lo.var_terms, values):
        if term.op in ("var", "bvar"):
            _RECENT_VARS[term.val] = val
            _RECENT_VARS.move_to_end(term.val)
        elif term.op == "select" and term.args[0].op == "array":
            name = term.args[0].val
            tab = _RECENT_READS.get(name)
            if tab is None:
                tab = _RECENT_READS[name] = OrderedDict()
            _RECENT_READS.move_to_end(name)
            tab[term] = val
            tab.move_to_end(term)
            while len(tab) > 256:
                tab.popitem(last=False)
    while len(_RECENT_VARS) > cfg.recent_size:
        _RECENT_VARS.popitem(last=False)
    while len(_RECENT_READS) > 1024:
        _RECENT_READS.popitem(last=False)


def _recent_parent(bucket: List[T.Term]) -> Optional[dict]:
    """Parent model of a bucket from the recent values of its symbols and array reads
    (keys: symbol names, and select terms — hash-consed, so the same read in a child
    query is the same key)."""
    from .independence import dependence_keys

    if _native_batch():
        from . import native_terms

        st = native_terms.batch_api()   # one store for the handle's whole life
        h = native_terms.recent_parent_handle(bucket, st)
        if h is None:
            return None
        try:
            return native_terms.parent_dict(h, st)
        finally:
            native_terms.free_parent(h, st)

    keys = set()
    for c in bucket:
        keys |= dependence_keys(c)
    out: dict = {}
    with _lock:
        for k in keys:
            if k.startswith("v:"):
                v = _RECENT_VARS.get(k[2:])
                if v is not None:
                    out[k[2:]] = v
            elif k.startswith("a:"):
                tab = _RECENT_READS.get(k[2:])
                if tab:
                    out.update(tab)
    return out or None


def _values(v) -> List[int]:
    """A witness's values as ints (the native pipeline keeps them as limb rows)."""
    if isinstance(v, np.ndarray):
        from . import native_terms

        return native_terms.ints_of(v)
    return v


def _union_thunk(parts, reg: UFRegistry):
    return lambda: Witness.union([Witness(lo, _values(v), reg) for lo, v in parts], reg)


def _set_seed(constraints: Sequence[T.Term]) -> int:
    # (h * 1000003) ^ hash over all conjuncts, mod 2^32: multiplication and xor only carry
    # upwards, so masking every step gives the unmasked chain's low 32 bits without the
    # big integer growing by ~20 bits per conjunct
    memo, h = T._SHASH, 0
    for c in constraints:
        v = memo.get(c)
        h = ((h * 1000003) ^ (v if v is not None else T.struct_hash(c))) & 0xFFFFFFFF
    return h


_NATIVE_TERMS = os.environ.get("PF_NATIVE_TERMS", "1") != "0"


def _witness_limbs(eng, db, mine: List[int], base: int, progs, found, seed_: int) -> np.ndarray:
    """The witnesses' variables as limb rows, in ``mine`` order.  When every witness of the
    batch is candidate 0 of a program whose variables all carry parent values (a single
    query whose hint model holds), those values are the rows (the generator keeps them at
    candidate 0: native_terms.candidate0_limbs) and no materialise launch is made; otherwise
    one launch materialises them all."""
    from . import native_terms

    if all(int(found[k]) == 0 for k in mine):
        parts = []
        for k in mine:
            rows = native_terms.candidate0_limbs(progs[k])
            if rows is None:
                break
            parts.append(rows)
        else:
            return np.concatenate(parts) if parts else np.zeros((0, 8), dtype=np.uint32)
    return eng.materialize_limbs(db, [k - base for k in mine], [int(found[k]) for k in mine], seed=seed_)


def _probe_candidate0(eng, progs, lows, keys, reg, cfg) -> Dict[int, np.ndarray]:
    """{program index: candidate-0 limb rows} for the long programs whose every variable
    carries a parent value and whose bucket holds at that assignment — decided on the device
    by the bucket's per-conjunct explicit programs (mythril_amd/model_cache.py, cached across
    queries) in one pf_eval_programs launch, the leaves valued by the native witness
    interpretation of the assignment (the one the host re-check uses).  A bucket whose
    explicit form is out of reach (lowering, a leaf the native evaluator declines, an engine
    without pf_eval_programs) is left to the search."""
    from .. import model_cache as MC
    from . import native_terms

    if not hasattr(eng, "eval_programs"):
        return {}
    out: Dict[int, np.ndarray] = {}
    for k, prog in enumerate(progs):
        r = getattr(prog, "native_result", None)
        if r is None or int(r.info[6]) < cfg.probe_min_ins:
            continue
        # only where the host's hint solver left every (distinct) root true under its model
        # (info[13] n_sat): a probe that fails costs its launch on top of the search (the
        # hint is a guess; the device decides)
        n_roots = int(r.info[10])
        if n_roots == 0 or int(r.info[13]) < len(set(r.get(native_terms.GET_ROOTS, n_roots, 1).tolist())):
            continue
        rows = native_terms.candidate0_limbs(prog)
        if rows is None:
            continue
        cs = [c for c in keys[k][0] if c is not T.TRUE]
        if not cs:
            continue
        try:
            leaves, program = MC.explicit_groups(T.and_(*cs) if len(cs) > 1 else cs[0])
        except LoweringError:
            continue
        nw = native_terms.NativeWitness.build([(lows[k], rows)], reg)
        if nw is None:
            continue
        if leaves:
            vals, ok = native_terms.witness_values_many([nw], list(leaves), reg, 1)
            if not ok.all():
                continue
            block = vals
        else:
            block = np.zeros((1, 0, 8), dtype=np.uint32)
        sat = MC.eval_rows(program, block if leaves else [b""], eng)
        with _lock:
            STATS.probe_split += 1
        if bool(sat[0]):
            out[k] = rows
            with _lock:
                STATS.probe_split_sat += 1
    return out


def _long_hint_miss(prog, min_ins: int) -> bool:
    """A native program of at least ``min_ins`` instructions (min_ins > 0) with variables whose
    host hint model (candidate 0) satisfies fewer roots than the DAG has.  info[13] n_sat
    counts the distinct roots the host evaluator finds true (a UF application it cannot
    evaluate reads as false) against info[10], all of them: a short program's "miss" may be
    no miss, and its probe walk is cheap anyway."""
    r = getattr(prog, "native_result", None)
    return (r is not None and 0 < min_ins <= int(r.info[6]) and int(r.info[0]) > 0
            and int(r.info[13]) < int(r.info[10]))


def _native_batch() -> bool:
    """check_sets' native pipeline (libpflower.so batch entry points): buckets lowered on
    host threads, packed, re-checked and recorded in C++ — no Python term decoding."""
    if not _NATIVE_TERMS:
        return False
    from . import native_terms

    return native_terms.batch_api() is not None


def _lower_bucket(bucket: List[T.Term], reg: UFRegistry, parent: Optional[dict], hints: bool):
    """Terms -> (witness metadata, program): natively in libpflower.so when it is built
    (smt/native_terms.py, the same program node for node), else the Python reference
    (to_dag.TermLowering -> seed.apply_hints -> lower.lower)."""
    if _NATIVE_TERMS:
        from . import native_terms

        if native_terms.store() is not None:
            return native_terms.lower_bucket(bucket, reg, parent, hints, _set_seed(bucket))
    tl = TermLowering(reg, parent)
    lo = tl.lower(bucket)
    if hints:
        seed.apply_hints(lo.dag)
    return lo, lower(lo.dag, seed=_set_seed(bucket))


def _origin(idx: int, prog, hinted: bool, parented: bool) -> str:
    """Provenance of a bucket witness: "search" = a later GPU candidate; candidate 0 is the
    host hint model ("hint"), the parent model ("parent") or the generator's first
    candidate ("first")."""
    if idx > 0:
        return "search"
    if prog.has_parent:
        return "hint" if hinted else ("parent" if parented else "first")
    return "first"


def _lower_chunk(job):
    """Worker: lower a chunk of buckets; the DAG stays behind (witnesses need only the
    variable / UF / array-read terms)."""
    items, reg, hints = job
    out = []
    for bucket, parent in items:
        try:
            lo, prog = _lower_bucket(bucket, reg, parent, hints)
            out.append((Lowered(None, lo.var_terms, lo.uf_apps, lo.array_reads), prog, None))
            lo = None
        except (LoweringError, ValueError, OverflowError, RecursionError) as e:
            # one bucket the lowering cannot take (or whose native emission fails; or, on the
            # Python lowering, a term nested past the recursion limit) is that bucket's
            # failure only: the rest of the batch is still searched
            out.append((None, None, f"{type(e).__name__}: {e}" if not isinstance(e, LoweringError) else str(e)))
    return out


_POOL = None
_POOL_N = 0


def _pool(n: int):
    global _POOL, _POOL_N
    if _POOL is None or _POOL_N != n:
        import multiprocessing as mp

        if _POOL is not None:
            _POOL.terminate()
        # spawn, never fork: the parent may hold an initialised HIP runtime
        _POOL = mp.get_context("spawn").Pool(n)
        _POOL_N = n
        import atexit

        atexit.register(_shutdown_pool)
    return _POOL


def _warm(_):
    from . import to_dag  # noqa: F401  (the worker's imports, paid once)

    return 0


def warm_pool(cfg: Optional[GpuConfig] = None) -> int:
    """Start the lowering workers now (a long-lived analysis pays their spawn once; a
    latency-sensitive caller can do it up front).  Returns the worker count."""
    cfg = cfg or CONFIG
    n = max(1, cfg.workers)
    if n > 1 and not _native_batch():   # the native pipeline lowers on host threads instead
        _pool(n).map(_warm, range(n), chunksize=1)
    return n


def _shutdown_pool() -> None:
    global _POOL
    if _POOL is not None:
        _POOL.terminate()
        _POOL.join()
        _POOL = None


def _lower_all(jobs, reg: UFRegistry, cfg: GpuConfig):
    """[(bucket, parent)] -> [(Lowered | None, Program | None, error | None)], in order."""
    n = min(cfg.workers, len(jobs))
    if n <= 1 or len(jobs) < cfg.parallel_min:
        return _lower_chunk((jobs, reg, cfg.hints))
    per = max(1, (len(jobs) + 4 * n - 1) // (4 * n))
    chunks = [(jobs[i:i + per], reg, cfg.hints) for i in range(0, len(jobs), per)]
    out = []
    for part in _pool(n).map(_lower_chunk, chunks):
        out.extend(part)
    return out


def check_sets(sets: Sequence[Sequence[T.Term]], registry: Optional[UFRegistry] = None,
               parents: Optional[Sequence[Optional[dict]]] = None,
               config: Optional[GpuConfig] = None) -> List[Optional[WitnessModel]]:
    import time

    from ..engine import get_engine  # the GPU is required from here on: no host fallback

    cfg = config or CONFIG
    reg = registry or DEFAULT_REGISTRY
    t0 = time.perf_counter()
    out: List[Optional[WitnessModel]] = [None] * len(sets)
    set_buckets: List[Optional[List[tuple]]] = []
    found: Dict[tuple, Optional[Tuple[Lowered, List[int]]]] = {}   # bucket key -> witness
    todo: Dict[tuple, int] = {}                                     # bucket key -> program idx
    progs, lows, keys = [], [], []
    origin: Dict[tuple, str] = {}   # bucket key -> "hint" / "search" (this call's searches)
    n_lowered = hits = 0
    # the keccak interpretation depends on the registry (intervals, concrete hashes): a
    # cached witness is only valid for the registry state it was found under
    reg_sig = tuple(sorted((n, s.lo, len(s.concrete)) for n, s in reg.keccak.items()))
    jobs, job_keys, pending = [], [], set()
    nat = _native_batch()
    st = None
    if nat:
        from . import native_terms

        if native_terms.new_generation(cfg.store_limit):
            reset_cache()   # cached witnesses hold results of the retired store
        # this call's store, pinned: another thread's check_sets may retire the process's
        # store (new_generation) while this one holds parent handles whose read keys are
        # this store's term ids — every handle is made, lowered against and freed here
        st = native_terms.batch_api()
    phases: Dict[str, float] = {}
    tp = [t0]

    def lap(name):
        now = time.perf_counter()
        phases[name] = phases.get(name, 0.0) + now - tp[0]
        tp[0] = now

    csets = [[c for c in cs if c is not T.TRUE] for cs in sets]
    pre_bks: Dict[int, list] = {}
    if cfg.split and _NATIVE_TERMS and len(csets) > 1:
        # a batch's queries bucketed in one native call (pflt_buckets_many)
        from . import native_terms

        live = [i for i, cs in enumerate(csets) if not any(c is T.FALSE for c in cs)]
        many = native_terms.buckets_many([csets[i] for i in live]) if live else None
        if many is not None:
            pre_bks = dict(zip(live, many))
    for i, cs in enumerate(csets):
        if any(c is T.FALSE for c in cs):
            set_buckets.append(None)
            continue
        parent = parents[i] if parents else None
        bks = pre_bks.get(i)
        if bks is None and cfg.split and _NATIVE_TERMS:
            from . import native_terms

            bks = native_terms.buckets(cs)      # the same partition (pflt_buckets)
        if bks is None:
            bks = buckets(cs) if cfg.split else [cs]
        ks = []
        for b in bks:
            # a witness answers its bucket whatever parent model seeded the search
            key = (tuple(b), reg_sig)
            ks.append(key)
            if key in found or key in pending:
                continue
            cached = _CACHE.get(key)
            if cached is not None:
                found[key] = cached
                hits += 1
                if cfg.parents:
                    with _lock:
                        _note_witness(cached[0], cached[1], cfg)
                continue
            if _neg_key(key, cfg) in _NEG:  # a complete search found nothing: same answer
                found[key] = None
                hits += 1
                continue
            pending.add(key)
            if nat:
                # parent handles: the caller's model, or the store's recent values now (cache
                # hits above recorded theirs first, as _note_witness does)
                if parent is not None:
                    with st.lock:
                        bp = (native_terms._parent_handle(st, parent), bool(parent))
                elif cfg.parents:
                    h = native_terms.recent_parent_handle(b, st)
                    bp = (h, h is not None)
                else:
                    bp = (None, False)
            else:
                bp = parent if parent is not None else (_recent_parent(b) if cfg.parents else None)
            jobs.append((b, bp))
            job_keys.append(key)
        set_buckets.append(ks)
    lap("bucket")
    failed = set()
    parented: List[bool] = []
    if nat:
        job_parent = {k: j[1][1] for k, j in zip(job_keys, jobs)}
        try:
            lowered_all = native_terms.lower_many(
                [(b, h) for b, (h, _) in jobs], reg, cfg.hints, [_set_seed(b) for b, _ in jobs],
                _host_threads(cfg, len(jobs)), st=st)
        finally:
            for _, (h, _) in jobs:
                native_terms.free_parent(h, st)
    else:
        job_parent = {k: bool(j[1]) for k, j in zip(job_keys, jobs)}
        lowered_all = _lower_all(jobs, reg, cfg)
    lap("lower")
    for key, (lo, prog, err) in zip(job_keys, lowered_all):
        if err is not None:
            err = err.split(":")[0][:60]
            with _lock:
                STATS.lowering_failures[err] = STATS.lowering_failures.get(err, 0) + 1
            found[key] = None
            failed.add(key)
            continue
        todo[key] = len(progs)
        progs.append(prog)
        lows.append(lo)
        keys.append(key)
        parented.append(job_parent[key])
    for ks in set_buckets:
        if ks is not None and not any(k in failed or (k in found and found[k] is None) for k in ks):
            n_lowered += 1

    res = None
    if progs:
        eng = get_engine()
        # long hinted buckets: candidate 0 by their conjuncts side by side first
        pre: Dict[int, np.ndarray] = {}
        if nat and 0 < cfg.probe_min_ins and len(progs) <= cfg.probe_max_progs and any(
                int(getattr(getattr(p, "native_result", None), "info", [0] * 7)[6]) >= cfg.probe_min_ins
                for p in progs):
            pre = _probe_candidate0(eng, progs, lows, keys, reg, cfg)
            lap("probe")
        search = [k for k in range(len(progs)) if k not in pre]
        found_all = np.full(len(progs), 0xFFFFFFFF, dtype=np.uint32)
        for k in pre:
            found_all[k] = 0
        timed_out = False
        vals_of = {}
        limb_rows = []   # native: the witnesses' variables as limbs, in `sat` order
        if search:
            sprogs = [progs[k] for k in search]
            # one batch per device of the engine (cost-balanced shards), searched concurrently
            dbs = eng.upload_sharded(sprogs) if hasattr(eng, "upload_sharded") else [eng.upload(sprogs)]
            lap("upload")
            flags = cfg.flags
            if nat and cfg.hints and any(_long_hint_miss(p, cfg.probe_min_ins) for p in sprogs):
                # the device's candidate-0 probe launch would walk that long program once in
                # vain before the search walks it again
                flags |= ir.FLAG_NO_PROBE
            if len(dbs) == 1:
                res = eng.check(dbs[0], budget=cfg.budget, seed=cfg.seed, flags=flags,
                                timeout_ms=cfg.timeout_ms)
            else:
                res = eng.check_many(dbs, budget=cfg.budget, seed=cfg.seed, flags=flags,
                                     timeout_ms=cfg.timeout_ms)
            timed_out = bool(res.timed_out)
            lap("search")
            for i, k in enumerate(search):
                found_all[k] = res.found[i]
            ssat = [i for i in range(len(search)) if res.found[i] != 0xFFFFFFFF]
            base = 0
            for db in dbs:
                mine = [i for i in ssat if base <= i < base + len(db)]
                if mine:
                    sids, cids = [i - base for i in mine], [int(res.found[i]) for i in mine]
                    if nat:
                        if hasattr(eng, "materialize_limbs"):
                            rows = _witness_limbs(eng, db, mine, base, sprogs, res.found, cfg.seed)
                        else:
                            rows = ir.limbs_array([x for vs in eng.materialize(db, sids, cids, seed=cfg.seed)
                                                   for x in vs])
                        o = 0
                        for i in mine:
                            nv = int(db.batch.descs[i - base][5])
                            vals_of[search[i]] = rows[o:o + nv]
                            o += nv
                    else:
                        got = eng.materialize(db, sids, cids, seed=cfg.seed)
                        vals_of.update(zip([search[i] for i in mine], got))
                base += len(db)
                db.free()
        vals_of.update(pre)
        sat = [k for k in range(len(progs)) if found_all[k] != 0xFFFFFFFF]
        vals = [vals_of[k] for k in sat]
        if nat:
            limb_rows = [np.asarray(v, dtype=np.uint32).reshape(-1, 8) for v in vals]
        lap("materialize")
        status = None
        if nat and sat:
            # the host re-check of every witness at once, on host threads (pflt_recheck_many)
            status = native_terms.recheck_many([lows[k] for k in sat], np.concatenate(limb_rows), reg,
                                               _host_threads(cfg, len(sat)))
        for k in range(len(progs)):
            found[keys[k]] = None
        if not timed_out:  # a deadline-cut search is not a complete answer
            sat_set = set(sat)
            with _lock:
                for k in range(len(progs)):
                    if k not in sat_set:
                        _NEG[_neg_key(keys[k], cfg)] = None
                while len(_NEG) > cfg.cache_size:
                    _NEG.popitem(last=False)
        for j, (k, v) in enumerate(zip(sat, vals)):
            key = keys[k]
            # provenance of the witness: candidate 0 of a hinted program is the host's
            # constraint-directed hint model itself; any other index was found by the search
            idx = int(found_all[k])
            origin[key] = _origin(idx, progs[k], cfg.hints, parented[k])
            # re-check on the host under the same interpretation before trusting it:
            # natively (pflt_recheck, the Witness interpretation bit for bit) when built
            ok = None
            if status is not None:
                st_j = int(status[j])
                ok = None if st_j < 0 else bool(st_j)
                if ok is None:
                    v = native_terms.ints_of(v)
            elif _NATIVE_TERMS:
                from . import native_terms

                ok = native_terms.recheck(list(key[0]), lows[k], v, reg)
            if ok is None:
                w = Witness(lows[k], v, reg)
                ok = all(w.ev(c) for c in key[0])
            if not ok:
                # the program disagrees with the terms under this assignment: a lowering
                # or interpretation bug — sound (the bucket stays unanswered), but counted
                with _lock:
                    STATS.recheck_failures += 1
                    prog = progs[k].decode() if hasattr(progs[k], "decode") else progs[k]
                    _RECHECK_DEBUG.append((key[0], lows[k], v, prog, int(found_all[k])))
                    del _RECHECK_DEBUG[:-8]
            else:
                found[key] = (lows[k], v)
                with _lock:
                    _CACHE[key] = (lows[k], v)
                    while len(_CACHE) > cfg.cache_size:
                        _CACHE.popitem(last=False)
                    _note_witness(lows[k], v, cfg)
        if nat:   # programs are uploaded: keep only the witness metadata
            native_terms.shrink_many(lows)
        lap("recheck")

    n_sat = 0
    for i, ks in enumerate(set_buckets):
        if ks is None:
            continue
        parts = [found.get(k) for k in ks]
        if any(p is None for p in parts):
            continue
        cs = [c for c in sets[i] if c is not T.TRUE]
        # buckets() partitions every conjunct of the set: each bucket's witness was
        # re-checked on exactly its conjuncts above (or when it entered the cache), so the
        # model's interpretation is only built when it is first read
        w = _union_thunk(parts, reg)
        ok = True
        if cfg.recheck_union and len(parts) > 1:
            w = w()
            ok = all(w.ev(c) for c in cs)
        if ok:
            out[i] = WitnessModel(w, list(sets[i]))
            out[i].parts, out[i].reg = parts, reg    # the native witness's ingredients (model_cache)
            # per bucket: _origin(); the set takes the strongest of its buckets: "search" if
            # some bucket needed a later candidate, else "hint" / "parent" / "first" if such a
            # candidate 0 answered some bucket, else "cache"
            kinds = {origin.get(k, "cache") for k in ks}
            out[i].origin = next((c for c in ("search", "hint", "parent", "first") if c in kinds), "cache")
            n_sat += 1
    lap("models")
    with _lock:
        for name, v in phases.items():
            STATS.phase_s[name] = STATS.phase_s.get(name, 0.0) + v
        for o in origin.values():
            STATS.bucket_origin[o] = STATS.bucket_origin.get(o, 0) + 1
        STATS.sets += len(sets)
        STATS.lowered += n_lowered
        STATS.sat += n_sat
        STATS.buckets += len(progs)
        STATS.bucket_hits += hits
        if res is not None:
            STATS.kernel_ms += res.kernel_ms
            STATS.evals += res.cands_decided
        STATS.host_s += time.perf_counter() - t0 - (res.kernel_ms / 1e3 if res is not None else 0.0)
    return out
