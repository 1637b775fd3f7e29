"""A quick-sat workload in a Mythril-shaped process: up to 100 cached models — GPU witnesses
(integration.Z3WitnessView) and z3-shaped models (fake_z3.ModelRef, explicit
interpretations) — and a stream of LASER-shaped queries as ``simplify(And(*cs)).raw``
z3 expressions (support/model.py:96).  Used by tests/test_model_cache.py (the GPU-resident
ModelCache against the reference loop) and by bench.py's quick-sat leg.

Test infrastructure only (needs tests/fake_z3.py and tests/mythril_standin.py).
"""

from __future__ import annotations

import random
from typing import List, Tuple

from mythril_amd import corpus as C
from mythril_amd import integration
from mythril_amd.smt import gpu_check, z3_bridge
from mythril_amd.smt import terms as T


def to_z3(z3, terms: List[T.Term]):
    """Engine terms -> z3 ASTs (smt/z3_bridge.Converter, pointed at the given z3 module)."""
    saved = z3_bridge.z3
    z3_bridge.z3 = z3
    try:
        conv = z3_bridge.Converter()
        return [conv(t) for t in terms]
    finally:
        z3_bridge.z3 = saved


def _symbols(cs: List[T.Term]):
    seen, out, stack = set(), [], list(cs)
    while stack:
        t = stack.pop()
        if t in seen:
            continue
        seen.add(t)
        if t.op in ("var", "bvar", "array", "apply"):
            out.append(t)
        stack.extend(t.args)
    return out


def z3_model_of(z3, query: C.Query, registry, rng: random.Random, perturb: bool):
    """A z3-shaped model interpreting the query's symbols as its planted model does (arrays
    as tables with a random else value, every UF application's value as an entry of the
    function's table) — optionally with one scalar nudged, which usually breaks it."""
    ev = C._PlantedEval(query.planted, registry)
    interp = {}
    funcs = {}
    scalars = []
    for s in _symbols(query.constraints):
        if s.op == "var":
            interp[z3.BitVec(s.val, s.width).decl()] = int(ev.ev(s))
            scalars.append(z3.BitVec(s.val, s.width).decl())
        elif s.op == "bvar":
            interp[z3.Bool(s.val).decl()] = bool(ev.ev(s))
        elif s.op == "array":
            tab = dict(query.planted.arrays.get(s.val, {}))
            d = z3.Array(s.val, z3.BitVecSort(s.sort[1]), z3.BitVecSort(s.sort[2])).decl()
            interp[d] = (tab, 0 if s.val != "balance" else rng.randrange(1 << 64))
        else:
            name, doms = s.val
            f = z3.Function(name, *[z3.BitVecSort(w) for w in doms], z3.BitVecSort(s.width))
            ent = funcs.setdefault(f, ({}, rng.randrange(1 << min(s.width, 64))))
            try:
                ent[0][tuple(int(ev.ev(a)) for a in s.args)] = int(ev.ev(s))
            except Exception:  # noqa: BLE001 - an application the planted model cannot value
                pass
    interp.update(funcs)
    if perturb and scalars:
        d = rng.choice(scalars)
        interp[d] = (interp[d] + 1) % (1 << d.range().size())
    return z3.ModelRef(interp)


def build(z3, ns, n_models: int = 100, n_scenarios: int = 8, seed: int = 7,
          n_queries: int = 60, gpu_frac: float = 0.4, empty_frac: float = 0.1) -> Tuple[list, list, list, object]:
    """(models most recent LAST, in ``put`` order; query ASTs; the corpus queries; the
    corpus's keccak registry).

    The models (default mix): 40 % GPU witnesses of corpus queries (searched through the
    current engine), 10 % empty ``Model()``s, the rest z3-shaped models (half of them
    perturbed).  The
    queries: corpus queries in issue order plus a contradiction no model satisfies."""
    rng = random.Random(seed)
    corp = C.build(n_scenarios=n_scenarios, txs=2, seed=seed)
    reg = corp.kfm.registry
    sat_qs = [q for q in corp.queries if q.label == "sat"]
    n_gpu = int(gpu_frac * n_models)
    n_empty = int(empty_frac * n_models)
    picks = [sat_qs[i % len(sat_qs)] for i in rng.sample(range(len(sat_qs)), min(len(sat_qs), n_gpu))]
    witnesses = gpu_check.check_sets([q.constraints for q in picks], registry=reg)
    models = [ns.Model([integration.Z3WitnessView(w)]) for w in witnesses if w is not None]
    n_z3 = max(0, n_models - len(models) - n_empty)
    for i in range(n_z3):
        q = sat_qs[rng.randrange(len(sat_qs))]
        models.append(ns.Model([z3_model_of(z3, q, reg, rng, perturb=(i % 2 == 1))]))
    models += [ns.Model() for _ in range(n_empty)]
    rng.shuffle(models)
    qs = corp.queries[:n_queries]
    queries = []
    for q in qs:
        asts = to_z3(z3, q.constraints)
        queries.append(z3.simplify(z3.And(*asts)))
    x = z3.BitVec("x_unsat", 256)
    queries.append(z3.simplify(z3.And(z3.ULT(x, z3.BitVecVal(5, 256)), z3.ULT(z3.BitVecVal(9, 256), x))))
    return models, queries, qs, reg


def twin(ns, models):
    """The same models as new objects with empty evaluation memos: a GPU witness's Witness
    memoises every term value it computes, so two caches timed on the SAME witness objects
    would each profit from the other's evaluations."""
    import copy

    from mythril_amd.smt.model import WitnessModel

    out = []
    for m in models:
        if not m.raw:
            out.append(ns.Model())
            continue
        im = m.raw[0]
        if isinstance(im, integration.Z3WitnessView):
            wm = im.internal
            w = copy.copy(wm.w)
            w._memo, w._pos, w._keccak_tables = {}, None, {}
            w._first = w._building = None
            wm2 = WitnessModel(w, wm.constraints)
            wm2.origin = wm.origin
            wm2.parts, wm2.reg = wm.parts, wm.reg    # a native witness is built per cache entry
            out.append(ns.Model([integration.Z3WitnessView(wm2)]))
        else:
            out.append(ns.Model([copy.deepcopy(im)]))
    return out


# ---- a Mythril-shaped process for bench.py (the tests use pytest's monkeypatch instead) -----
class _Patch:
    """monkeypatch's setitem / setattr / setenv / delenv, undone by ``undo()``."""

    def __init__(self):
        self._undo = []

    def setitem(self, d, k, v):
        old = d.get(k, _MISSING)
        self._undo.append(lambda: d.__setitem__(k, old) if old is not _MISSING else d.pop(k, None))
        d[k] = v

    def setattr(self, o, k, v):
        old = getattr(o, k)
        self._undo.append(lambda: setattr(o, k, old))
        setattr(o, k, v)

    def setenv(self, k, v):
        import os

        self.setitem(os.environ, k, v)

    def delenv(self, k):
        import os

        old = os.environ.pop(k, _MISSING)
        if old is not _MISSING:
            self._undo.append(lambda: os.environ.__setitem__(k, old))

    def undo(self):
        for f in reversed(self._undo):
            f()
        self._undo.clear()


_MISSING = object()


def _stats(xs):
    import numpy as np

    if not xs:
        return None
    return {"median": round(float(np.median(xs)), 4), "mean": round(float(np.mean(xs)), 4),
            "p95": round(float(np.percentile(xs, 95)), 4), "max": round(float(np.max(xs)), 4)}


def quick_sat_profile(n_models: int = 100, n_scenarios: int = 16, n_queries: int = 80,
                      gpu_frac: float = 0.4, empty_frac: float = 0.1, seed: int = 7) -> dict:
    """Per-query quick-sat cost with ``n_models`` cached models: the reference loop
    (deep copy + eval per model, support_utils.py:61-68) vs the GPU-resident ModelCache, on
    the same models and queries in the same order; every choice must agree."""
    import time

    import fake_z3 as z3
    import mythril_standin
    from mythril_amd import model_cache as MC

    mp = _Patch()
    try:
        ns = mythril_standin.install(mp, z3)
        models, queries, _, _ = build(z3, ns, n_models=n_models, n_scenarios=n_scenarios, seed=seed,
                                      n_queries=n_queries, gpu_frac=gpu_frac, empty_frac=empty_frac)
        twins = twin(ns, models)
        pos_a = {id(m): i for i, m in enumerate(models)}
        pos_b = {id(m): i for i, m in enumerate(twins)}
        ref = ns.ModelCache()
        gpu = MC.gpu_model_cache_class()()
        for a, b in zip(models, twins):
            ref.put(a, 1)
            gpu.put(b, 1)
        MC.STATS.__init__()
        t_ref, t_gpu, agree, hits = [], [], 0, 0
        slowest = (0.0, -1, {})
        for qi, q in enumerate(queries):
            t0 = time.perf_counter()
            a = ref.check_quick_sat(q)
            t1 = time.perf_counter()
            ph0 = dict(MC.STATS.phase_s)
            b = gpu.check_quick_sat(q)
            t2 = time.perf_counter()
            if t2 - t1 > slowest[0]:
                slowest = (t2 - t1, qi, {k: round(1e3 * (v - ph0.get(k, 0.0)), 3) for k, v in MC.STATS.phase_s.items()})
            t_ref.append(1e3 * (t1 - t0))
            t_gpu.append(1e3 * (t2 - t1))
            agree += (a is False and b is False) or (
                a is not False and b is not False and pos_a[id(a)] == pos_b[id(b)])
            hits += a is not False
        kinds = {}
        for m in models:
            k = type(m.raw[0]).__name__ if m.raw else "empty Model()"
            kinds[k] = kinds.get(k, 0) + 1
        st = MC.STATS
        return {"cached_models": len(models), "model_kinds": kinds, "queries": len(queries),
                "answered_from_cache": hits, "choices_agree": agree,
                "reference_loop_ms": _stats(t_ref), "gpu_model_cache_ms": _stats(t_gpu),
                "speedup_mean": round(sum(t_ref) / max(sum(t_gpu), 1e-9), 2),
                "engine_calls": st.engine_calls, "models_on_engine": st.models_engine,
                "models_by_reference_statement": st.models_host, "leaf_evals": st.leaf_evals,
                "leaf_evals_native": st.leaf_evals_native,
                "slowest_query": {"index": slowest[1], "ms": round(1e3 * slowest[0], 3), "phase_ms": slowest[2]},
                "verdicts": {"memo": st.verdicts_memo, "native": st.verdicts_native, "engine": st.verdicts_engine},
                "baseline": "reference_loop_ms is the stand-in's loop (tests/mythril_standin.py "
                            "ModelCache.check_quick_sat: deepcopy + eval per model) over the stand-in z3 "
                            "(tests/fake_z3.py ModelRef) and Z3WitnessView models, not libz3",
                "phase_ms_per_query": {k: round(1e3 * v / max(st.queries, 1), 4) for k, v in st.phase_s.items()}}
    finally:
        mp.undo()


def funnel_profile(n_scenarios: int = 16, n_queries: int = 200, seed: int = 11) -> dict:
    """The real funnel's per-query cost (support/model.py:63-125 restated in
    tests/mythril_standin.py) with the drop-in installed (GpuOptimize + GpuModelCache):
    ``Constraints.is_possible()`` per corpus query in issue order, with its phases —
    ``simplify(And(*cs))`` (timed on the same constraints), quick-sat, the ``ThreadPool(1)``
    spawn / terminate around the worker (timed on its own), and ``GpuOptimize.check``."""
    import time
    from multiprocessing.pool import ThreadPool

    import fake_z3 as z3
    import mythril_standin
    from mythril_amd import corpus as Cp

    mp = _Patch()
    try:
        ns = mythril_standin.install(mp, z3)
        integration.install()
        funnel = ns.funnel
        corp = Cp.build(n_scenarios=n_scenarios, txs=2, seed=seed)
        from mythril_amd.integration import sync_keccak_registry  # noqa: F401
        from mythril_amd.smt import to_dag

        # the corpus's keccak interpretation is the process registry's (the live funnel
        # mirrors the keccak manager into it, integration.sync_keccak_registry)
        saved_reg = dict(to_dag.DEFAULT_REGISTRY.keccak)
        to_dag.DEFAULT_REGISTRY.keccak.clear()
        to_dag.DEFAULT_REGISTRY.keccak.update(corp.kfm.registry.keccak)
        gpu_check.reset_cache()
        qs = corp.queries[:n_queries]
        bools = [[ns.Bool(a) for a in to_z3(z3, q.constraints)] for q in qs]
        opt = funnel.Optimize
        t_check, t_qs = [], []
        orig_check = opt.check

        def timed_check(self, *a):
            t0 = time.perf_counter()
            try:
                return orig_check(self, *a)
            finally:
                t_check.append(1e3 * (time.perf_counter() - t0))

        mp.setattr(opt, "check", timed_check)
        mc = funnel.model_cache
        orig_qs = mc.check_quick_sat

        def timed_qs(c):
            t0 = time.perf_counter()
            try:
                return orig_qs(c)
            finally:
                t_qs.append(1e3 * (time.perf_counter() - t0))

        mc.check_quick_sat = timed_qs
        walls, sat = [], 0
        smt = sys_mod("mythril.laser.smt")
        t_simp = []
        for bs in bools:
            t0 = time.perf_counter()
            smt.simplify(smt.And(*bs))
            t_simp.append(1e3 * (time.perf_counter() - t0))
        for bs in bools:
            c = ns.Constraints(bs)
            t0 = time.perf_counter()
            sat += bool(c.is_possible())
            walls.append(1e3 * (time.perf_counter() - t0))
        t_pool = []
        for _ in range(50):
            t0 = time.perf_counter()
            pool = ThreadPool(1)
            try:
                pool.apply_async(int, (0,)).get(10)
            finally:
                pool.terminate()
            t_pool.append(1e3 * (time.perf_counter() - t0))
        to_dag.DEFAULT_REGISTRY.keccak.clear()
        to_dag.DEFAULT_REGISTRY.keccak.update(saved_reg)
        n = max(len(walls), 1)
        phases = {"simplify_and": sum(t_simp) / n, "quick_sat": sum(t_qs) / n,
                  "thread_pool": sum(t_pool) / max(len(t_pool), 1) * (len(t_check) / n),
                  "gpu_optimize_check": sum(t_check) / n}
        phases["other"] = sum(walls) / n - sum(phases.values())
        return {"queries": len(walls), "sat": sat, "funnel_query_ms": _stats(walls),
                "phase_mean_ms": {k: round(v, 4) for k, v in phases.items()},
                "dominant_phase": max(phases, key=phases.get),
                "quick_sat_answered": len(walls) - len(t_check),
                "note": "stand-in funnel (tests/mythril_standin.py) over fake z3 ASTs; z3's own "
                        "simplify/eval costs are the stand-in's, not libz3's"}
    finally:
        mp.undo()


def sys_mod(name):
    import sys

    return sys.modules[name]
