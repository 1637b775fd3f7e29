"""The GPU-resident ModelCache (mythril_amd/model_cache.py) against the reference's quick-sat
loop (support/support_utils.py:57-71, restated in tests/mythril_standin.py).

Both caches hold the same models in the same LRU order; every query of a LASER-shaped
stream is answered by both and must return the SAME model object, leaving the SAME LRU
order (the reference bumps the chosen model).  The models mix GPU witnesses, z3-shaped
models (tests/fake_z3.ModelRef: explicit interpretations, an independent SMT-LIB evaluator)
and empty ``Model()``s; the stream ends with a query no model satisfies.  The CPU test runs
the engine call on the C oracle (tests/oracle_engine.py), the ``gpu`` test on the MI355X.
"""

import numpy as np
import pytest

import fake_z3 as z3
import model_cache_workload as W
import mythril_standin
import oracle_engine
from mythril_amd import integration
from mythril_amd import model_cache as MC
from mythril_amd.smt import gpu_check
from mythril_amd.smt import native_terms
from mythril_amd.smt import terms as T
from mythril_amd.z3_terms import converter


@pytest.fixture
def standin(monkeypatch):
    ns = mythril_standin.install(monkeypatch, z3)
    monkeypatch.setattr(gpu_check.CONFIG, "budget", 4096)
    integration._BATCH_CACHE.clear()
    return ns


def _lru(cache):
    return [id(m) for m in cache.model_cache.lru_cache.keys()]


def _run_both(ns, models, queries):
    ref = ns.ModelCache()
    gpu = MC.gpu_model_cache_class()()
    for m in models:
        ref.put(m, 1)
        gpu.put(m, 1)
    picks = []
    for q in queries:
        a = ref.check_quick_sat(q)
        b = gpu.check_quick_sat(q)
        assert a is b, (q, a, b)
        assert _lru(ref) == _lru(gpu)
        mru = list(reversed(ref.model_cache.lru_cache.keys()))
        picks.append(None if a is False else mru.index(a))
    return picks


def _check_stream(ns, models, queries):
    MC.STATS.__init__()
    picks = _run_both(ns, models, queries)
    assert picks[-1] is None                       # the contradiction: no model
    assert any(p is not None for p in picks)       # some query answered from the cache
    assert MC.STATS.engine_calls > 0 and MC.STATS.models_engine > 0
    assert MC.STATS.reference_loops == 0
    return picks


@pytest.mark.parametrize("first_stage,memo", [(0, True), (4, True), (0, False), (4, False)])
def test_quick_sat_choice_matches_reference_loop(standin, monkeypatch, first_stage, memo):
    """first_stage 0: every model in one launch; 4: the production two-launch setting; with
    and without the per-(model, conjunct) verdict memo."""
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "FIRST_STAGE", first_stage)
    monkeypatch.setattr(MC, "VERDICT_MEMO", memo)
    models, queries, _, _ = W.build(z3, standin, n_models=100, n_scenarios=6, n_queries=30)
    assert len(models) == 100
    picks = _check_stream(standin, models, queries)
    # both kinds of model answer somewhere in the stream
    assert len({p for p in picks if p is not None}) >= 1


@pytest.mark.parametrize("host_pairs", [0, 256])
def test_quick_sat_witness_only_cache(standin, monkeypatch, host_pairs):
    """A cache of GPU witnesses only — the live case: every model's leaves native, one
    launch from the (models, leaves, 8) block (host_pairs 0), or small batches of unknown
    (model, conjunct) verdicts by the native witness evaluator (256) — same choices as the
    reference loop."""
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "HOST_VERDICT_PAIRS", host_pairs)
    models, queries, _, _ = W.build(z3, standin, n_models=40, n_scenarios=4, n_queries=20, gpu_frac=1.0,
                                    empty_frac=0.0)
    models = [m for m in models if m.raw and isinstance(m.raw[0], integration.Z3WitnessView)]
    assert len(models) >= 10
    MC.STATS.__init__()
    picks = _run_both(standin, models, queries)
    assert picks[-1] is None and any(p is not None for p in picks)
    assert MC.STATS.models_host == 0 and MC.STATS.leaf_evals == 0
    if host_pairs:
        assert MC.STATS.verdicts_native > 0 and MC.STATS.verdicts_memo > 0
    else:
        assert MC.STATS.leaf_evals_native > 0 and MC.STATS.verdicts_engine > 0 and MC.STATS.verdicts_native == 0


def test_quick_sat_small_caches_and_empty(standin, monkeypatch):
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "FIRST_STAGE", 0)
    models, queries, _, _ = W.build(z3, standin, n_models=12, n_scenarios=3, n_queries=12)
    _run_both(standin, models, queries)
    gpu = MC.gpu_model_cache_class()()
    assert gpu.check_quick_sat(queries[0]) is False   # no models
    gpu.put(standin.Model(), 1)                        # an empty Model(): eval is None
    assert gpu.check_quick_sat(queries[1]) is False


def test_quick_sat_literal_true_and_false(standin, monkeypatch):
    oracle_engine.install(monkeypatch)
    m1, m2 = standin.Model([z3.ModelRef({})]), standin.Model([z3.ModelRef({})])
    gpu = MC.gpu_model_cache_class()()
    gpu.put(m1, 1)
    gpu.put(m2, 1)
    assert gpu.check_quick_sat(z3.BoolVal(True)) is m2     # most recent first
    assert list(gpu.model_cache.lru_cache.values()) == [1, 2]
    assert gpu.check_quick_sat(z3.BoolVal(False)) is False


def test_leaf_values_are_memoised_per_model(standin, monkeypatch):
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "FIRST_STAGE", 0)
    x = z3.BitVec("x", 256)
    A = z3.Array("A", z3.BitVecSort(256), z3.BitVecSort(256))
    zm = z3.ModelRef({x.decl(): 5, A.decl(): ({5: 7}, 1)})
    gpu = MC.gpu_model_cache_class()()
    gpu.put(standin.Model([zm]), 1)
    MC.STATS.__init__()
    for k in range(6):
        q = z3.simplify(z3.And(z3.ULT(x, z3.BitVecVal(10 + k, 256)),
                               z3.Select(A, x) == z3.BitVecVal(7, 256)))
        assert gpu.check_quick_sat(q) is not False
    assert MC.STATS.leaf_evals == 2       # x and A[x], once for the whole stream
    q = z3.simplify(z3.Select(z3.Store(A, x, z3.BitVecVal(3, 256)), z3.BitVecVal(6, 256)) == z3.BitVecVal(1, 256))
    assert gpu.check_quick_sat(q) is not False   # A[6] is A's else value 1


def test_a_model_the_leaves_cannot_value_goes_to_the_reference_statement(standin, monkeypatch):
    """A z3 model whose eval rejects a leaf is decided by deepcopy + eval in its place."""
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "FIRST_STAGE", 0)

    class Picky(z3.ModelRef):
        def __deepcopy__(self, memo):
            return Picky(self._interp)

        def eval(self, e, model_completion=False):
            # rejects the leaf forms (a select, or the leaves' concatenation of the batched
            # evaluation), accepts the whole query
            if e.decl().kind() in (z3.Z3_OP_SELECT, z3.Z3_OP_CONCAT):
                raise z3.Z3Exception("no")
            return super().eval(e, model_completion)

    x = z3.BitVec("x", 256)
    A = z3.Array("A", z3.BitVecSort(256), z3.BitVecSort(256))
    q = z3.simplify(z3.And(z3.ULT(x, z3.BitVecVal(10, 256)), z3.Select(A, x) == z3.BitVecVal(7, 256)))
    good = standin.Model([z3.ModelRef({x.decl(): 5, A.decl(): ({5: 7}, 1)})])
    picky = standin.Model([Picky({x.decl(): 5, A.decl(): ({5: 7}, 1)})])
    gpu = MC.gpu_model_cache_class()()
    gpu.put(good, 1)
    gpu.put(picky, 1)
    MC.STATS.__init__()
    assert gpu.check_quick_sat(q) is picky    # decided by deepcopy + eval of the whole query
    assert MC.STATS.models_host == 1 and MC.STATS.models_engine == 1


def test_native_witness_leaves_equal_python_witness(standin, monkeypatch):
    """pflt_witness_values (csrc/pf_recheck.cpp) gives interp.Witness.leaf_value's value for
    every quick-sat leaf of the corpus queries under every GPU witness of the workload; a
    registry that gained hashes since is re-parsed (the Python witness reads it live)."""
    oracle_engine.install(monkeypatch)
    if not native_terms.has_explicit():
        pytest.skip("libpflower.so not built")
    models, _, qs, reg = W.build(z3, standin, n_models=30, n_scenarios=4, n_queries=40)
    wms = [m.raw[0].internal for m in models if m.raw and isinstance(m.raw[0], integration.Z3WitnessView)]
    assert wms and all(wm.parts for wm in wms)
    lvs = [MC.leaf_values_of(z3, integration.Z3WitnessView(wm)) for wm in wms]
    assert all(isinstance(lv, MC.NativeLeafValues) for lv in lvs)
    leaves = {}
    for q in qs:
        try:
            ls, _ = MC.explicit_program(T.and_(*q.constraints) if len(q.constraints) > 1 else q.constraints[0])
        except Exception:  # noqa: BLE001 - a query the explicit lowering declines
            continue
        leaves.update(dict.fromkeys(ls))
    leaves = list(leaves)
    assert len(leaves) > 10
    MC.STATS.__init__()
    rows = MC.native_rows(lvs, leaves)
    assert len(rows) >= 0.9 * len(lvs) and MC.STATS.leaf_evals_native == len(rows) * len(leaves)
    for j, r in rows.items():
        w = wms[j].w
        for t, limbs in zip(leaves, r):
            want = w.leaf_value(t) & T.M(max(t.width, 1))
            assert native_terms.ints_of(limbs[None])[0] == want, t
    # slot renumbering (a new epoch every few terms): the values stay the witness's
    monkeypatch.setattr(native_terms, "_SLOTS_MAX", 7)
    for lo in range(0, min(len(leaves), 40), 5):
        part = leaves[lo:lo + 5]
        again = MC.native_rows(lvs, part)
        for j, r in again.items():
            assert native_terms.ints_of(r) == [native_terms.ints_of(rows[j][leaves.index(t)][None])[0]
                                               for t in part]
    # a hash registered after the witnesses were built: both evaluators see it
    k = next(iter(reg.keccak))
    app = T.apply(f"keccak256_{k}", 256, T.const(12345, k))
    reg.keccak[k].concrete[12345] = 0xABCDEF
    rows = MC.native_rows(lvs, [app])
    assert len(rows) == len(lvs)
    for j, r in rows.items():
        assert native_terms.ints_of(r)[0] == wms[j].w.leaf_value(app) == 0xABCDEF


def test_first_stage_counts_only_dear_models():
    """The first launch takes the newest models up to the (k + 1)-th whose leaves are dear
    (z3 models, unvaluable ones); natively held witnesses ride along."""
    nat = MC.NativeLeafValues.__new__(MC.NativeLeafValues)
    z = MC.LeafValues(lambda t: 0)
    assert MC.first_stage_end([nat] * 10, 4) == 10
    assert MC.first_stage_end([z] * 10, 4) == 4
    assert MC.first_stage_end([nat, z, nat, None, z, z, nat, z, nat], 4) == 7
    assert MC.first_stage_end([z] * 10, 0) == 10
    assert MC.first_stage_end([], 4) == 0


def test_explicit_lowering_native_equals_python(standin, monkeypatch):
    oracle_engine.install(monkeypatch)
    if not native_terms.has_explicit():
        pytest.skip("libpflower.so not built")
    from mythril_amd import corpus as C

    corp = C.build(n_scenarios=6, txs=2, seed=3)
    n = 0
    for q in corp.queries[:80]:
        conj = [c for c in q.constraints if c is not T.TRUE]
        lv1, p1 = MC._lower_explicit(conj)
        lv2, p2 = MC.lower_explicit_py(conj)
        assert lv1 == lv2
        assert np.array_equal(np.asarray(p1.words), np.asarray(p2.words))
        assert list(p1.consts) == list(p2.consts)
        assert [(v.name, v.width) for v in p1.vars] == [(v.name, v.width) for v in p2.vars]
        n += 1
    assert n == min(80, len(corp.queries))


def test_explicit_program_holds_under_the_planted_models(monkeypatch):
    """The explicit program computes the conjunction from its leaves: with every leaf valued
    by a planted model (the engine's interpretation of arrays and keccak), each SAT-labelled
    corpus query's program is true, and its value agrees with evaluating the terms
    directly under that model for every query."""
    import pyoracle as O
    from mythril_amd import corpus as C
    from mythril_amd import ir

    oracle_engine.install(monkeypatch)
    corp = C.build(n_scenarios=6, txs=2, seed=9)
    n_sat = 0
    for q in corp.queries[:120]:
        if q.planted is None:
            continue
        conj = [c for c in q.constraints if c is not T.TRUE]
        leaves, prog = MC._lower_explicit(conj)
        ev = C._PlantedEval(q.planted, corp.kfm.registry)
        vals = [int(ev.ev(t)) & ((1 << max(t.width, 1)) - 1) for t in leaves]
        got = bool(O.SetView.from_batch(ir.Batch([prog]), 0).evaluate(vals))
        assert got == all(bool(ev.ev(c)) for c in conj), q.origin
        n_sat += got
    assert n_sat > 20


def test_install_rebinds_the_funnel_cache(standin):
    m = standin.Model([z3.ModelRef({})])
    standin.funnel.model_cache.put(m, 3)
    MC.install()
    mc = standin.funnel.model_cache
    assert type(mc).__name__ == "GpuModelCache"
    assert list(mc.model_cache.lru_cache.items()) == [(m, 3)]
    MC.install()                                  # idempotent
    assert standin.funnel.model_cache is mc


@pytest.mark.gpu
@pytest.mark.parametrize("first_stage", [0, 4])
def test_gpu_quick_sat_choice_matches_reference_loop(standin, engine, monkeypatch, first_stage):
    monkeypatch.setattr(MC, "FIRST_STAGE", first_stage)
    models, queries, _, _ = W.build(z3, standin, n_models=100, n_scenarios=8, n_queries=60)
    _check_stream(standin, models, queries)


@pytest.mark.gpu
def test_gpu_eval_program_matches_oracle(engine, monkeypatch):
    """pf_eval_program (one call: validate, upload, one launch) gives the oracle's verdict on
    explicit assignments of corpus queries' explicit programs — random values and the
    planted models' values (SAT by construction under the engine's interpretation)."""
    import random

    import pyoracle as O
    from mythril_amd import corpus as C
    from mythril_amd import ir

    corp = C.build(n_scenarios=4, txs=2, seed=5)
    rng = random.Random(1)
    n = 0
    for q in corp.queries[:40]:
        leaves, prog = MC._lower_explicit([c for c in q.constraints if c is not T.TRUE])
        ev = C._PlantedEval(q.planted, corp.kfm.registry) if q.planted is not None else None
        rows = []
        for k in range(70):
            vals = []
            for t in leaves:
                if k == 0 and ev is not None:
                    v = int(ev.ev(t))
                else:
                    v = rng.choice([0, 1, rng.getrandbits(max(t.width, 1))])
                vals.append(v & ((1 << max(t.width, 1)) - 1))
            rows.append(vals)
        soa = MC.soa_of(MC.rows_of_ints(rows), MC.n_vars(prog))
        got = engine.eval_program(prog, soa)
        sv = O.SetView.from_batch(ir.Batch([prog]), 0)
        want = [bool(sv.evaluate(r)) for r in rows]
        assert want[0] or q.label != "sat", q.origin   # the planted model satisfies its query
        assert list(got) == want, q.origin
        db = engine.upload([prog])
        try:
            assert list(engine.eval_assignments(db, 0, soa)) == want
        finally:
            db.free()
        n += 1
    assert n == 40


def _group_case(corp, rng, q, n_rows=70):
    """(query term, leaves, groups, rows) of one corpus query split into conjunct groups."""
    from mythril_amd import corpus as C

    cs = [c for c in q.constraints if c is not T.TRUE]
    query = T.and_(*cs) if len(cs) > 1 else cs[0]
    leaves, groups = MC.explicit_groups(query)
    ev = C._PlantedEval(q.planted, corp.kfm.registry) if q.planted is not None else None
    rows = []
    for k in range(n_rows):
        vals = []
        for t in leaves:
            v = int(ev.ev(t)) if k == 0 and ev is not None else rng.choice([0, 1, rng.getrandbits(max(t.width, 1))])
            vals.append(v & ((1 << max(t.width, 1)) - 1))
        rows.append(vals)
    return query, leaves, groups, rows


def test_conjunct_groups_equal_the_whole_program(standin, monkeypatch):
    """A long query split into conjunct groups (explicit_groups, evaluated per group and
    and-ed) gives the whole-conjunction program's verdict on every explicit assignment —
    random values and the planted model; and the quick-sat choices stay the reference's."""
    import random

    import pyoracle as O
    from mythril_amd import corpus as C
    from mythril_amd import ir

    eng = oracle_engine.install(monkeypatch)
    if not native_terms.has_explicit():
        pytest.skip("libpflower.so not built")
    monkeypatch.setattr(MC, "SPLIT_NODES", 24)    # split small queries too
    MC._GROUPS.clear()
    corp = C.build(n_scenarios=4, txs=2, seed=5)
    rng = random.Random(3)
    split = 0
    for q in corp.queries[:40]:
        query, leaves, groups, rows = _group_case(corp, rng, q, n_rows=12)
        if not isinstance(groups, MC.ExplicitGroups):
            continue
        split += 1
        assert len(groups.programs) >= 2 and sorted(set(groups.gather.tolist())) == list(range(len(leaves)))
        whole_leaves, whole = MC.explicit_program(query)
        sv = O.SetView.from_batch(ir.Batch([whole]), 0)
        idx = [leaves.index(t) for t in whole_leaves]
        want = [bool(sv.evaluate([r[i] for i in idx])) for r in rows]
        got = MC.eval_rows(groups, MC.rows_of_ints(rows), eng)
        assert list(got) == want, q.origin
    assert split >= 10
    models, queries, _, _ = W.build(z3, standin, n_models=30, n_scenarios=4, n_queries=20)
    _check_stream(standin, models, queries)
    MC._GROUPS.clear()


def test_conjunct_programs_cached_across_queries(standin, monkeypatch):
    """CONJ_PROGRAMS: one cached program per flattened conjunct, every query's conjuncts in
    one pf_eval_programs call — the same choices as the reference loop, and a conjunct shared
    by later queries is lowered once."""
    oracle_engine.install(monkeypatch)
    if not native_terms.has_explicit():
        pytest.skip("libpflower.so not built")
    monkeypatch.setattr(MC, "CONJ_PROGRAMS", True)
    MC._GROUPS.clear()
    MC._CONJ.clear()
    lowered = []
    real = MC._lower_explicit
    monkeypatch.setattr(MC, "_lower_explicit", lambda conj: (lowered.append(conj[0]), real(conj))[1])
    models, queries, _, _ = W.build(z3, standin, n_models=30, n_scenarios=4, n_queries=30)
    _check_stream(standin, models, queries)
    assert len(lowered) == len(set(lowered))          # every conjunct lowered once
    assert len(MC._CONJ) == len(lowered)
    MC._GROUPS.clear()
    MC._CONJ.clear()


@pytest.mark.gpu
def test_gpu_eval_programs_match_per_group_programs(engine, monkeypatch):
    """pf_eval_programs (every group of a query in one launch) gives each group's
    pf_eval_program verdicts, and their conjunction the whole program's."""
    import random

    from mythril_amd import corpus as C

    monkeypatch.setattr(MC, "SPLIT_NODES", 24)
    MC._GROUPS.clear()
    corp = C.build(n_scenarios=4, txs=2, seed=5)
    rng = random.Random(4)
    split = 0
    for q in corp.queries[:40]:
        query, leaves, groups, rows = _group_case(corp, rng, q)
        if not isinstance(groups, MC.ExplicitGroups):
            continue
        split += 1
        soa = MC.soa_of(MC.rows_of_ints(rows), len(leaves))[groups.gather]
        got = engine.eval_programs(groups.pack(), soa)
        ends = groups.offsets[1:] + [len(groups.gather)]
        for s, (prog, lo, hi) in enumerate(zip(groups.programs, groups.offsets, ends)):
            part = np.ascontiguousarray(soa[lo:hi]) if hi > lo else MC.soa_of(MC.rows_of_ints(rows), 0)
            assert list(got[s]) == list(engine.eval_program(prog, part)), (q.origin, s)
        whole_leaves, whole = MC.explicit_program(query)
        idx = [leaves.index(t) for t in whole_leaves]
        want = engine.eval_program(whole, MC.soa_of(MC.rows_of_ints([[r[i] for i in idx] for r in rows]),
                                                    MC.n_vars(whole)))
        assert list(got.all(axis=0)) == list(want), q.origin
    assert split >= 10
    MC._GROUPS.clear()


@pytest.mark.gpu
def test_gpu_eval_programs_edge_shapes(engine):
    """pf_eval_programs over sets of unlike shapes in one call — no variables (always true /
    always false), config-3 DAG programs (16 registers' worth in the wide kernel), LASER-like
    sets — and 130 candidates (three waves per set): each set's verdicts equal the oracle's
    on its own SoA rows."""
    import random

    import pyoracle as O
    from mythril_amd import ir, synth
    from mythril_amd.lower import Dag, lower

    progs = []
    for b in (True, False):
        d = Dag()
        d.assert_(d.bconst(b))
        progs.append(lower(d))
    progs += [synth.random_dag_set(700 + i, plant=False)[0] for i in range(3)]
    progs += [synth.mythril_like_set(i) for i in range(2)]
    b = ir.Batch(progs)
    pack = tuple(np.ascontiguousarray(a, dtype=np.uint32).reshape(-1) for a in (b.code, b.consts, b.schema, b.descs))
    n_vars = len(b.schema)
    n_cand = 130
    rng = random.Random(11)
    soa = np.zeros((max(n_vars, 1), 8, n_cand), dtype=np.uint32)
    for v in range(n_vars):
        w = (int(b.schema[v][0]) >> 8) & 0x3FF
        for c in range(n_cand):
            x = rng.choice([0, 1, rng.getrandbits(w)])
            soa[v, :, c] = [(x >> (32 * k)) & 0xFFFFFFFF for k in range(8)]
    got = engine.eval_programs(pack, soa[:n_vars] if n_vars else soa)
    assert got.shape == (len(progs), n_cand)
    for s in range(len(progs)):
        sv = O.SetView.from_batch(b, s)
        off, nv = int(b.descs[s][4]), int(b.descs[s][5])
        want = [bool(sv.evaluate([O.limbs_to_int(soa[off + v, :, c]) for v in range(nv)])) for c in range(n_cand)]
        assert list(got[s]) == want, s
    assert got[0].all() and not got[1].any()


@pytest.mark.gpu
def test_gpu_witness_leaves_native_equal_python(standin, engine):
    """The same equality as the CPU test, on witnesses the MI355X found: every corpus leaf's
    value from pflt_witness_values equals interp.Witness.leaf_value."""
    models, _, qs, reg = W.build(z3, standin, n_models=30, n_scenarios=4, n_queries=40)
    wms = [m.raw[0].internal for m in models if m.raw and isinstance(m.raw[0], integration.Z3WitnessView)]
    assert wms and all(wm.parts for wm in wms)
    lvs = [MC.leaf_values_of(z3, integration.Z3WitnessView(wm)) for wm in wms]
    leaves = {}
    for q in qs:
        try:
            ls, _ = MC.explicit_program(T.and_(*q.constraints) if len(q.constraints) > 1 else q.constraints[0])
        except Exception:  # noqa: BLE001 - a query the explicit lowering declines
            continue
        leaves.update(dict.fromkeys(ls))
    leaves = list(leaves)
    rows = MC.native_rows(lvs, leaves)
    assert len(rows) >= 0.9 * len(lvs)
    for j, r in rows.items():
        w = wms[j].w
        for t, limbs in zip(leaves, r):
            assert native_terms.ints_of(limbs[None])[0] == w.leaf_value(t) & T.M(max(t.width, 1)), t


@pytest.mark.parametrize("batched", [True, False])
def test_completion_shared_between_leaves_matches_whole_conjunction(standin, monkeypatch, batched):
    """z3's model completion ADDS interpretations to the model it evaluates on (fake_z3
    ModelRef does the same), so evaluating a query's leaves one by one on one private copy —
    or all of them in one eval of their concatenation — could in principle differ from the
    reference's single eval of the whole conjunction (support_utils.py:62-63) when leaves
    share symbols the model does not interpret.  Models here interpret only some of the
    symbols the queries read (a scalar, an array, a function), the queries read the
    uninterpreted ones through several leaves, and the choice must equal the reference
    loop's on every query, per leaf and batched."""
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "FIRST_STAGE", 0)
    if not batched:
        orig = MC._z3_leaf_evaluators
        monkeypatch.setattr(MC, "_z3_leaf_evaluators", lambda z, im: (orig(z, im)[0], None))
    x, y = z3.BitVec("x", 256), z3.BitVec("y", 256)
    A = z3.Array("A", z3.BitVecSort(256), z3.BitVecSort(256))
    f = z3.Function("f", z3.BitVecSort(256), z3.BitVecSort(256))
    V = lambda v: z3.BitVecVal(v, 256)  # noqa: E731
    models = [standin.Model([z3.ModelRef(interp)]) for interp in (
        {},                                          # nothing interpreted
        {x.decl(): 3},                               # x only
        {y.decl(): 4, A.decl(): ({4: 9}, 2)},        # y and A
        {A.decl(): ({0: 1}, 0), f: ({(5,): 6}, 7)},
        {x.decl(): 0, y.decl(): 0},
    )]
    queries = [
        z3.And(z3.Select(A, y) == V(0), y == V(0)),                    # completes y, A
        z3.And(z3.Select(A, y + V(1)) == z3.Select(A, y), x == V(0)),
        z3.And(f(y) == f(V(0)), z3.Select(A, x) == V(0)),
        z3.And(f(x) == V(0), z3.ULT(y, V(5)), z3.Select(A, y) == V(9)),
        z3.And(z3.Select(A, x) == V(1), f(V(5)) == V(6)),
        z3.And(f(x + y) == f(y + x), z3.Select(A, V(4)) == V(2)),
        z3.And(y == V(1), y == V(2)),                                   # no model
    ]
    picks = _run_both(standin, models, [z3.simplify(q) for q in queries])
    assert picks[-1] is None and sum(p is not None for p in picks) >= 3


def test_verdict_memo_is_bounded(standin, monkeypatch):
    """A model's per-conjunct verdict memo is cleared once it passes VERDICTS_MAX entries,
    and the choices stay the reference loop's."""
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(MC, "VERDICTS_MAX", 3)
    models, queries, _, _ = W.build(z3, standin, n_models=12, n_scenarios=3, n_queries=12)
    _run_both(standin, models, queries)
    gpu = MC.gpu_model_cache_class()()
    for m in models:
        gpu.put(m, 1)
    for q in queries:
        gpu.check_quick_sat(q)
    assert all(len(lv.verdicts) <= 3 + 16 for _, lv in gpu._leaves.values())
