"""The Mythril seams in a Mythril-shaped process: the z3-AST walker, the drop-in ``Optimize``
inside the query funnel, the GPU witness as a ``Model`` that survives ``ModelCache``'s
deep copies, and the tx-boundary batch over ``WorldState``s.

z3 and Mythril are not installed here; tests/fake_z3.py and tests/mythril_standin.py stand
in for them with the reference's calling conventions (see their docstrings).  The CPU tests
run the engine's host pipeline on the C oracle (tests/oracle_engine.py); the ``gpu`` tests
run the same flows on the MI355X engine.
"""

import copy

import pytest

import fake_z3 as z3
import mythril_standin
import oracle_engine
from mythril_amd import integration
from mythril_amd.lower import LoweringError
from mythril_amd.smt import gpu_check
from mythril_amd.smt import terms as T
from mythril_amd.smt.interp import Witness
from mythril_amd.smt.solver import SolverStatistics
from mythril_amd.smt.to_dag import Lowered, TermLowering, UFRegistry
from mythril_amd.z3_terms import Z3Converter, converter


def _ev(term, env):
    """Evaluate a term under {name: value} (free symbols not in env complete to 0)."""
    names = sorted(env)
    vs = [T.var(n, w) for n, (v, w) in ((n, env[n]) for n in names)]
    w = Witness(Lowered(None, vs, [], {}), [env[n][0] for n in names], UFRegistry())
    return w.ev(term)


# ---- the z3-AST walker ---------------------------------------------------------------------
def _mythril_like(x, y, cd, size):
    """Shapes LASER builds: signed compares, bvsdiv, calldata byte reads, SUB, no-overflow."""
    byte = z3.If(z3.BitVecVal(4, 256) < size, z3.Select(cd, z3.BitVecVal(4, 256)), z3.BitVecVal(0, 8))
    return [
        z3.ULT(x - y, z3.BitVecVal(1000, 256)),
        x / z3.BitVecVal(3, 256) == y,
        z3.Not(z3.BVAddNoOverflow(x, y, False)),
        z3.BVSubNoUnderflow(x, y, False),
        z3.BVMulNoOverflow(x, z3.BitVecVal(2, 256), False),
        z3.Extract(7, 0, x) == byte,
        z3.Concat(z3.Extract(255, 8, y), byte) != x,
        z3.UGE(z3.LShR(x, 3) | (y << 2), z3.URem(x, y)),
    ]


@pytest.mark.parametrize("simplified", [False, True])
def test_walker_matches_z3_semantics(simplified):
    """Each converted constraint evaluates like the z3 expression's SMT-LIB meaning, raw and
    after the simplifier's rewrites (SUB as bvadd/bvmul -1, ULT as not bvule, zero_extend as
    concat) — checked on values that flip every predicate."""
    x, y = z3.BitVec("x", 256), z3.BitVec("y", 256)
    cd, size = z3.Array("1_calldata", z3.BitVecSort(256), z3.BitVecSort(8)), z3.BitVec("1_calldatasize", 256)
    cs = _mythril_like(x, y, cd, size)
    if simplified:
        cs = [z3.simplify(c) for c in cs]
    conv = Z3Converter(z3)
    ts = conv.terms(cs)
    M = (1 << 256) - 1
    cases = [(5, 2), (M, 1), (M, M), (1 << 255, 7), (1000, 999), (3, 4), (0, 0), (2 ** 200 + 9, 3)]
    for xv, yv in cases:
        env = {"x": (xv, 256), "y": (yv, 256), "1_calldatasize": (0, 256)}
        got = [bool(_ev(t, env)) for t in ts]
        want = [
            ((xv - yv) & M) < 1000,
            _sdiv(xv, 3) == yv,
            xv + yv > M,
            yv <= xv,
            xv * 2 <= M,
            (xv & 0xFF) == 0,                       # size 0 -> byte 0
            (((yv >> 8) << 8) | 0) != xv,
            ((xv >> 3) | ((yv << 2) & M)) >= (xv if yv == 0 else xv % yv),
        ]
        assert got == want, (xv, yv, got, want)


def _sdiv(a, b):
    sa = a - (1 << 256) if a >> 255 else a
    q = abs(sa) // b
    return (q if sa >= 0 else -q) & ((1 << 256) - 1)


def test_walker_caches_by_ast_and_keeps_the_ast():
    x = z3.BitVec("x", 256)
    e = z3.ULT(x + 1, z3.BitVecVal(9, 256))
    conv = Z3Converter(z3)
    t1 = conv.term(e)
    m = conv.misses
    t2 = conv.term(e)
    assert t1 is t2 and conv.misses == m and conv.hits >= 1
    # the entry holds the AST itself, so its id cannot be recycled while cached
    assert any(ast is e for ast, _ in conv._cache.values())
    conv2 = Z3Converter(z3, max_entries=2)
    conv2.terms([z3.ULT(x, z3.BitVecVal(k, 256)) for k in range(5)])
    assert len(conv2._cache) <= 2


def test_walker_keccak_and_uf_shapes():
    """keccak256_<n> / inverse UFs (keccak_function_manager.py:71-84), arrays over stores and
    const arrays convert to the lowering's UF / array terms."""
    k512 = z3.Function("keccak256_512", z3.BitVecSort(512), z3.BitVecSort(256))
    inv = z3.Function("keccak256_512-1", z3.BitVecSort(256), z3.BitVecSort(512))
    a = z3.BitVec("a", 256)
    key = z3.Concat(a, z3.BitVecVal(1, 256))
    st = z3.Store(z3.K(z3.BitVecSort(256), z3.BitVecVal(0, 256)), k512(key), z3.BitVecVal(5, 256))
    cs = [inv(k512(key)) == key, z3.Select(st, k512(key)) == z3.BitVecVal(5, 256)]
    ts = converter(z3).terms(cs)
    assert ts[0].args[0].op == "apply" and ts[0].args[0].val[0] == "keccak256_512-1"
    TermLowering(UFRegistry()).lower(ts)  # lowers (no LoweringError)


def test_walker_rejects_unsupported_sorts_loudly():
    class _Q:
        pass

    conv = Z3Converter(z3)
    with pytest.raises(Exception):
        conv.term(_Q())


# ---- the witness as a Mythril Model ----------------------------------------------------------
@pytest.fixture
def standin(monkeypatch):
    ns = mythril_standin.install(monkeypatch, z3)
    eng = oracle_engine.install(monkeypatch)
    monkeypatch.setattr(gpu_check.CONFIG, "budget", 4096)
    integration._BATCH_CACHE.clear()
    st = SolverStatistics()
    st.gpu_sat = st.gpu_attempts = 0
    ns.engine = eng
    return ns


def _witness_model(cs):
    terms = converter(z3).terms(cs)
    m = gpu_check.check_sets([terms])[0]
    assert m is not None
    return m


def test_witness_model_survives_deepcopy_and_completes(standin):
    """ModelCache.check_quick_sat deep-copies every cached model (support_utils.py:62-68):
    the GPU model must copy, evaluate expressions over symbols outside its query with z3's
    model_completion defaults, and expose decls() for Model.eval's relevance rule."""
    x = z3.BitVec("call_value1", 256)
    internal = _witness_model([z3.ULT(x, z3.BitVecVal(1000, 256)), x != z3.BitVecVal(0, 256)])
    model = standin.Model([integration.Z3WitnessView(internal)])
    cp = copy.deepcopy(model)
    xv = cp.eval(x, model_completion=True)
    assert z3.is_bv_value(xv) and 0 < xv.as_long() < 1000
    new = z3.BitVec("sender_2", 256)          # a symbol of a later transaction
    assert cp.eval(new, model_completion=True).as_long() == 0
    assert z3.is_true(cp.eval(z3.ULT(x, z3.BitVecVal(1000, 256)), model_completion=True))
    assert z3.is_false(cp.eval(z3.And(new == z3.BitVecVal(1, 256), x == x), model_completion=True))
    names = {d.name() for d in model.decls()}
    assert "call_value1" in names
    assert x.decl() in list(model.raw[0].decls())
    assert model[x.decl()].as_long() == xv.as_long()


def test_funnel_answers_from_gpu_and_quick_sat_reuses_the_witness(standin):
    """get_model (support/model.py:63-125) with the rebound Optimize: the first objective-free
    query is answered by the engine, its model enters model_cache, and a later query that
    the same witness satisfies is answered by check_quick_sat's deep-copy + eval path."""
    integration.install()
    assert standin.funnel.Optimize.__name__ == "GpuOptimize"
    B = standin.Bool
    x = z3.BitVec("call_value1", 256)
    c1 = standin.Constraints([B(z3.ULT(x, z3.BitVecVal(50, 256))), B(x != z3.BitVecVal(0, 256))])
    assert c1.is_possible()
    st = SolverStatistics()
    assert st.gpu_sat == 1
    cached = list(standin.funnel.model_cache.model_cache.lru_cache.keys())
    assert len(cached) == 1
    launches = standin.engine.launches
    c2 = standin.Constraints([B(z3.ULT(x, z3.BitVecVal(60, 256))), B(x != z3.BitVecVal(0, 256))])
    assert c2.is_possible()
    assert standin.engine.launches == launches      # answered by quick-sat, no search


def test_funnel_unanswered_query_falls_back_to_z3(standin):
    """No witness -> the original z3 check() runs (the stand-in z3 answers unknown ->
    SolverTimeOutException -> is_possible() False under the default timeout,
    constraints.py:38-43); a contradiction is never reported SAT."""
    integration.install()
    B = standin.Bool
    x = z3.BitVec("x", 256)
    c = standin.Constraints([B(z3.ULT(x, z3.BitVecVal(5, 256))), B(z3.ULT(z3.BitVecVal(9, 256), x))])
    assert not c.is_possible()
    assert c.is_possible(solver_timeout=100) is True   # short custom timeout -> True (:44-46)
    assert SolverStatistics().gpu_sat == 0


def test_objectives_bypass_the_gpu(standin):
    """Minimising queries (analysis/solver.py:217-257) always go to z3 unchanged."""
    integration.install()
    opt = standin.funnel.Optimize()
    x = z3.BitVec("x", 256)
    opt.add(standin.Bool(z3.ULT(x, z3.BitVecVal(5, 256))))
    opt.minimize(standin.Bool(x))
    launches = standin.engine.launches
    assert opt.check() == z3.unknown
    assert standin.engine.launches == launches


def test_solver_timeout_becomes_the_device_deadline(standin, monkeypatch):
    """set_timeout(ms) (support/model.py:38) bounds the GPU search: check_sets receives a
    config whose timeout_ms is the solver timeout."""
    integration.install()
    seen = {}

    def fake_check(sets, registry=None, parents=None, config=None):
        seen["timeout"] = (config or gpu_check.CONFIG).timeout_ms
        return [None] * len(sets)

    monkeypatch.setattr(gpu_check, "check_sets", fake_check)
    opt = standin.funnel.Optimize()
    opt.set_timeout(1234)
    opt.add(standin.Bool(z3.ULT(z3.BitVec("x", 256), z3.BitVecVal(5, 256))))
    opt.check()
    assert seen["timeout"] == 1234


def test_tx_boundary_batch_over_world_states(standin):
    """stop_sym_trans hook -> one batch over the open WorldStates (svm.py:85,380:
    WorldState.constraints, world_state.py:39); the next iteration's is_possible() pass
    (svm.py:279-283) is answered from the parked witnesses without another search."""
    integration.install()
    B = standin.Bool
    cv = z3.BitVec("call_value1", 256)
    size = z3.BitVec("1_calldatasize", 256)
    states = [standin.WorldState([B(z3.ULT(cv, z3.BitVecVal(1000, 256))), B(cv != z3.BitVecVal(0, 256))]),
              standin.WorldState([B(z3.ULT(z3.BitVecVal(3, 256), size)), B(z3.ULT(size, z3.BitVecVal(68, 256)))]),
              standin.WorldState([B(z3.ULT(cv, z3.BitVecVal(5, 256))), B(z3.ULT(z3.BitVecVal(9, 256), cv))])]
    assert not hasattr(states[0], "world_state")
    laser_cls, builder_cls = integration._plugin_classes()

    class SVM:
        def __init__(self):
            self.hooks = {}
            self.open_states = states

        def laser_hook(self, name):
            def deco(fn):
                self.hooks.setdefault(name, []).append(fn)
                return fn
            return deco

    svm = SVM()
    builder_cls()().initialize(svm)
    svm.hooks["stop_sym_trans"][0]()
    launches = standin.engine.launches
    kept = [s for s in states if s.constraints.is_possible()]
    assert kept == states[:2]
    # no further search: witnesses were parked, and the contradiction's complete
    # (deadline-free) negative search is cached per search configuration
    assert standin.engine.launches == launches


def test_batch_cache_rechecks_and_is_cleared(standin):
    """A parked witness is returned only for the query it satisfies (re-checked), and a new
    batch drops the previous one's witnesses."""
    B = standin.Bool
    x = z3.BitVec("x", 256)
    s = standin.WorldState([B(z3.ULT(x, z3.BitVecVal(10, 256)))])
    kfm = standin.kfm
    assert integration.batch_open_states([s], kfm=kfm, registry=UFRegistry()) == 1
    terms = integration.state_terms(s)
    m = integration._lookup_batch(terms)
    assert m is not None
    # poison the parked model: a structurally different witness must fail the re-check
    key = integration._query_key(terms)
    bad = integration._BATCH_CACHE[key]
    bad.w.vars["x"] = 99
    bad.w._memo.clear()
    assert integration._lookup_batch(terms) is None
    integration.batch_open_states([], kfm=kfm, registry=UFRegistry())
    assert integration._BATCH_CACHE == {}


# ---- the same flows on the GPU ---------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_funnel_and_deepcopy(monkeypatch, engine):
    """The funnel with the rebound Optimize on the MI355X engine: GPU witness, ModelCache
    deep copy + completion, and the tx-boundary batch over WorldStates."""
    ns = mythril_standin.install(monkeypatch, z3)
    gpu_check.reset_cache()
    integration._BATCH_CACHE.clear()
    integration.install()
    B = ns.Bool
    x = z3.BitVec("call_value1", 256)
    c1 = ns.Constraints([B(z3.ULT(x, z3.BitVecVal(50, 256))), B(x != z3.BitVecVal(0, 256)),
                         B(z3.Not(z3.BVAddNoOverflow(x, z3.BitVecVal(2 ** 256 - 30, 256), False)))])
    assert c1.is_possible()
    model = list(ns.funnel.model_cache.model_cache.lru_cache.keys())[0]
    cp = copy.deepcopy(model)
    xv = cp.eval(x, model_completion=True).as_long()
    assert 30 <= xv < 50
    assert cp.eval(z3.BitVec("sender_9", 256), model_completion=True).as_long() == 0
    states = [ns.WorldState([B(z3.ULT(x, z3.BitVecVal(7, 256))), B(z3.ULT(z3.BitVecVal(5, 256), x))]),
              ns.WorldState([B(z3.ULT(x, z3.BitVecVal(5, 256))), B(z3.ULT(z3.BitVecVal(9, 256), x))])]
    assert integration.batch_open_states(states, kfm=ns.kfm, registry=UFRegistry()) == 1
    assert [s.constraints.is_possible() for s in states] == [True, False]


# ---- query accounting ---------------------------------------------------------
def _mythril_stats():
    import sys

    return sys.modules["mythril.laser.smt.solver.solver_statistics"].SolverStatistics()


def test_query_accounting_counts_each_query_once(standin):
    """GpuOptimize.check carries Mythril's own @stat_smt_query (solver_statistics.py:7-25)
    like BaseSolver.check (solver.py:72): a GPU-discharged query and a z3 fallback each
    bump query_count by exactly one (not two), and "% discharged" is gpu_sat / query_count."""
    integration.install()
    st = _mythril_stats()
    st.enabled = True                      # mythril_analyzer.py:147
    B = standin.Bool
    x = z3.BitVec("call_value1", 256)
    opt = standin.funnel.Optimize()
    opt.add(B(z3.ULT(x, z3.BitVecVal(50, 256))), B(x != z3.BitVecVal(0, 256)))
    assert opt.check() == z3.sat
    assert st.query_count == 1 and st.solver_time > 0
    opt2 = standin.funnel.Optimize()     # contradiction: no witness -> z3 (the stand-in: unknown)
    opt2.add(B(z3.ULT(x, z3.BitVecVal(5, 256))), B(z3.ULT(z3.BitVecVal(9, 256), x)))
    assert opt2.check() == z3.unknown
    assert st.query_count == 2
    opt3 = standin.funnel.Optimize()     # objectives: z3 only, still counted once
    opt3.add(B(z3.ULT(x, z3.BitVecVal(5, 256))))
    opt3.minimize(B(x))
    opt3.check()
    assert st.query_count == 3
    assert SolverStatistics().gpu_sat == 1
    assert integration.discharge_ratio() == pytest.approx(1 / 3)
    st.enabled = False
    opt.check()
    assert st.query_count == 3           # disabled statistics count nothing (:11-12)


def test_funnel_query_count_through_is_possible(standin):
    """Through the funnel (support/model.py:63-125): quick-sat hits never reach a solver, so
    only the GPU query is counted — what Mythril's printed statistics show
    (mythril_analyzer.py:187)."""
    integration.install()
    st = _mythril_stats()
    st.enabled = True
    B = standin.Bool
    x = z3.BitVec("call_value1", 256)
    assert standin.Constraints([B(z3.ULT(x, z3.BitVecVal(50, 256))), B(x != z3.BitVecVal(0, 256))]).is_possible()
    assert standin.Constraints([B(z3.ULT(x, z3.BitVecVal(60, 256))), B(x != z3.BitVecVal(0, 256))]).is_possible()
    assert st.query_count == 1
    assert integration.discharge_ratio() == 1.0


# ---- the witness eval never raises (support_utils.py:63-67 has no try) -------------------------
def _unsupported_pred(a, b):
    """A Bool operator outside the lowering's vocabulary (a signed-overflow predicate kind
    the converter has no entry for)."""
    d = z3.FuncDeclRef("bvsmul_noovfl", 0x7FFF, [a.sort(), b.sort()], z3.BoolSort())
    return z3._mk(d, [a, b])


def test_quick_sat_with_unsupported_op_moves_on_to_z3(standin):
    """A GPU model sits in model_cache; a later query with an operator the converter rejects
    is evaluated by check_quick_sat without raising (False: this model is skipped) and the
    funnel then asks the solver — z3's own ModelRef.eval would not raise either."""
    integration.install()
    B = standin.Bool
    x = z3.BitVec("call_value1", 256)
    assert standin.Constraints([B(z3.ULT(x, z3.BitVecVal(50, 256))), B(x != z3.BitVecVal(0, 256))]).is_possible()
    model = list(standin.funnel.model_cache.model_cache.lru_cache.keys())[0]
    odd = _unsupported_pred(x, z3.BitVecVal(3, 256))
    assert z3.is_false(model.eval(odd, model_completion=True))
    assert standin.funnel.model_cache.check_quick_sat(z3.And(odd, x != z3.BitVecVal(0, 256))) is False
    c = standin.Constraints([B(odd), B(x != z3.BitVecVal(0, 256))])
    assert c.is_possible(solver_timeout=100) is True   # reached the (stand-in) solver: unknown


def test_witness_eval_unsupported_op_by_substitution(standin):
    """Substitution + simplify decides what it can: an unsupported op over concrete values
    folds only if z3 folds it; a supported subterm still evaluates exactly."""
    x = z3.BitVec("call_value1", 256)
    internal = _witness_model([z3.ULT(x, z3.BitVecVal(1000, 256)), x != z3.BitVecVal(0, 256)])
    view = integration.Z3WitnessView(internal)
    xv = view.eval(x, model_completion=True).as_long()
    # a BitVec expression with an unsupported Bool inside: returned partially evaluated
    d = z3.FuncDeclRef("bvfoo", 0x7FFE, [x.sort()], x.sort())
    e = z3._mk(d, [x + 1])
    r = view.eval(e, model_completion=True)
    assert r.decl().name() == "bvfoo" and z3.is_bv_value(r.arg(0)) and r.arg(0).as_long() == xv + 1


def test_witness_eval_without_completion_returns_unassigned_symbols(standin):
    """model_completion=False (model.py:45-59 contract): a symbol the witness does not
    interpret comes back as itself, an expression over it partially evaluated; assigned
    symbols evaluate to their values."""
    x = z3.BitVec("call_value1", 256)
    internal = _witness_model([z3.ULT(x, z3.BitVecVal(1000, 256)), x != z3.BitVecVal(0, 256)])
    view = integration.Z3WitnessView(internal)
    other = z3.BitVec("sender_7", 256)
    assert view.eval(other, model_completion=False) is other
    assert view.eval(other, model_completion=True).as_long() == 0
    xv = view.eval(x, model_completion=False)
    assert z3.is_bv_value(xv) and 0 < xv.as_long() < 1000
    part = view.eval(other + x, model_completion=False)
    assert not z3.is_bv_value(part)
    assert any(z3.is_bv_value(a) and a.as_long() == xv.as_long() for a in part.children())


def test_batch_skips_states_that_do_not_convert(standin):
    """An open state with an unconvertible constraint is left to z3; the others are still
    batched (the hook must not abort the symbolic run, svm.py:306-307)."""
    B = standin.Bool
    x = z3.BitVec("x", 256)
    good = standin.WorldState([B(z3.ULT(x, z3.BitVecVal(10, 256)))])
    bad = standin.WorldState([B(_unsupported_pred(x, z3.BitVecVal(2, 256)))])
    assert integration.batch_open_states([bad, good], kfm=standin.kfm, registry=UFRegistry()) == 1
    assert integration._lookup_batch(integration.state_terms(good)) is not None


def test_batch_survives_an_engine_error(standin, monkeypatch):
    def boom(*a, **k):
        raise RuntimeError("device lost")

    monkeypatch.setattr(gpu_check, "check_sets", boom)
    B = standin.Bool
    s = standin.WorldState([B(z3.ULT(z3.BitVec("x", 256), z3.BitVecVal(10, 256)))])
    assert integration.batch_open_states([s], kfm=standin.kfm, registry=UFRegistry()) == 0


# ---- parent models in the live path (instructions.py:1638,1662) ------------------
def test_child_query_starts_from_the_parent_witness(standin, monkeypatch):
    """A child = the parent's constraints + one JUMPI condition.  With the host hints off,
    the bucket the condition changes starts its search from the parent's witness values
    (candidate 0 = the parent model), recorded from the parent query's witness."""
    from dataclasses import replace

    cfg = replace(gpu_check.CONFIG, hints=False, budget=4096)
    x = z3.BitVec("call_value1", 256)
    k1, k2 = 0xDEADBEEF_0000_1234_5678, 0x0BAD_F00D_9999_0000_0000_1111
    v = k1 ^ k2
    pc = (x ^ z3.BitVecVal(k1, 256)) == z3.BitVecVal(k2, 256)
    parent = converter(z3).terms([pc])
    # the generator does not find it from scratch at this budget (not a harvested constant) ...
    assert gpu_check.check_sets([parent], config=replace(cfg, parents=False))[0] is None
    # ... a z3 model of the parent (the funnel notes it, integration._note_z3_model)
    gpu_check.note_values({"call_value1": v})
    child = converter(z3).terms([pc, z3.ULT(z3.BitVecVal(5, 256), x)])
    m = gpu_check.check_sets([child], config=cfg)[0]
    assert m is not None and m.origin == "parent"
    assert m.w.vars["call_value1"] == v
    # a sibling whose new condition the parent value misses: mutations of it search on
    y = z3.BitVec("call_value2", 256)
    gpu_check.note_values({"call_value2": v})
    sib = converter(z3).terms([z3.Extract(255, 8, y) == z3.BitVecVal(v >> 8, 248),
                               z3.Extract(7, 0, y) != z3.BitVecVal(v & 0xFF, 8)])
    m2 = gpu_check.check_sets([sib], config=cfg)[0]
    assert m2 is not None and m2.origin == "search"
    assert (m2.w.vars["call_value2"] >> 8) == (v >> 8)


def test_gpu_witness_feeds_later_parents(standin):
    """Accepted witnesses are recorded per symbol: a later query over the same symbol gets
    them as its parent model."""
    x = z3.BitVec("call_value1", 256)
    m = _witness_model([z3.ULT(x, z3.BitVecVal(1000, 256)), x != z3.BitVecVal(0, 256)])
    got = gpu_check._recent_parent(converter(z3).terms([z3.ULT(x, z3.BitVecVal(7, 256))]))
    assert got == {"call_value1": m.w.vars["call_value1"]}
