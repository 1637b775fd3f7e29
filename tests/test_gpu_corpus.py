"""GPU: the discharge pipeline on LASER-shaped queries (mythril_amd/corpus.py) through the
drop-in funnel ``get_models`` — independence buckets, hint models, ONE search launch,
witness materialisation and host re-check (mythril_amd/smt/gpu_check.py).

Soundness: every returned model satisfies its query under Model.eval (the host restatement
of the kernel's interpretation).  Coverage: at least 90 % of the planted-SAT queries are
discharged (the remainder exceed the lowering's register + spill capacity and go to z3).
"""

import pytest

from mythril_amd import corpus
from mythril_amd.smt import gpu_check
from mythril_amd.smt.model import Model
from mythril_amd.support.model import get_models

pytestmark = pytest.mark.gpu


def test_corpus_discharge_and_models(engine):
    c = corpus.build(12, 2, seed=5)
    corpus.validate(c)
    gpu_check.reset_cache()
    models = get_models([q.constraints for q in c.queries], registry=c.kfm.registry)
    planted = [(m, q) for m, q in zip(models, c.queries) if q.label == "sat"]
    hit = sum(1 for m, _ in planted if m is not None)
    assert hit >= 0.9 * len(planted), (hit, len(planted))
    for m, q in zip(models, c.queries):
        if m is None:
            continue
        assert isinstance(m, Model)
        for t in q.constraints:
            assert bool(m.eval(t)), q.origin


def test_bucket_cache_answers_repeated_queries(engine, monkeypatch):
    """A repeated batch is answered from the bucket caches: never a lost witness, and with
    parent models off (a deterministic search) exactly the same answers.  With parents on, a
    re-posed query may gain a witness — its new buckets start from the first pass's."""
    c = corpus.build(4, 2, seed=9)
    sets = [q.constraints for q in c.queries]
    for parents in (False, True):
        monkeypatch.setattr(gpu_check.CONFIG, "parents", parents)
        gpu_check.reset_cache()
        first = get_models(sets, registry=c.kfm.registry)
        hits0 = gpu_check.STATS.bucket_hits
        again = get_models(sets, registry=c.kfm.registry)
        assert gpu_check.STATS.bucket_hits > hits0
        assert all(a is not None for a, f in zip(again, first) if f is not None)
        if not parents:
            assert [m is None for m in first] == [m is None for m in again]
    assert gpu_check.STATS.recheck_failures == 0


def _run_pipeline(eng, c, cfg, live):
    """check_sets over the corpus (one batch, or fork pairs one call at a time in live
    order) on ``eng``; returns the verdicts, witness values, the bucket cache's witnesses and
    every launch's per-bucket smallest witness indices."""
    from mythril_amd.smt import native_terms

    launches = []
    orig = eng.check

    def check(db, *a, **k):
        r = orig(db, *a, **k)
        launches.append(r.found.tolist())
        return r

    eng.check = check
    try:
        gpu_check.reset_cache()
        groups = corpus.live_order_groups(c.queries) if live else [c.queries]
        models = []
        for g in groups:
            models += gpu_check.check_sets([q.constraints for q in g], registry=c.kfm.registry, config=cfg)
    finally:
        eng.check = orig
    verdicts = [m is not None for m in models]
    values = [dict(m.w.vars) if m is not None else None for m in models]

    def ints(v):
        return native_terms.ints_of(v) if hasattr(v, "dtype") else [int(x or 0) for x in v]

    cache = {k: ints(v) for k, (_, v) in gpu_check._CACHE.items()}
    return verdicts, values, cache, launches


@pytest.mark.parametrize("hints,parents,live", [(True, False, False), (False, False, False),
                                                (False, True, True)])
def test_gpu_pipeline_equals_oracle_pipeline(engine, monkeypatch, hints, parents, live):
    """The same discharge pipeline (independence buckets, hint models, parent models, native
    lowering, batch packing, witness materialisation and re-check) with only the engine
    swapped — the MI355X kernel vs the C oracle (tests/oracle_engine.py) — gives identical
    per-query verdicts and witness values, identical bucket witnesses, and identical
    smallest witness indices in every launch: ref support_utils.py:57-71's predicate on
    LASER shapes, end to end."""
    from dataclasses import replace

    import oracle_engine
    import mythril_amd.engine as E

    c = corpus.build(6, 2, seed=7)
    cfg = replace(gpu_check.CONFIG, hints=hints, parents=parents, budget=2048, timeout_ms=0)
    gpu = _run_pipeline(E.get_engine(), c, cfg, live)
    ora_eng = oracle_engine.OracleEngine()
    monkeypatch.setattr(E, "get_engine", lambda device=None: ora_eng)
    ora = _run_pipeline(ora_eng, c, cfg, live)
    gpu_check.reset_cache()
    assert gpu[0] == ora[0]
    assert gpu[1] == ora[1]
    assert gpu[2] == ora[2]
    assert gpu[3] == ora[3]
    assert sum(gpu[0]) > 0 and len(gpu[3]) > 0
