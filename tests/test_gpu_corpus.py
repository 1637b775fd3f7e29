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
