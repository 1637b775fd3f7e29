"""The split candidate-0 probe (gpu_check._probe_candidate0): a single query's long hinted
bucket is decided at candidate 0 by its per-conjunct explicit programs side by side
(pf_eval_programs) instead of a lone wave walking the whole program — on the C oracle here,
the same verdicts, witnesses and re-checks as without it."""

from dataclasses import replace

import pytest

import oracle_engine
from mythril_amd import corpus
from mythril_amd.smt import gpu_check


@pytest.fixture(scope="module")
def corp():
    with pytest.MonkeyPatch.context() as mp:   # the corpus hashes through the engine
        oracle_engine.install(mp)
        return corpus.build(8, 2, seed=2024)


def test_probe_decides_long_hinted_buckets_like_the_search(corp, monkeypatch):
    oracle_engine.install(monkeypatch)
    _compare(corp, [q for q in corp.queries if q.label == "sat"][:24])


def _compare(corp, qs):
    got = {}
    for pm in (0, 400):
        gpu_check.STATS.__init__()
        cfg = replace(gpu_check.CONFIG, probe_min_ins=pm)
        out = []
        for q in qs:
            gpu_check.reset_cache()
            m = gpu_check.check_sets([q.constraints], registry=corp.kfm.registry, config=cfg)[0]
            out.append(None if m is None else (m.origin, tuple(sorted(str(d) for d in m.decls()))))
        got[pm] = (out, gpu_check.STATS.probe_split, gpu_check.STATS.probe_split_sat,
                   gpu_check.STATS.recheck_failures)
    assert got[0][0] == got[400][0]                 # same answers, same provenance
    assert got[0][1] == 0 and got[400][1] > 0 and got[400][2] == got[400][1]
    assert got[400][3] == 0


def test_probe_stays_out_of_batches(corp, monkeypatch):
    oracle_engine.install(monkeypatch)
    gpu_check.reset_cache()
    gpu_check.STATS.__init__()
    gpu_check.check_sets([q.constraints for q in corp.queries[:40]], registry=corp.kfm.registry)
    assert gpu_check.STATS.probe_split == 0


@pytest.mark.gpu
def test_gpu_probe_decides_long_hinted_buckets_like_the_search(corp, engine):
    """The same on the MI355X: pf_eval_programs' verdict at candidate 0 and the search's."""
    _compare(corp, [q for q in corp.queries if q.label == "sat"][:48])
