"""The soundness half of "% discharged": queries that are UNSAT by construction — the
reference's UNSAT KATs (tests/laser/keccak_tests.py, tests/laser/state/calldata_test.py,
rebuilt with the facade) and planted contradictions over the corpus' SAT queries
(mythril_amd.corpus.labelled_unsat) — are never answered sat.  CPU: the host pipeline on
the C oracle; GPU: on the MI355X engine (bench.py reports the same count).  Also checks that
witnesses carry their provenance (hint model vs search)."""

import pytest

import oracle_engine
import pyoracle as O
from mythril_amd import corpus
from mythril_amd import keccak_manager as KM
from mythril_amd.smt import gpu_check, symbol_factory
from mythril_amd.smt import terms as T


def _host_keccak(monkeypatch):
    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))


def _run(c, unsat):
    fps, n = [], 0
    for reg in {id(r): r for _, _, r in unsat}.values():
        group = [(cs, o) for cs, o, r in unsat if r is reg]
        ms = gpu_check.check_sets([cs for cs, _ in group], registry=reg)
        n += len(group)
        fps += [o for (cs, o), m in zip(group, ms) if m is not None]
    return fps, n


def test_labelled_unsat_never_sat_cpu(monkeypatch):
    _host_keccak(monkeypatch)
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(gpu_check.CONFIG, "budget", 4096)
    c = corpus.build(6, 2, seed=11)
    unsat = corpus.labelled_unsat(c, n=48, seed=5)
    assert sum(o.startswith("kat:") for _, o, _ in unsat) == 8
    fps, n = _run(c, unsat)
    assert n == len(unsat) and fps == []
    ms = gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
    kinds = {m.origin for m in ms if m is not None}
    assert kinds <= {"hint", "first", "search", "cache"} and kinds
    gpu_check.reset_cache()


@pytest.mark.gpu
def test_labelled_unsat_never_sat_gpu(engine):
    gpu_check.reset_cache()
    c = corpus.build(12, 2, seed=11)
    unsat = corpus.labelled_unsat(c, n=256, seed=5)
    fps, n = _run(c, unsat)
    assert fps == [], fps[:3]
    gpu_check.reset_cache()


def test_union_of_bucket_witnesses_satisfies_the_set(monkeypatch):
    """check_sets trusts the union of per-bucket re-checked witnesses (independence makes
    it a model of the set); re-evaluating every constraint under the union changes nothing."""
    _host_keccak(monkeypatch)
    oracle_engine.install(monkeypatch)
    monkeypatch.setattr(gpu_check.CONFIG, "budget", 1024)
    c = corpus.build(6, 2, seed=23)
    qs = [q.constraints for q in c.queries]
    gpu_check.reset_cache()
    fast = gpu_check.check_sets(qs, registry=c.kfm.registry)
    gpu_check.reset_cache()
    monkeypatch.setattr(gpu_check.CONFIG, "recheck_union", True)
    full = gpu_check.check_sets(qs, registry=c.kfm.registry)
    got = [m is not None for m in fast]
    assert got == [m is not None for m in full] and sum(got) > len(qs) // 2
    for m in fast:
        if m is not None:
            assert all(m.w.ev(cs) for cs in m.constraints if cs is not T.TRUE)
    gpu_check.reset_cache()
