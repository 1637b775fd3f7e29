"""check_sets' native pipeline (include/pf_lower.h "batches": pflt_lower_many, pflt_pack_batch,
pflt_recheck_many, the recent-value tables behind parent models) against the Python pipeline
it replaces (gpu_check with _NATIVE_TERMS off: to_dag/seed/lower, ir.Batch, interp.Witness,
_note_witness/_recent_parent): the same programs and batch arrays, the same re-check
verdicts, the same parent models through LRU eviction, and the same answers, witness values
and provenance over the corpus in live order (fork pairs one call at a time, parents on).
The device is the C oracle (tests/oracle_engine.py)."""

import random

import numpy as np
import pytest

import oracle_engine

from mythril_amd import corpus, ir
from mythril_amd.lower import LoweringError
from mythril_amd.smt import gpu_check
from mythril_amd.smt import native_terms as NT
from mythril_amd.smt import terms as T
from mythril_amd.smt.independence import buckets
from mythril_amd.smt.interp import Witness

pytestmark = pytest.mark.skipif(NT.batch_api() is None, reason="libpflower.so without the batch API")


@pytest.fixture(scope="module")
def small_corpus():
    import mythril_amd.engine as E

    eng = oracle_engine.OracleEngine()
    saved = E.get_engine
    E.get_engine = lambda device=None: eng
    try:
        c = corpus.build(6, 2, seed=5)
    finally:
        E.get_engine = saved
    bks, seen = [], set()
    for q in c.queries:
        for b in buckets(q.constraints):
            if tuple(b) not in seen:
                seen.add(tuple(b))
                bks.append(b)
    return c, bks


def test_lower_many_matches_single_lowering(small_corpus):
    """Threaded pflt_lower_many = pflt_lower per bucket: same programs, variables, metadata."""
    c, bks = small_corpus
    reg = c.kfm.registry
    seeds = [gpu_check._set_seed(b) for b in bks]
    many = NT.lower_many([(b, None) for b in bks], reg, True, seeds, 8)
    assert len(many) == len(bks)
    ok = 0
    for b, s, (lo, prog, err) in zip(bks, seeds, many):
        try:
            lo1, prog1 = NT.lower_bucket(b, reg, None, True, s)
        except LoweringError as e:
            assert lo is None and err == str(e)
            continue
        ok += 1
        assert err is None
        np.testing.assert_array_equal(prog.words, prog1.words)
        assert prog.consts == prog1.consts and prog.vars == prog1.vars and prog.seed == prog1.seed
        assert prog.has_parent == prog1.has_parent
        assert lo.var_terms == lo1.var_terms and lo.uf_apps == lo1.uf_apps
        assert lo.array_reads == lo1.array_reads
    assert ok > 0.9 * len(bks)


def test_pack_batch_matches_python_batch(small_corpus):
    c, bks = small_corpus
    reg = c.kfm.registry
    many = [x for x in NT.lower_many([(b, None) for b in bks], reg, True,
                                     [gpu_check._set_seed(b) for b in bks], 4) if x[2] is None]
    progs = [p for _, p, _ in many]
    nat = ir.Batch(progs)
    py = ir.Batch([ir.PackedProgram(p.words, list(p.consts), list(p.vars), p.seed) for p in progs])
    for f in ("code", "consts", "schema", "parents", "descs"):
        np.testing.assert_array_equal(getattr(nat, f), getattr(py, f), err_msg=f)
    # hints off: no parent values at all
    many = [x for x in NT.lower_many([(b, None) for b in bks[:30]], reg, False, [7] * 30, 4) if x[2] is None]
    progs = [p for _, p, _ in many]
    nat = ir.Batch(progs)
    py = ir.Batch([ir.PackedProgram(p.words, list(p.consts), list(p.vars), p.seed) for p in progs])
    for f in ("code", "consts", "schema", "parents", "descs"):
        np.testing.assert_array_equal(getattr(nat, f), getattr(py, f), err_msg=f)


def test_recheck_many_matches_witness(small_corpus):
    """pflt_recheck_many's verdicts = interp.Witness on every conjunct, for hint models and
    random assignments, batched over many results at once."""
    c, bks = small_corpus
    reg = c.kfm.registry
    rng = random.Random(3)
    many = [x for x in NT.lower_many([(b, None) for b in bks], reg, True, [5] * len(bks), 4) if x[2] is None]
    for trial in range(3):
        los, rows, want = [], [], []
        for lo, prog, _ in many:
            if trial == 0:
                vals = [v.parent or 0 for v in prog.vars]
            else:
                vals = [rng.choice((0, 1, 4, 68, rng.getrandbits(v.width))) & ir.mask(v.width) for v in prog.vars]
            los.append(lo)
            rows.append(ir.limbs_array(vals) if vals else np.zeros((0, 8), dtype=np.uint32))
            bucket = [t for t in lo.res.get(NT.GET_IN_ROOTS, lo.res.info[14], 1).tolist()]
            want.append(all(bool(Witness(lo, vals, reg).ev(NT.store().terms[t])) for t in bucket))
        got = NT.recheck_many(los, np.concatenate(rows), reg, 8)
        assert got.tolist() == [1 if w else 0 for w in want]
        if trial == 0:
            assert sum(want) > 0.8 * len(want)


def _py_recent(seq, recent_size):
    """The Python tables after a sequence of notes (gpu_check._note_witness / note_values)."""
    gpu_check._RECENT_VARS.clear()
    gpu_check._RECENT_READS.clear()
    cfg = gpu_check.GpuConfig(recent_size=recent_size)
    for kind, lo, vals in seq:
        if kind == "z3":
            for k, v in vals.items():
                gpu_check._RECENT_VARS[k] = v
                gpu_check._RECENT_VARS.move_to_end(k)
            while len(gpu_check._RECENT_VARS) > recent_size:
                gpu_check._RECENT_VARS.popitem(last=False)
        else:
            gpu_check._note_witness(lo._get(), vals, cfg)


def test_recent_parents_match_python_tables(small_corpus, monkeypatch):
    """pflt_note_result / pflt_note_vars / pflt_recent_parent keep the Python tables' LRU
    contents: after witnesses and z3 models are noted (with eviction at a small
    recent_size), every bucket gets the same parent model."""
    c, bks = small_corpus
    reg = c.kfm.registry
    rng = random.Random(8)
    many = [x for x in NT.lower_many([(b, None) for b in bks], reg, False, [1] * len(bks), 4) if x[2] is None]
    seq = []
    for lo, prog, _ in many[:80]:
        vals = [rng.getrandbits(v.width) for v in prog.vars]
        seq.append(("w", lo, vals))
        if rng.random() < 0.2:
            names = [t.val for t in lo.var_terms if t.op == "var"][:3]
            seq.append(("z3", None, {n: rng.getrandbits(256) for n in names}))
    for recent_size in (16, 1 << 14):
        # native tables
        NT.recent_clear()
        for kind, lo, vals in seq:
            if kind == "z3":
                NT.note_vars(vals, recent_size)
            else:
                NT.note_result(lo, ir.limbs_array(vals) if vals else np.zeros((0, 8), np.uint32), recent_size)
        nat = []
        for b in bks:
            h = NT.recent_parent_handle(b)
            nat.append(None if h is None else NT.parent_dict(h))
            NT.free_parent(h)
        # the Python tables, queried by the Python _recent_parent
        monkeypatch.setattr(gpu_check, "_NATIVE_TERMS", False)
        _py_recent(seq, recent_size)
        py = [gpu_check._recent_parent(b) for b in bks]
        monkeypatch.setattr(gpu_check, "_NATIVE_TERMS", True)
        assert nat == py
        assert sum(p is not None for p in py) > 0.3 * len(bks)
    NT.recent_clear()
    gpu_check.reset_cache()


def _live(monkeypatch, native, groups, reg):
    monkeypatch.setattr(gpu_check, "_NATIVE_TERMS", native)
    gpu_check.reset_cache()
    gpu_check.STATS.recheck_failures = 0
    from dataclasses import replace

    cfg = replace(gpu_check.CONFIG, hints=False, parents=True, budget=512, workers=4)
    out = []
    for g in groups:
        out += gpu_check.check_sets([q.constraints for q in g], registry=reg, config=cfg)
    return out


def test_live_order_answers_match_python_pipeline(small_corpus, monkeypatch):
    """The corpus in live order (hints off, parents on: parent models decide what the search
    finds) answers the same through both pipelines — same sets discharged, same provenance,
    same witness values."""
    eng = oracle_engine.install(monkeypatch)
    c, _ = small_corpus
    groups = corpus.live_order_groups(c.queries)[:40]
    nat = _live(monkeypatch, True, groups, c.kfm.registry)
    assert gpu_check.STATS.recheck_failures == 0
    py = _live(monkeypatch, False, groups, c.kfm.registry)
    assert gpu_check.STATS.recheck_failures == 0
    assert [m is None for m in nat] == [m is None for m in py]
    assert [m.origin for m in nat if m] == [m.origin for m in py if m]
    assert sum(m is not None for m in nat) > 0.5 * len(nat)
    assert any(m.origin == "parent" for m in nat if m)
    for a, b in zip(nat, py):
        if a is not None:
            assert a.w.vars == b.w.vars and a.w.bools == b.w.bools and a.w.reads == b.w.reads
    assert eng.launches > 0
    gpu_check.reset_cache()


def test_candidate_zero_witnesses_are_not_materialised(small_corpus, monkeypatch):
    """A query whose witnesses are all candidate 0 of fully parented programs (the hint
    model held) reads them from the host's parent values: no materialise launch.  The
    answers and witness values are those of the Python pipeline, which materialises all."""
    c, _ = small_corpus
    qs = [q.constraints for q in c.queries][:24]
    eng = oracle_engine.install(monkeypatch)
    launches = []
    orig = eng.materialize_limbs
    monkeypatch.setattr(eng, "materialize_limbs", lambda *a, **k: launches.append(1) or orig(*a, **k))
    before = gpu_check.STATS.bucket_origin.get("hint", 0)
    nat = []
    for q in qs:
        gpu_check.reset_cache()
        nat += gpu_check.check_sets([q], registry=c.kfm.registry)
    answered = sum(m is not None for m in nat)
    assert gpu_check.STATS.bucket_origin.get("hint", 0) > before and len(launches) < answered
    monkeypatch.setattr(gpu_check, "_NATIVE_TERMS", False)
    py = []
    for q in qs:
        gpu_check.reset_cache()
        py += gpu_check.check_sets([q], registry=c.kfm.registry)
    assert [m is None for m in nat] == [m is None for m in py]
    for a, b in zip(nat, py):
        if a is not None:
            assert a.w.vars == b.w.vars


def test_worker_pool_survives_fork(small_corpus):
    """a forked child of a process that used the persistent worker pool (the
    default fork context of tools/full_pass.py's ProcessPoolExecutor) lowers on host threads
    too — it gets a fresh pool instead of waiting for the parent's workers, which it lacks."""
    import os
    import signal

    c, bks = small_corpus
    reg = c.kfm.registry
    jobs = [(b, None) for b in bks[:24]]
    NT.lower_many(jobs, reg, True, [3] * len(jobs), 8)      # the parent's pool is running
    pid = os.fork()
    if pid == 0:   # child: the same call, bounded by an alarm
        signal.alarm(60)
        try:
            out = NT.lower_many(jobs, reg, True, [3] * len(jobs), 8)
            os._exit(0 if len(out) == len(jobs) else 2)
        except BaseException:
            os._exit(3)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
