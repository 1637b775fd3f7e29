"""One process driving several GPUs (SURVEY §8e partitioning for the live analysis: Mythril is
one process, so a tx-boundary batch is split across the node's devices inside
libpathfeas.so — pf_init(device_mask), pf_batch_create_on, pf_check_batches).

CPU: the size-balanced split and the gather logic of Engine.upload_sharded / check_many and
of gpu_check.check_sets on a stand-in engine with several "devices" (the C oracle per shard)
give exactly the single-device verdicts and witnesses.
GPU: on the one visible device, a one-bit mask engine and two batches searched through
pf_check_batches give identical results to the single-batch path.
"""

import numpy as np
import pytest

import oracle_engine
from mythril_amd import engine as E
from mythril_amd import ir, synth
from mythril_amd.dist import shard_bounds
from mythril_amd.smt import gpu_check


def _progs(n, first=0, plant=True):
    return [synth.random_dag_set(first + i, plant=plant)[0] for i in range(n)]


def test_shards_balance_the_cost_model():
    progs = _progs(24)
    costs = [p.sched_cost() for p in progs]
    b = shard_bounds(costs, 4)
    assert b[0][0] == 0 and b[-1][1] == len(progs)
    assert all(b[i][1] == b[i + 1][0] for i in range(3))
    loads = [sum(costs[lo:hi]) for lo, hi in b]
    assert max(loads) - min(loads) <= max(costs) + 1


class _MultiOracle(oracle_engine.OracleEngine):
    """The oracle engine with n "devices": upload_sharded / check_many follow Engine's code."""

    def __init__(self, n):
        super().__init__()
        self.devices = list(range(n))
        self.device = 0
        self.uploads = []

    def upload(self, programs, device=None):
        db = super().upload(programs)
        db.device = self.device if device is None else device
        self.uploads.append((db.device, len(db)))
        return db

    upload_sharded = E.Engine.upload_sharded

    def check_many(self, dbs, budget=65536, seed=0, flags=2, timeout_ms=0):
        rs = [self.check(db, budget, seed, flags, timeout_ms) for db in dbs]
        return E.CheckResult(np.concatenate([r.found for r in rs]), 0, 0, 0, 0.0, False)


def test_check_sets_sharded_equals_single(monkeypatch):
    """The same constraint sets through check_sets on 1 and on 3 stand-in devices: identical
    verdicts and witness values; each device got one contiguous shard."""
    import pyoracle as O
    from mythril_amd import corpus
    from mythril_amd import keccak_manager as KM
    from mythril_amd.smt import symbol_factory

    # concrete hashes from the oracle's Keccak (the product computes them on the GPU)
    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))
    c = corpus.build(6, 2, seed=7)
    sets = [q.constraints for q in c.queries][:60]
    results = {}
    for n in (1, 3):
        eng = _MultiOracle(n)
        monkeypatch.setattr(E, "get_engine", lambda device=None, eng=eng: eng)
        monkeypatch.setattr(gpu_check.CONFIG, "workers", 1)
        monkeypatch.setattr(gpu_check.CONFIG, "budget", 2048)
        gpu_check.reset_cache()
        ms = gpu_check.check_sets(sets, registry=c.kfm.registry)
        results[n] = [None if m is None else sorted(m.w.vars.items()) for m in ms]
        if n == 3:
            assert sorted(d for d, _ in eng.uploads) == [0, 1, 2]
    assert results[1] == results[3]
    assert any(r is not None for r in results[1])
    gpu_check.reset_cache()


def test_device_spec_from_environment(monkeypatch):
    seen = {}

    class _E:
        def __init__(self, device=0, devices=None):
            seen["devices"] = devices if devices is not None else [device]

    monkeypatch.setattr(E, "Engine", _E)
    monkeypatch.setattr(E, "_engine", None)
    monkeypatch.setenv("PF_DEVICES", "0,2,5")
    E.get_engine()
    assert seen["devices"] == [0, 2, 5]
    monkeypatch.setattr(E, "_engine", None)
    monkeypatch.delenv("PF_DEVICES")
    monkeypatch.setenv("LOCAL_RANK", "3")
    E.get_engine()
    assert seen["devices"] == [3]
    monkeypatch.setattr(E, "_engine", None)


@pytest.mark.gpu
def test_gpu_mask_engine_and_check_many(engine):
    """A one-bit device-mask engine (the visible GPU) and pf_check_batches over two batches
    on it reproduce the single-batch verdicts exactly."""
    progs = _progs(96, first=500, plant=False)
    eng = E.Engine(devices=[0])
    whole = eng.upload(progs)
    r1 = eng.check(whole, budget=4096, seed=0, flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)
    a, b = eng.upload(progs[:40], device=0), eng.upload(progs[40:], device=0)
    r2 = eng.check_many([a, b], budget=4096, seed=0, flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)
    assert np.array_equal(r1.found, r2.found)
    assert r2.cands_decided > 0
    # check_each (bench steps): the batches enqueued back to back on one stream, each with
    # its own verdicts and counters — the full sweep too
    for flags in (ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT, 0):
        ra, rb = eng.check(a, budget=4096, seed=0, flags=flags), eng.check(b, budget=4096, seed=0, flags=flags)
        each = eng.check_each([a, b], budget=4096, seed=0, flags=flags)
        assert [len(r.found) for r in each] == [40, 56]
        assert np.array_equal(each[0].found, ra.found) and np.array_equal(each[1].found, rb.found)
        assert (each[0].evals_full, each[1].evals_full) == (ra.evals_full, rb.evals_full)
        assert each[0].kernel_ms > 0 and each[1].kernel_ms > 0
    for db in (whole, a, b):
        db.free()


def test_plugin_batch_spreads_over_all_visible_devices(monkeypatch):
    """The live analysis is one process: once the plugin is loaded (install() defaults
    PF_DEVICES to "all"), the engine it gets drives every visible device, and a
    tx-boundary batch (stop_sym_trans hook, svm.py:306-307) is split into one shard per
    device — 3 stand-in devices here."""
    import fake_z3 as z3
    import mythril_standin
    from mythril_amd import _lib, integration

    ns = mythril_standin.install(monkeypatch, z3)
    made = {}

    def fake_engine(device=0, devices=None):
        made["devices"] = devices
        eng = _MultiOracle(len(devices))
        made["eng"] = eng
        return eng

    class _L:
        def pf_device_count(self):
            return 3

    monkeypatch.setattr(_lib, "lib", lambda: _L())
    monkeypatch.setattr(E, "Engine", fake_engine)
    monkeypatch.setattr(E, "_engine", None)
    monkeypatch.setattr(gpu_check.CONFIG, "workers", 1)
    monkeypatch.setattr(gpu_check.CONFIG, "budget", 1024)
    monkeypatch.setattr(integration, "sync_keccak_registry", lambda kfm, registry=None: None)
    gpu_check.reset_cache()
    B = ns.Bool
    states = []
    for k in range(12):
        x = z3.BitVec(f"call_value{k}", 256)
        states.append(ns.WorldState([B(z3.ULT(x, z3.BitVecVal(100 + k, 256))),
                                     B(z3.ULT(z3.BitVecVal(k, 256), x))]))

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
    integration._plugin_classes()[1](**{})().initialize(svm)
    svm.hooks["stop_sym_trans"][0]()
    assert made["devices"] == [0, 1, 2]
    assert sorted({d for d, _ in made["eng"].uploads}) == [0, 1, 2]
    assert all(s.constraints.is_possible() for s in states)
    monkeypatch.setattr(E, "_engine", None)
    gpu_check.reset_cache()


@pytest.mark.gpu
def test_gpu_two_contexts_on_one_device(engine, monkeypatch):
    """The node split as it runs on a multi-GPU box, on the one visible GPU: the device named
    twice (PF_DEVICES=0,0) makes two execution contexts (pf_init_contexts), each with its own
    stream.  upload_sharded cuts the batch into two cost-balanced shards, one per context,
    pf_check_batches enqueues both before reading either, and the gathered verdicts equal the
    single-context search — bare programs and check_sets' whole pipeline alike."""
    progs = _progs(160, first=900, plant=False)
    flags = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT
    one = E.Engine(devices=[0])
    whole = one.upload(progs)
    r1 = one.check(whole, budget=8192, seed=0, flags=flags)
    two = E.Engine(devices=[0, 0])
    assert len(two.devices) == 2 and len(set(two.devices)) == 2 and min(two.devices) >= 64
    dbs = two.upload_sharded(progs)
    assert len(dbs) == 2 and sum(len(d) for d in dbs) == len(progs)
    assert [d.device for d in dbs] == two.devices
    r2 = two.check_many(dbs, budget=8192, seed=0, flags=flags)
    assert np.array_equal(r1.found, r2.found)
    # the witnesses materialise from either context's batch
    sat = [k for k in range(len(progs)) if r2.found[k] != E.NOT_FOUND]
    assert sat
    k0 = sat[0]
    base = 0 if k0 < len(dbs[0]) else len(dbs[0])
    db = dbs[0] if k0 < len(dbs[0]) else dbs[1]
    assert two.materialize(db, [k0 - base], [int(r2.found[k0])]) == \
        one.materialize(whole, [k0], [int(r1.found[k0])])
    for d in dbs + [whole]:
        d.free()
    # check_sets through an engine of two contexts: the same answers as through one
    import pyoracle as O
    from mythril_amd import corpus
    from mythril_amd import keccak_manager as KM
    from mythril_amd.smt import symbol_factory

    monkeypatch.setattr(KM.KeccakFunctionManager, "find_concrete_keccak", staticmethod(
        lambda data: symbol_factory.BitVecVal(
            int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)))
    c = corpus.build(6, 2, seed=7)
    sets = [q.constraints for q in c.queries][:80]
    answers = {}
    for name, eng in (("one", one), ("two", two)):
        monkeypatch.setattr(E, "get_engine", lambda device=None, eng=eng: eng)
        gpu_check.reset_cache()
        ms = gpu_check.check_sets(sets, registry=c.kfm.registry)
        answers[name] = [None if m is None else sorted(m.w.vars.items()) for m in ms]
    assert answers["one"] == answers["two"]
    assert any(a is not None for a in answers["one"])
    gpu_check.reset_cache()


@pytest.mark.gpu
def test_gpu_batch_uploads_while_contexts_are_added(engine):
    """pf_batch_create runs its device lookup and upload without the library lock, so it can
    race a pf_init_contexts that grows the device table.  The table's entries are
    heap objects that never move and the lookup holds the table's own lock: uploads on one
    thread while another adds contexts must neither crash nor mix up devices, and every
    batch still searches to the single-thread answer."""
    import threading

    from mythril_amd import _lib

    progs = _progs(24, first=1700, plant=True)
    flags = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT
    ref = engine.check(engine.upload(progs), budget=1024, seed=0, flags=flags).found
    errors = []
    stop = threading.Event()

    def add_contexts():
        try:
            for k in range(1, 9):   # distinct device tuples: each call adds contexts
                _lib.init_contexts([0] * k)
                if stop.is_set():
                    break
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    t = threading.Thread(target=add_contexts)
    t.start()
    try:
        for _ in range(12):
            db = engine.upload(progs)
            got = engine.check(db, budget=1024, seed=0, flags=flags).found
            db.free()
            assert np.array_equal(got, ref)
    finally:
        stop.set()
        t.join()
    assert not errors, errors
