"""GPU parity at scale: the search kernels' smallest witness index against the C oracle
(oracle/coracle.c, the same restatement the CPU tests pin against pyoracle and the
reference's vectors) over hundreds of config-3 sets — every candidate before the first
witness is an evaluation the two must agree on.  Both register files (8-register kernels,
3 waves/SIMD, and 16-register kernels), with and without early exit / short-circuit, and
LASER-shaped sets.  Bit-exact: integer work, no tolerance.  (The host lowering bug fixed in
round 2 — one config-3 DAG in ~30,000 — was found by the 1M-DAG planted pass; this test is
the per-commit guard on the kernel side.)"""

import coracle_py
import numpy as np
import pytest

from mythril_amd import ir, synth
from mythril_amd.lower import lower

pytestmark = pytest.mark.gpu

BUDGET, SEED = 4096, 0x5EED_0F_5CA1E


def _dag(dag_id, plant):
    got = {}
    orig = synth.lower
    synth.lower = lambda dag, **k: got.setdefault("dag", dag) and orig(dag, **k)
    try:
        prog = synth.random_dag_set(dag_id, plant=plant)[0]
    finally:
        synth.lower = orig
    return got["dag"], prog


def _oracle_first(progs, budget, seed):
    pk = coracle_py.Packed(ir.Batch(progs))
    return [pk.first_sat(s, seed, budget) for s in range(len(progs))]


def _compare(engine, progs, flags, want):
    res = engine.check(engine.upload(progs), budget=BUDGET, seed=SEED, flags=flags)
    got = [None if f == 0xFFFFFFFF else int(f) for f in res.found]
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:10]
    return got


@pytest.fixture(scope="module")
def config3():
    dags = [_dag(20_000 + 7 * i, plant=(i % 5 == 0)) for i in range(768)]
    progs = [p for _, p in dags]
    return dags, progs, _oracle_first(progs, BUDGET, SEED)


@pytest.mark.parametrize("flags", [0, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT])
def test_config3_sets_match_oracle(engine, config3, flags):
    _, progs, want = config3
    got = _compare(engine, progs, flags, want)
    assert sum(g is not None for g in got) > len(progs) // 4  # a real mix of SAT and not


def test_config3_wide_register_file_matches_oracle(engine, config3):
    dags, _, _ = config3
    wide = [lower(d, nw=ir.NW) for d, _ in dags[:256]]
    _compare(engine, wide, ir.FLAG_EARLY_EXIT, _oracle_first(wide, BUDGET, SEED))


def test_laser_shaped_sets_match_oracle(engine):
    progs = [synth.mythril_like_set(i) for i in range(96)]
    _compare(engine, progs, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT,
             _oracle_first(progs, BUDGET, SEED))


def test_early_exit_large_batch_matches_full_sweep(engine, config3):
    """A batch big enough that the early-exit work queue grows its chunks (pathfeas.hip
    geometry(): at most 64 items per wave; 4,608 sets x 1,024 groups -> 16-group chunks):
    the smallest witness of every set equals the full sweep's, and the oracle's below 4,096."""
    _, progs, want = config3
    big = progs * 6
    b = engine.upload(big)
    full = [int(f) for f in engine.check(b, budget=65536, seed=SEED, flags=0).found]
    early = [int(f) for f in engine.check(b, budget=65536, seed=SEED,
                                          flags=ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT).found]
    bad = [(i, f, e) for i, (f, e) in enumerate(zip(full, early)) if f != e]
    assert not bad, bad[:10]
    for i, f in enumerate(early):
        w = want[i % len(progs)]
        assert f == w if w is not None else (f == 0xFFFFFFFF or f >= BUDGET), (i, f, w)
