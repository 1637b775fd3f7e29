"""The native config-3 generator (pflt_synth, csrc/pf_terms.cpp) against synth.random_dag_set:
numpy's Philox Generator stream, the DAG builder, the planted values and the lowering restated
in C++ must give the same packed batch, DAG for DAG, unplanted and planted."""

import numpy as np
import pytest

from mythril_amd import ir, synth
from mythril_amd.smt import native_terms


def _batch_arrays(progs):
    b = ir.Batch(progs)
    return [np.asarray(x) for x in (b.code, b.consts, b.schema, b.parents, b.descs)]


@pytest.mark.parametrize("first,n,plant", [(0, 300, False), (0, 120, True), (999_700, 300, False),
                                           (123_456, 64, True), (4_000_000_000, 16, False)])
def test_native_generator_equals_python(first, n, plant):
    got = native_terms.synth_programs(first, n, plant, synth._MIX_CDF)
    if got is None:
        pytest.skip("libpflower.so without pflt_synth")
    progs, wit, nv = got
    py = [synth.random_dag_set(first + i, plant=plant) for i in range(n)]
    for i, (p, w) in enumerate(py):
        assert int(nv[i]) == len(w), first + i
        rows = wit[i, :len(w)].astype("<u4").tobytes()
        assert [int.from_bytes(rows[32 * v:32 * v + 32], "little") for v in range(len(w))] == w, first + i
    a, b = _batch_arrays(progs), _batch_arrays([p for p, _ in py])
    for x, y, name in zip(a, b, ("code", "consts", "schema", "parents", "descs")):
        assert x.shape == y.shape and np.array_equal(x, y), name


def test_random_dag_programs_wrapper():
    progs, wit = synth.random_dag_programs(10, 5, plant=True)
    for i in range(5):
        p, w = synth.random_dag_set(10 + i, plant=True)
        assert wit[i] == w
        assert [v.parent for v in progs[i].vars] == [v.parent for v in p.vars]
        assert progs[i].seed == p.seed
