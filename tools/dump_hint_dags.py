"""Dump the hint solver's inputs (packed DAG nodes, constant pool, roots, variable widths and
soft values: pfl_hints' arguments) of the largest bucket of chosen single-query sample
queries (tools/sq_tail.py numbering) to gpurun_out/hint_dags.npz, so pfl_hints can be timed
and profiled on any host.  GPU-box tool (the corpus build hashes on the engine).

usage: python tools/dump_hint_dags.py i,j,..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import corpus  # noqa: E402
from mythril_amd.lower import limbs, pack_nodes  # noqa: E402
from mythril_amd.smt import native_terms, terms as T  # noqa: E402
from mythril_amd.smt.to_dag import TermLowering  # noqa: E402

idx = [int(i) for i in sys.argv[1].split(",")]
c = corpus.build(48, 2, seed=2024)
sample = [q for q in c.queries if q.label == "sat"][:96]
out = {}
for i in idx:
    cs = [x for x in sample[i].constraints if x is not T.TRUE]
    bk = max(native_terms.buckets(cs), key=len)
    dag = TermLowering(c.kfm.registry, None).lower(list(bk)).dag
    nodes, pool_a, pool = pack_nodes(dag)
    out[f"q{i}_nodes"] = nodes
    out[f"q{i}_pool"] = pool_a
    out[f"q{i}_roots"] = np.array(dag.roots or [0], dtype=np.uint32)
    out[f"q{i}_widths"] = np.array([v.width for v in dag.vars], dtype=np.uint32)
    out[f"q{i}_soft"] = limbs([(v.parent or 0) & ((1 << v.width) - 1) for v in dag.vars])
    out[f"q{i}_meta"] = np.array([len(dag.nodes), len(pool), len(dag.roots), len(dag.vars)], dtype=np.uint64)
    print(f"q{i}: {len(dag.nodes)} nodes, {len(dag.vars)} vars, {len(dag.roots)} roots")
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/hint_dags.npz", **out)
