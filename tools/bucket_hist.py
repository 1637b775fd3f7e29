"""Development aid: size and opcode mix of the programs the discharge pipeline lowers for
one corpus query (host only; the C-oracle keccak stands in for the GPU's)."""

import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import discharge_oracle as D  # noqa: E402

from mythril_amd import corpus, ir  # noqa: E402
from mythril_amd.smt.gpu_check import _lower_bucket  # noqa: E402
from mythril_amd.smt.independence import buckets  # noqa: E402


def main():
    D.host_keccak()
    c = corpus.build(24, 2, seed=2024)
    pick = sys.argv[1] if len(sys.argv) > 1 else "tx2-boundary"
    qs = [q for q in c.queries if pick in q.origin]
    q = qs[min(3, len(qs) - 1)]
    print(q.origin, len(q.constraints), "constraints")
    for b in buckets(q.constraints):
        lo, p = _lower_bucket(b, c.kfm.registry, None, True)
        h = Counter(ir.OPNAMES[i.op] for i in p.code)
        print(f"  {len(b)} constraints, {len(lo.dag.nodes)} nodes, {len(p.code)} ins, "
              f"{len(p.vars)} vars: {h.most_common(10)}")


if __name__ == "__main__":
    main()
