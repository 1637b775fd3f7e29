"""Probe: derive the hint model of a LASER-shaped constraint set and report which roots it
satisfies (host only; development aid for mythril_amd/seed.py)."""

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import seed  # noqa: E402
from mythril_amd.smt import (UGE, ULT, Array, Concat, If, Not, Or, UDiv,  # noqa: E402
                             symbol_factory)
from mythril_amd.smt.to_dag import ACTORS, TermLowering  # noqa: E402

BVV = symbol_factory.BitVecVal
BV = symbol_factory.BitVecSym


def main():
    cd = Array("1_calldata", 256, 8)
    size = BV("1_calldatasize", 256)

    def word(off):
        return Concat([If(BVV(off + i, 256) < size, cd[BVV(off + i, 256)], BVV(0, 8)) for i in range(32)])

    sel = UDiv(word(0), BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)
    caller = BV("sender_1", 256)
    val = BV("call_value1", 256)
    bal = Array("balance", 256, 256)
    cs = [Or(*[caller == BVV(a, 256) for a in ACTORS]),
          UGE(bal[caller], val),
          Not(ULT(size, BVV(4, 256))),
          sel == BVV(0xA9059CBB, 256),
          If(val == BVV(0, 256), BVV(1, 256), BVV(0, 256)) != BVV(0, 256),
          ULT(word(4), BVV(1000, 256)),
          Not(word(36) == BVV(0, 256)),
          caller == BVV(ACTORS[1], 256)]
    lo = TermLowering().lower([c.raw for c in cs])
    t = time.time()
    ok = seed.apply_hints(lo.dag)
    dt = time.time() - t
    print(f"roots satisfied by the hint model: {ok} of {len(set(lo.dag.roots))}  "
          f"({dt * 1e3:.1f} ms, {len(lo.dag.nodes)} nodes)")
    for v in lo.dag.vars:
        if v.parent:
            print(f"  {v.name} = {v.parent:#x}")


if __name__ == "__main__":
    main()
