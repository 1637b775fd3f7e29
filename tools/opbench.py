#!/usr/bin/env python3
"""Per-opcode throughput of pf_check_kernel (diagnostic, not the headline bench).

For each opcode: sets whose program is a 32-deep chain x = op(x, y) over two generated
256-bit variables, searched over 65,536 candidates with early exit off.  Reports algorithmic
int32 ops/s, node-evaluations/s and the implied cycles per node per wave.
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import ir  # noqa: E402
from mythril_amd.engine import Engine  # noqa: E402
from mythril_amd.lower import Dag, lower  # noqa: E402

OPS = {
    "add": ir.W_ADD, "sub": ir.W_SUB, "and": ir.W_AND, "xor": ir.W_XOR, "mul": ir.W_MUL,
    "udiv": ir.W_UDIV, "urem": ir.W_UREM, "sdiv": ir.W_SDIV, "shl": ir.W_SHL,
    "lshr": ir.W_LSHR, "ashr": ir.W_ASHR, "exp": ir.W_EXP, "hash": ir.W_HASH,
    "ult_ite": "ult_ite", "var": "var", "concat8": "concat8",
    "udiv_q1": "udiv_q1", "udiv_q8": "udiv_q8",
    "add4": "add4", "mul4": "mul4", "add1": "add1", "mul1": "mul1",
}


def chain_program(kind, depth, seed):
    dag = Dag()
    x = dag.var("x", 256)
    y = dag.var("y", 256)
    if kind in ("add4", "mul4", "add1", "mul1"):
        # hand-scheduled bytecode (the lowering's post-order would serialise the chains):
        # "*4" = 4 interleaved independent chains (consecutive instructions independent),
        # "*1" = the same instruction count as one dependent chain
        op = ir.W_ADD if kind.startswith("add") else ir.W_MUL
        p = ir.Program(vars=[ir.Var("y", 256), ir.Var("x", 256)], seed=seed)
        p.emit(ir.W_VAR, 256, dst=0, aux0=0)
        p.emit(ir.W_VAR, 256, dst=1, aux0=1)
        for k in range(2, 5):
            p.emit(ir.W_ADD, 256, dst=k, a=1, b=0)
        for i in range(depth):
            r = 1 + (i % 4) if kind.endswith("4") else 1
            p.emit(op, 256, dst=r, a=r, b=0)
        p.emit(ir.B_EQ, 256, dst=0, a=1, b=2)
        p.emit(ir.ASSERT, 1, a=0)
        return p.finish()
    for i in range(depth):
        if kind == "ult_ite":
            c = dag.op(ir.B_ULT, 256, x, y)
            x = dag.op(ir.W_ITE, 256, c, dag.op(ir.W_XOR, 256, x, y), x)
        elif kind == "var":
            x = dag.op(ir.W_XOR, 256, x, dag.var(f"v{i}", 256))
        elif kind == "concat8":
            x = dag.op(ir.W_CONCAT, 256, dag.op(ir.W_EXTRACT, 248, x, aux=0),
                       dag.op(ir.W_EXTRACT, 8, y, aux=i % 32), aux=8)
        elif kind in ("udiv_q1", "udiv_q8"):
            # fresh 256-bit numerator each step; divisor y >> 8 (1 quotient digit) or
            # y mod 2^32 (7-8 digits)
            num = dag.op(ir.W_XOR, 256, x, y)
            den = (dag.op(ir.W_LSHR, 256, y, dag.const(8, 256)) if kind == "udiv_q1" else
                   dag.op(ir.W_AND, 256, y, dag.const(0xFFFFFFFF, 256)))
            x = dag.op(ir.W_UDIV, 256, num, den)
        elif kind == ir.W_HASH:
            x = dag.op(ir.W_HASH, 256, x, aux=i)
        elif kind == ir.W_SHL or kind == ir.W_LSHR or kind == ir.W_ASHR:
            x = dag.op(kind, 256, x, dag.op(ir.W_AND, 256, y, dag.const(0xFF, 256)))
        else:
            x = dag.op(kind, 256, x, y)
    dag.assert_(dag.op(ir.B_EQ, 256, x, dag.const(12345, 256)))
    return lower(dag, seed=seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=512)
    ap.add_argument("--budget", type=int, default=65536)
    ap.add_argument("--depth", type=int, default=32)
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--lib", default=None, help="alternative build of libpathfeas.so (variants)")
    args = ap.parse_args()
    if args.lib:
        from mythril_amd import _lib

        _lib.load_library(args.lib)
    eng = Engine(0)
    out = {}
    for name in args.ops.split(","):
        kind = OPS[name]
        depth = 4 if name == "exp" else args.depth
        progs = [chain_program(kind, depth, s) for s in range(args.sets)]
        db = eng.upload(progs)
        eng.check(db, budget=args.budget, seed=1, flags=ir.FLAG_COUNT_OPS)  # warm
        r = eng.check(db, budget=args.budget, seed=2, flags=ir.FLAG_COUNT_OPS)
        s = r.kernel_ms / 1e3
        nodes = sum(len(p.code) for p in progs) * args.budget
        # cycles per instruction per wave: 256 CU * 4 SIMD * 2.4e9 cycles/s over waves
        waves_instr = nodes / 64
        cyc = (s * 256 * 4 * 2.4e9) / waves_instr
        out[name] = {"kernel_ms": r.kernel_ms, "tops": r.ops / s / 1e12,
                     "frac_int32_peak": r.ops / s / (256 * 4 * 32 * 2.4e9),
                     "instr_per_s": nodes / s, "simd_cycles_per_wave_instr": cyc}
        print(name, json.dumps(out[name]), flush=True)
        db.free()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
