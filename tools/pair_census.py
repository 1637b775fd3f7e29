#!/usr/bin/env python3
"""Instruction and dependent-pair census of config-3 device programs (pf_device_program:
the programs the kernel runs, after pf_batch_create's peepholes) — which back-to-back pairs
a fused instruction would cover (lever "fused instruction pairs").

A pair (a, b) is counted when b immediately follows a and reads a's destination register in
the same register file.  Static counts over the programs (no early exit).

    python tools/pair_census.py [--dags 2000] [--top 25]
"""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import _lib, ir, synth  # noqa: E402

I_KA, I_KB = 1 << 25, 1 << 26   # w0 device flags: operand a / b is a folded constant


def device_program(b):
    L = _lib.lib()
    code = np.ascontiguousarray(b.code, dtype=np.uint32)
    descs = np.ascontiguousarray(b.descs, dtype=np.uint32)
    consts = np.ascontiguousarray(b.consts, dtype=np.uint32)
    out = np.zeros_like(code)
    dout = np.zeros_like(descs)
    n = ctypes.c_size_t()
    _lib.check(L.pf_device_program(_lib.ptr_u32(code), len(code), _lib.ptr_u32(consts.reshape(-1)), len(consts),
                                   _lib.ptr_u32(descs), len(descs), _lib.ptr_u32(out), ctypes.byref(n),
                                   _lib.ptr_u32(dout)), "pf_device_program")
    return out[:n.value], dout


def is_b(op):
    return op >= ir.B_CONST


def reads(op, w1):
    """(register file, register) operands read by an instruction."""
    a, bb, c = (w1 >> 8) & 0xFF, (w1 >> 16) & 0xFF, (w1 >> 24) & 0xFF
    if op in ir.W_BINARY:
        return [("W", a), ("W", bb)]
    if op in ir.W_UNARY or op in (ir.W_EXTRACT, ir.W_SEXT, ir.W_SPILL):
        return [("W", a)]
    if op == ir.W_CONCAT:
        return [("W", a), ("W", bb)]
    if op == ir.W_ITE:
        return [("B", a), ("W", bb), ("W", c)]
    if op in (ir.B_EQ, ir.B_ULT, ir.B_ULE, ir.B_SLT, ir.B_SLE, ir.B_UADD_NOOVF, ir.B_UMUL_NOOVF):
        return [("W", a), ("W", bb)]
    if op in ir.B_LOGIC:
        return [("B", a), ("B", bb)]
    if op in (ir.B_NOT, ir.B_SPILL, ir.ASSERT):
        return [("B", a)]
    if op == ir.B_ITE:
        return [("B", a), ("B", bb), ("B", c)]
    return []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dags", type=int, default=2000)
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    progs, _ = synth.random_dag_programs(0, args.dags, plant=False)
    code, descs = device_program(ir.Batch(progs))
    ops = collections.Counter()
    pairs = collections.Counter()
    total = 0
    for s in range(len(descs)):
        off, n = int(descs[s][0]), int(descs[s][1])
        prev = None
        for i in range(off, off + n):
            w0, w1 = int(code[i][0]), int(code[i][1])
            op = w0 & 0xFF
            if op == ir.END:
                break
            total += 1
            ops[ir.OPNAMES.get(op, op)] += 1
            if prev is not None:
                pop, pdst = prev
                pf = "B" if is_b(pop) else "W"
                rd = reads(op, w1)
                if w0 & I_KA and rd:      # operand a / b is a constant index (PF_I_KA / KB)
                    rd[0] = None
                if w0 & I_KB and len(rd) > 1:
                    rd[1] = None
                if (pf, pdst) in rd:
                    pairs[(ir.OPNAMES.get(pop, pop), ir.OPNAMES.get(op, op))] += 1
            prev = (op, w1 & 0xFF)
    print(f"{args.dags} DAGs, {total} device instructions ({total / args.dags:.1f} per program)")
    print("ops:", ", ".join(f"{k} {v / total:.3f}" for k, v in ops.most_common(20)))
    print("dependent back-to-back pairs (share of instructions):")
    for (a, b), v in pairs.most_common(args.top):
        print(f"  {a:>14} -> {b:<14} {v / total:.3f}")


if __name__ == "__main__":
    main()
