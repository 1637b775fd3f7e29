#!/usr/bin/env python3
"""Spill census of config-3 programs: how many sets spill, which slots, and
how many spill live ranges (SPILL .. FILL of a slot) cross an instruction that uses EXP's
LDS table entries (W_EXP, B_UMUL_NOOVF) — the ranges an LDS spill slot in those entries
could not hold.

    python tools/spill_scan.py [--dags 2000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import ir, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dags", type=int, default=2000)
    args = ap.parse_args()
    progs, _ = synth.random_dag_programs(0, args.dags, plant=False)
    b = ir.Batch(progs)
    fills = crossing = 0
    max_slot = []
    for s in range(len(progs)):
        off, n = int(b.descs[s][0]), int(b.descs[s][1])
        ops = (b.code[off:off + n, 0] & 0xFF).tolist()
        aux = b.code[off:off + n, 2].tolist()
        open_, ms = {}, -1
        for i, (op, a) in enumerate(zip(ops, aux)):
            if op in (ir.W_SPILL, ir.B_SPILL):
                open_[a] = i
                ms = max(ms, a)
            elif op in (ir.W_FILL, ir.B_FILL) and a in open_:
                fills += 1
                crossing += any(o in (ir.W_EXP, ir.B_UMUL_NOOVF) for o in ops[open_[a]:i])
        max_slot.append(ms)
    ms = np.array(max_slot)
    print(json.dumps({"dags": args.dags, "sets_spilling": float((ms >= 0).mean()),
                      "sets_by_highest_slot": {("none" if k == 0 else str(k - 1)): int(v)
                                              for k, v in enumerate(np.bincount(ms + 1)) if v},
                      "fills": fills, "fills_per_set": fills / args.dags,
                      "ranges_crossing_exp_table_users": crossing,
                      "crossing_frac": crossing / max(fills, 1)}))


if __name__ == "__main__":
    main()
