"""Division census of the config-3 workload (host only; tools, not product).

For a sample of config-3 DAGs and 64-candidate waves, record every division node's
operands per lane (through the oracle's evaluator) and classify each (wave, node) by the
path pf::udivrem256 takes: all-zero quotient, short (every divisor one limb), one-digit
(every quotient one digit), general.  For the general path report the quotient digits the
wave cannot skip and the widest divisor, which is what the wave pays for.

usage: python tools/divcensus.py [n_dags] [waves_per_dag]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as po  # noqa: E402
from mythril_amd import ir, synth  # noqa: E402

DIVS = {po.OP["W_UDIV"]: "u", po.OP["W_UREM"]: "u", po.OP["W_SDIV"]: "s",
        po.OP["W_SREM"]: "s", po.OP["W_SMOD"]: "s"}


def limbs(x):
    return (x.bit_length() + 31) // 32


def main():
    n_dags = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    waves = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    progs = [synth.random_dag_set(i, plant=False)[0] for i in range(n_dags)]
    batch = ir.Batch(progs)
    rec = []
    orig = dict(po._WBIN)

    def wrap(op, f, kind):
        def g(a, b, w):
            if kind == "s":
                sa, sb = po.to_signed(a, w), po.to_signed(b, w)
                rec.append((op, abs(sa), abs(sb)))
            else:
                rec.append((op, a, b))
            return f(a, b, w)
        return g

    for op, kind in DIVS.items():
        po._WBIN[op] = wrap(op, orig[op], kind)
    paths = collections.Counter()
    gen_digits = collections.Counter()
    gen_nmax = collections.Counter()
    lane_cls = collections.Counter()
    gen_cls = collections.Counter()
    gen_multi_maxdig = collections.Counter()
    gen_multi_span = collections.Counter()
    work_uniform = work_lane = work_nmax = work_split = work_nbound = work_two = work_pow = 0
    for s in range(n_dags):
        sv = po.SetView.from_batch(batch, s)
        for wv in range(waves):
            base = wv * 4096
            cands = np.arange(base, base + 64, dtype=np.uint64)
            per_lane = []
            for a in sv.gen_assignments(cands, 0):
                rec.clear()
                sv.evaluate(a)
                per_lane.append(list(rec))
            for k in range(len(per_lane[0])):
                ops = [pl[k] for pl in per_lane]
                live = [(a, b) for (_, a, b) in ops if b != 0 and a >= b]
                for (_, a, b) in ops:
                    if b == 0 or a < b:
                        lane_cls["q0"] += 1
                    elif b < 2**32:
                        lane_cls["short"] += 1
                    elif a.bit_length() <= b.bit_length() + 31:
                        lane_cls["onedigit"] += 1
                    else:
                        lane_cls["multi"] += 1
                if not live:
                    paths["zero"] += 1
                elif all(b < 2**32 for (_, _, b) in ops):
                    paths["short"] += 1
                elif all(a.bit_length() <= b.bit_length() + 31 for (a, b) in live):
                    paths["onedigit"] += 1
                else:
                    paths["general"] += 1
                    digs = set()
                    for (a, b) in live:
                        q = a // b
                        for j in range(8):
                            if (q >> (32 * j)) & 0xFFFFFFFF:
                                digs.add(j)
                    gen_digits[len(digs)] += 1
                    cls = frozenset("short" if b < 2**32 else ("one" if a.bit_length() <= b.bit_length() + 31 else "multi") for (a, b) in live)
                    gen_cls[tuple(sorted(cls))] += 1
                    md = [len([j for j in range(8) if ((a // b) >> (32 * j)) & 0xFFFFFFFF]) for (a, b) in live if b >= 2**32 and a.bit_length() > b.bit_length() + 31]
                    if md:
                        gen_multi_maxdig[max(md)] += 1
                        gen_multi_span[max(a.bit_length() - b.bit_length() for (a, b) in live if b >= 2**32 and a.bit_length() > b.bit_length() + 31) // 32 + 1] += 1
                    nmax = max(limbs(b) for (_, b) in live)
                    gen_nmax[nmax] += 1
                    work_uniform += sum(9 - j for j in digs)
                    for j in digs:
                        work_nmax += max(limbs(b) for (a, b) in live if ((a // b) >> (32 * j)) & 0xFFFFFFFF) + 1
                    for j in digs:
                        nb = 1 + max(limbs(b) for (a, b) in live if limbs(b) <= 8 - j)
                        work_two += 2 if nb <= 2 else 9 - j
                        work_pow += min(9 - j, 2 if nb <= 2 else (5 if nb <= 5 else 9))
                        work_nbound += min(9 - j, 1 + max(limbs(b) for (a, b) in live if limbs(b) <= 8 - j))
                    sh = [(a, b) for (a, b) in live if b >= 2**32]
                    dg = set(j for (a, b) in sh for j in range(8) if ((a // b) >> (32 * j)) & 0xFFFFFFFF)
                    work_split += sum(9 - j for j in dg)
                    work_lane += max(sum(limbs(b) + 1 for j in range(8) if ((a // b) >> (32 * j)) & 0xFFFFFFFF)
                                     for (a, b) in live)
    tot = sum(paths.values())
    print("divisions (wave x node):", tot)
    for k, v in paths.most_common():
        print(f"  path {k:9s} {v:6d}  {100 * v / tot:5.1f}%")
    lt = sum(lane_cls.values())
    print("lanes:", {k: f"{100 * v / lt:.1f}%" for k, v in lane_cls.items()})
    print("general: digits processed", sorted(gen_digits.items()))
    print("general: widest divisor limbs", sorted(gen_nmax.items()))
    print("general: lane classes present", gen_cls.most_common())
    print("general: multi lanes' max nonzero digits", sorted(gen_multi_maxdig.items()))
    print("general: multi lanes' max quotient span (digits)", sorted(gen_multi_span.items()))
    print("general: limb-steps, uniform (9-j per digit) vs widest lane only:", work_uniform, work_lane)
    print("general: limb-steps with per-digit width n_max_j + 1:", work_nmax, " short lanes split off:", work_split)
    print("general: limb-steps with width 1 + max{n <= 8 - j} over live lanes:", work_nbound, "two widths {2, 9-j}:", work_two, "three widths {2,5,9}:", work_pow)


if __name__ == "__main__":
    main()
