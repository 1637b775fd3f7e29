#!/usr/bin/env python3
"""Where pf_check_kernel's time goes on the config-3 workload (diagnostic).

Builds (here, on the CPU: `python tools/unitprof.py --build`) a profiling variant of the
library, mythril_amd/libpathfeas_prof.so (-DPF_PROFILE_UNITS: every bytecode instruction's
s_memtime delta is accumulated per datapath unit in SGPRs), then on the GPU runs one batch
of config-3 DAGs and prints each unit's share of the waves' instruction time next to the
static instruction mix.  The product library is unaffected.
"""

import argparse
import ctypes
import json
import os
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROF_SO = os.path.join(ROOT, "mythril_amd", "libpathfeas_prof.so")
BUCKETS = ["ALU", "MUL", "DIV", "SHIFT", "GEN", "CMP", "BOOL", "END", "EXP", "CONST", "FETCH",
           "DIV_zero", "DIV_short", "DIV_onedigit", "DIV_general", "EXP_window", "EXP_t", "EXP_horner"]


def build():
    csrc = os.path.join(ROOT, "mythril_amd", "csrc")
    from mythril_amd.build import FLAGS, HIPCC  # the product's flags + the profiling define

    subprocess.run([HIPCC, *FLAGS, "-DPF_PROFILE_UNITS", "-o", PROF_SO,
                    os.path.join(csrc, "pathfeas.hip")], check=True, cwd=csrc)
    print(PROF_SO)


def run(args):
    from mythril_amd import _lib, ir, synth

    L = _lib.load_library(PROF_SO)
    L.pf_prof_read.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.pf_prof_read.restype = ctypes.c_int
    from mythril_amd.engine import Engine

    eng = Engine(0)
    progs = [synth.random_dag_set(i, plant=False)[0] for i in range(args.sets)]
    mix = Counter()
    for p in progs:
        for ins in p.code:
            mix[ir.OPNAMES[ins.op]] += 1
    db = eng.upload(progs)
    eng.check(db, budget=args.budget, seed=1, flags=ir.FLAG_COUNT_OPS)  # warm
    r = eng.check(db, budget=args.budget, seed=1, flags=ir.FLAG_COUNT_OPS)
    nb = len(BUCKETS)
    out = (ctypes.c_uint64 * (nb + 1))()
    _lib.check(L.pf_prof_read(db.handle, out), "pf_prof_read")
    tot_ins = sum(out[:15])  # the EXP_* buckets are parts of EXP
    wave = out[nb]
    res = {"kernel_ms": r.kernel_ms, "wave_cycles": wave, "instr_cycles": tot_ins,
           "share": {BUCKETS[i]: round(out[i] / max(tot_ins, 1), 4) for i in range(len(BUCKETS))},
           "mix_per_set": {k: round(v / len(progs), 2) for k, v in mix.most_common()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--sets", type=int, default=512)
    ap.add_argument("--budget", type=int, default=65536)
    a = ap.parse_args()
    build() if a.build else run(a)
