#!/usr/bin/env python3
"""Wave-time shares of pf_check_kernel from one SQ PMC pass (tools/gpu_stalls.sh):
ACTIVE_INST_* / WAIT_* over SQ_WAVE_CYCLES, averaged over the bench's dispatches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import mean, per_dispatch  # noqa: E402

rows = per_dispatch(os.path.join(sys.argv[1], "run_counter_collection.csv"))
keys = sorted({k for r in rows for k in r})
wc = mean(rows, "SQ_WAVE_CYCLES")
print("| counter | per launch | share of SQ_WAVE_CYCLES |\n|---|---|---|")
for k in keys:
    v = mean(rows, k)
    print(f"| {k} | {v:.4g} | {100 * v / wc:.1f}% |")
