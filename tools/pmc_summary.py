#!/usr/bin/env python3
"""Summarise the PMC passes of tools/gpu_profile.sh into profiles/<tag>_pmc.{md,json}.

HBM traffic per launch of pf_check_kernel: FETCH_SIZE (KiB, x2 — on gfx950 it reports half the
bytes of wide coalesced reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (KiB), each from its own
pass, averaged over the bench's dispatches."""
import csv
import collections
import json
import os
import sys

KERNEL = "pf_check_kernel"


def per_dispatch(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        d = agg.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(agg.values())


def mean(rows, key):
    return sum(r[key] for r in rows) / len(rows)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fetch = per_dispatch(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = per_dispatch(os.path.join(src, "write", "run_counter_collection.csv"))
    sq = per_dispatch(os.path.join(src, "sq", "run_counter_collection.csv"))
    fetch_b = 2 * mean(fetch, "FETCH_SIZE") * 1024
    write_b = mean(write, "WRITE_SIZE") * 1024
    keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_SALU",
            "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"]
    sqm = {k: mean(sq, k) for k in keys}
    out = {"kernel": KERNEL, "dispatches": len(fetch), "fetch_bytes": fetch_b, "write_bytes": write_b,
           "traffic_bytes": fetch_b + write_b, "sq": sqm,
           "workload": "bench.py default (1024 config-3 DAGs x 65536 candidates, full sweep)"}
    with open(os.path.join(root, "profiles", f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    lines = [f"# {tag} — PMC passes of `bench.py --steps 2 --warmup 1` ({KERNEL})", "",
             "Each counter group is its own `rocprofv3 --pmc` run (tools/gpu_profile.sh).", "",
             "| quantity | per launch |", "|---|---|",
             f"| FETCH_SIZE x2 (gfx950 half-count correction) | {fetch_b / 1e6:.2f} MB |",
             f"| WRITE_SIZE | {write_b / 1e6:.2f} MB |"]
    for k in keys:
        lines.append(f"| {k} | {sqm[k]:.4g} |")
    w = sqm["SQ_WAVES"]
    lines += ["", f"per wave: {sqm['SQ_INSTS_VALU'] / w:.4g} VALU ({sqm['SQ_INSTS_VALU_INT64'] / w:.4g} int64), "
              f"{sqm['SQ_INSTS_SALU'] / w:.4g} SALU, {sqm['SQ_INSTS_BRANCH'] / w:.4g} branches, "
              f"{sqm['SQ_INSTS_SMEM'] / w:.4g} SMEM", ""]
    with open(os.path.join(root, "profiles", f"{tag}_pmc.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
