#!/usr/bin/env python3
"""Summarise the PMC passes of tools/gpu_profile.sh into profiles/<tag>_pmc.{md,json}.

HBM traffic per launch: FETCH_SIZE (KiB, x2 — on gfx950 it reports half the bytes of wide
coalesced reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (KiB), each from its own pass,
averaged over the bench's dispatches — for pf_check_kernel (config 3) and
pf_keccak_fixed_kernel (config 4).  Hardware VALU view of pf_check_kernel: wave-level VALU
instructions per launch (SQ_INSTS_VALU, int64 ones separately) and the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / kernel time); bench.py turns them into the VALU issue-slot
fraction with its live kernel time."""
import csv
import collections
import json
import os
import sys

KERNEL = "pf_check_kernel"
F64_KEYS = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_CVT")
KECCAK = "pf_keccak_fixed_kernel"
# pf_check_kernel is the full sweep only (the early-exit legs launch pf_check_early_kernel):
# every one of its dispatches is the workload the roofline line is quoted on


def per_dispatch(path, kernel=KERNEL):
    agg = collections.OrderedDict()
    if not os.path.exists(path):
        return []
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        d = agg.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(agg.values())


def mean(rows, key):
    return sum(r[key] for r in rows) / len(rows)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csvp = lambda p: os.path.join(src, p, "run_counter_collection.csv")  # noqa: E731
    fetch = per_dispatch(csvp("fetch"))
    write = per_dispatch(csvp("write"))
    sq = per_dispatch(csvp("sq"))
    fetch_b = 2 * mean(fetch, "FETCH_SIZE") * 1024
    write_b = mean(write, "WRITE_SIZE") * 1024
    keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_SALU",
            "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"]
    sqm = {k: mean(sq, k) for k in keys}
    import subprocess
    head = subprocess.run(["git", "-C", root, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    out = {"kernel": KERNEL, "head": head, "dispatches": len(fetch), "fetch_bytes": fetch_b, "write_bytes": write_b,
           "traffic_bytes": fetch_b + write_b, "sq": sqm,
           "workload": "bench.py default (1024 config-3 DAGs x 65536 candidates, full sweep)"}
    clk = per_dispatch(csvp("clk"))
    if clk:
        out["clk"] = {k: mean(clk, k) for k in ("GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES",
                                                 "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU")}
    f64 = per_dispatch(csvp("f64"))
    if f64:
        out["f64"] = {k: mean(f64, k) for k in F64_KEYS if k in f64[0]}
        # (round 3 also wrote a cycle-weighted "VALU pipeline busy" here, priced at
        # tools/movbench.hip's 4-wave rates; those are latency-limited, not issue costs, so
        # the summary now reports only the issue-slot fraction at the VALU's 2 cycles per
        # wave64 instruction — MI355X_MICROARCH.md "Wave scheduling")
    kf, kw = per_dispatch(csvp("fetch"), KECCAK), per_dispatch(csvp("write"), KECCAK)
    if kf and kw:
        k = {"kernel": KECCAK, "fetch_bytes": 2 * mean(kf, "FETCH_SIZE") * 1024,
             "write_bytes": mean(kw, "WRITE_SIZE") * 1024}
        k["traffic_bytes"] = k["fetch_bytes"] + k["write_bytes"]
        out["keccak"] = k
    lines = [f"# {tag} — PMC passes of `bench.py --steps 2 --warmup 1` ({KERNEL})", "",
             "Each counter group is its own `rocprofv3 --pmc` run (tools/gpu_profile.sh).", "",
             "| quantity | per launch |", "|---|---|",
             f"| FETCH_SIZE x2 (gfx950 half-count correction) | {fetch_b / 1e6:.2f} MB |",
             f"| WRITE_SIZE | {write_b / 1e6:.2f} MB |"]
    for key in keys:
        lines.append(f"| {key} | {sqm[key]:.4g} |")
    if "clk" in out:
        for key, v in out["clk"].items():
            lines.append(f"| {key} (clock pass) | {v:.4g} |")
    for key, v in out.get("f64", {}).items():
        lines.append(f"| {key} (f64 pass) | {v:.4g} |")
    if "clk" in out:
        eff = out["clk"]["GRBM_GUI_ACTIVE"] / 8.0  # per-XCD cycles of the launch
        out["valu_issue_frac"] = 2.0 * out["clk"]["SQ_INSTS_VALU"] / (1024 * eff)
        lines.append(f"| VALU issue-slot fraction (2 cycles per wave64 instruction, 1024 SIMDs x {eff:.4g} "
                     f"cycles) | {out['valu_issue_frac']:.3f} |")
        if "f64" in out:
            n64 = sum(out["f64"].values())
            ni = sqm["SQ_INSTS_VALU_INT64"]
            lines.append(f"| of which v_mad_u64_u32-class (INT64) / f64+cvt instructions | "
                         f"{2.0 * ni / (1024 * eff):.3f} / {2.0 * n64 / (1024 * eff):.3f} |")
    w = sqm["SQ_WAVES"]
    lines += ["", f"per wave: {sqm['SQ_INSTS_VALU'] / w:.4g} VALU ({sqm['SQ_INSTS_VALU_INT64'] / w:.4g} int64), "
              f"{sqm['SQ_INSTS_SALU'] / w:.4g} SALU, {sqm['SQ_INSTS_BRANCH'] / w:.4g} branches, "
              f"{sqm['SQ_INSTS_SMEM'] / w:.4g} SMEM", ""]
    if "keccak" in out:
        k = out["keccak"]
        lines += [f"{KECCAK} per launch: FETCH_SIZE x2 {k['fetch_bytes'] / 1e6:.1f} MB + WRITE_SIZE "
                  f"{k['write_bytes'] / 1e6:.1f} MB (algorithmic: 96 B x 2^24 messages = 1610.6 MB)", ""]
    with open(os.path.join(root, "profiles", f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(root, "profiles", f"{tag}_pmc.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
