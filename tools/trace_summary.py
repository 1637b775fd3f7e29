#!/usr/bin/env python3
"""Kernel-trace summary of a `rocprofv3 --kernel-trace --stats` run (tools/gpu_profile.sh
pass 1) into profiles/<tag>_bench_kernel_trace.md: calls, total and average duration per
kernel from the rocpd database's `kernels` view (durations in ns), and — for the two kernels
the bench line carries a live time for — the TIMED launches alone.

The bench launches each of them `warmup` times untimed, then `steps` timed launches
(bench.py run(): warm-up checks, then the K timed steps; keccak_leg: warmup + steps launches,
the first `warmup` not averaged).  Averaging every call mixes the warm-ups in (the first
launch pays the code-object load and cold caches), so the timed rows take, in start order,
launches [warmup, warmup + steps) of each kernel and report their median and mean — the
figures to set beside the line's `roofline.kernel_ms_avg` / `keccak.kernel_ms_avg`.

    python tools/trace_summary.py gpurun_out/prof_<tag>/trace <tag> [--warmup 2 --steps 5]
"""
import argparse
import glob
import json
import os
import sqlite3
import statistics

TIMED = ("pf_check_kernel", "pf_keccak_fixed_kernel")


def short(n):
    return n.split("(")[0] if n.startswith("pf_") else n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("tag")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--bench-line", default=None,
                    help="the bench JSON line of the traced run (to set its kernel_ms_avg beside)")
    a = ap.parse_args()
    db = sorted(glob.glob(os.path.join(a.src, "*.db")))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = [f"# {a.tag} kernel trace: bench --steps {a.steps} --warmup {a.warmup}", "",
             f"source: `{a.src}` (rocprofv3 --kernel-trace --stats; durations from the rocpd `kernels` view)", "",
             "## Timed launches only", "",
             f"Launches [{a.warmup}, {a.warmup + a.steps}) of each kernel in start order (the bench's "
             "timed steps; the first launches are its untimed warm-ups).", "",
             "| kernel | timed calls | median (ms) | mean (ms) | min (ms) | max (ms) | bench line (ms) | line / median |",
             "|---|---|---|---|---|---|---|---|"]
    line_ms = {}
    if a.bench_line and os.path.exists(a.bench_line):
        with open(a.bench_line) as f:
            txt = [ln for ln in f.read().splitlines() if ln.startswith("{")]
        if txt:
            d = json.loads(txt[-1])
            line_ms["pf_check_kernel"] = d.get("roofline", {}).get("kernel_ms_avg")
            line_ms["pf_keccak_fixed_kernel"] = (d.get("keccak") or {}).get("kernel_ms_avg")
    summary = {}
    for k in TIMED:
        durs = [r[1] / 1e6 for r in c.execute(
            f"select start, end - start from kernels where {name} like ? order by start", (k + "%",)).fetchall()]
        timed = durs[a.warmup:a.warmup + a.steps]
        if not timed:
            continue
        med, mean = statistics.median(timed), statistics.fmean(timed)
        ref = line_ms.get(k)
        summary[k] = {"timed_calls": len(timed), "median_ms": med, "mean_ms": mean,
                      "all_calls_mean_ms": statistics.fmean(durs), "bench_line_ms": ref}
        lines.append(f"| {k} | {len(timed)} | {med:.3f} | {mean:.3f} | {min(timed):.3f} | {max(timed):.3f} | "
                     f"{'' if ref is None else f'{ref:.3f}'} | {'' if ref is None else f'{ref / med:.4f}'} |")
    lines += ["", "## Every call", "", "| kernel | calls | total (ms) | average (ms) | % |", "|---|---|---|---|---|"]
    for n, k, s, av in rows:
        lines.append(f"| {short(n)} | {k} | {s / 1e6:.3f} | {av / 1e6:.3f} | {100 * s / tot:.2f} |")
    out = os.path.join(root, "profiles", f"{a.tag}_bench_kernel_trace.md")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(root, "profiles", f"{a.tag}_bench_kernel_trace.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main()
