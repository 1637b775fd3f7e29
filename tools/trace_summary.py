#!/usr/bin/env python3
"""Kernel-trace summary of a `rocprofv3 --kernel-trace --stats` run (tools/gpu_profile.sh
pass 1) into profiles/<tag>_bench_kernel_trace.md: calls, total and average duration per
kernel from the rocpd database's `kernels` view (durations in ns).

    python tools/trace_summary.py gpurun_out/prof_<tag>/trace <tag>
"""
import glob
import os
import sqlite3
import sys


def main():
    src, tag = sys.argv[1], sys.argv[2]
    db = sorted(glob.glob(os.path.join(src, "*.db")))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = [f"# {tag} kernel trace: bench --steps 5 --warmup 2 (timed legs only)", "",
             f"source: `{src}` (rocprofv3 --kernel-trace --stats; durations from the rocpd `kernels` view)", "",
             "| kernel | calls | total (ms) | average (ms) | % |", "|---|---|---|---|---|"]
    for n, k, s, a in rows:
        short = n.split("(")[0] if n.startswith("pf_") else n[:60]
        lines.append(f"| {short} | {k} | {s / 1e6:.3f} | {a / 1e6:.3f} | {100 * s / tot:.2f} |")
    out = os.path.join(root, "profiles", f"{tag}_bench_kernel_trace.md")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:12]))


if __name__ == "__main__":
    main()
