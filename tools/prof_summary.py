#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats database (or CSV dir) into profiles/<name>.md."""

import glob
import os
import sqlite3
import sys


def summarize(src, out, title):
    dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    lines = [f"# {title}", "", f"source: `{src}` (rocprofv3 --kernel-trace --stats; top_kernels is in us, kernels.duration in ns in the rocpd schema)", ""]
    for db in dbs:
        c = sqlite3.connect(db)
        lines.append("| kernel | calls | total (ms) | average (ms) | % |")
        lines.append("|---|---|---|---|---|")
        for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"):
            lines.append(f"| {r[0][:60]} | {r[1]} | {r[2] / 1e3:.3f} | {r[3] / 1e3:.3f} | {r[4]:.2f} |")
        lines.append("")
        skip = int(os.environ.get("PROF_SKIP", "0"))
        if skip:
            lines.append(f"timed launches only (first {skip} launches of each kernel skipped: warm-up):")
            lines.append("")
            lines.append("| kernel | launches | average (ms) | min (ms) | max (ms) |")
            lines.append("|---|---|---|---|---|")
            per = {}
            for r in c.execute("select name, duration from kernels order by start"):
                per.setdefault(r[0], []).append(r[1] / 1e6)
            for name, ds in per.items():
                ds = ds[skip:] if len(ds) > skip else ds
                lines.append(f"| {name[:60]} | {len(ds)} | {sum(ds) / len(ds):.3f} | {min(ds):.3f} | {max(ds):.3f} |")
            lines.append("")
        lines.append("per-dispatch resources (first dispatch of each kernel):")
        lines.append("")
        lines.append("| kernel | grid_x | wg_x | vgpr | agpr | sgpr | lds | scratch | duration (ms) |")
        lines.append("|---|---|---|---|---|---|---|---|---|")
        seen = set()
        for r in c.execute("select name, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, sgpr_count, "
                           "lds_size, scratch_size, duration from kernels order by start"):
            if r[0] in seen:
                continue
            seen.add(r[0])
            lines.append("| " + " | ".join(str(x)[:60] for x in r[:8]) + f" | {r[8] / 1e6:.3f} |")
        lines.append("")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    summarize(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 summary")
