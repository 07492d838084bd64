#!/usr/bin/env python3
"""Summarize a rocprofv3 kernel_stats.csv into markdown (for profiles/).

usage: summarize_profile.py STATS_CSV STEPS TITLE OUT_MD [TRACE_CSV]
Per-step time = total kernel time / STEPS (the profiled run's step count incl. warmup)."""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "dtr::"):
        n = n.replace(p, "")
    if n.startswith("_ZN3dtr"):
        import re
        m = re.match(r"_ZN3dtr\d+(\w+?)E", n)
        n = m.group(1) if m else n
    return n[:90]


def main():
    path, steps, title, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    fam = defaultdict(float)
    for r in rows:
        n = short(r["Name"])
        key = n.split("<")[0]
        fam[key] += float(r["TotalDurationNs"])
    lines = [f"# {title}", "",
             f"Kernel time per step: **{tot / steps / 1e6:.3f} ms** over {steps} steps; "
             f"{calls / steps:.0f} kernel launches per step.", "",
             "## By kernel family", "", "| family | ms/step | share |", "|---|---|---|"]
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        lines.append(f"| `{k}` | {v / steps / 1e6:.3f} | {100 * v / tot:.1f}% |")
    lines += ["", "## Top kernels (instantiations)", "",
              "| kernel | calls/step | avg us | ms/step | share |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        t = float(r["TotalDurationNs"])
        lines.append(f"| `{short(r['Name'])}` | {int(r['Calls']) / steps:.1f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {t / steps / 1e6:.3f} | {100 * t / tot:.1f}% |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:30]))


if __name__ == "__main__":
    main()
