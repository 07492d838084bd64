#!/usr/bin/env python3
"""Summarize a rocprofv3 (ROCm 7, rocpd SQLite output) kernel trace into markdown.

usage: rocpd_summary.py RUN_RESULTS_DB STEPS TITLE OUT_MD [--last N]

Per-step numbers are taken over the LAST `STEPS` steps' worth of dispatches
(the profiled run's timed steps; warmup and setup launches are excluded by
keeping the last N dispatches, N = total dispatches of the timed window, found
as the dispatches after the last synchronising fill/copy marker when `--last`
is not given: we simply take the final STEPS/(STEPS+WARMUP) fraction of
per-step kernels via the optimizer kernel, which runs exactly once per step).
Also reports the wall span of the timed window (first start to last end), so
kernel-sum vs wall shows the cross-stream overlap.
"""
import collections
import re
import sqlite3
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "dtr::"):
        n = n.replace(p, "")
    if n.startswith("_ZN3dtr"):
        m = re.match(r"_ZN3dtr\d+(\w+?)E", n)
        n = m.group(1) if m else n
    return n[:90]


def main():
    db, steps, title, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, duration, grid_x, grid_y, grid_z, lds_size, "
                     "vgpr_count, accum_vgpr_count, stream_id from kernels order by start").fetchall()
    # one optimizer launch per step: the window starts after the (K+1)-th-from-last one
    opt = [i for i, r in enumerate(rows) if "sgd_pack_kernel" in r[0] or "sgd_tiles_kernel" in r[0]]
    if len(opt) < steps + 1:
        raise SystemExit(f"found {len(opt)} optimizer launches, need > {steps}")
    lo, hi = opt[-steps - 1] + 1, opt[-1] + 1
    win = rows[lo:hi]
    wall = (max(r[2] for r in win) - min(r[1] for r in win)) / 1e6 / steps
    tot = sum(r[3] for r in win) / 1e6 / steps
    fam = collections.defaultdict(float)
    inst = collections.defaultdict(lambda: [0, 0.0, set(), 0, 0])
    for r in win:
        n = short(r[0])
        fam[n.split("<")[0]] += r[3] / 1e6 / steps
        e = inst[n]
        e[0] += 1
        e[1] += r[3] / 1e3
        e[2].add(r[4] * r[5] * r[6])
        e[3] = r[8]
        e[4] = r[7]
    lines = [f"# {title}", "",
             f"Per step (last {steps} timed steps): kernel time **{tot:.3f} ms**, wall span "
             f"**{wall:.3f} ms** (kernel sum > wall = cross-stream overlap); "
             f"{len(win) / steps:.0f} kernel launches per step.", "",
             "## By kernel family", "", "| family | ms/step | share |", "|---|---|---|"]
    for k, v in sorted(fam.items(), key=lambda x: -x[1]):
        lines.append(f"| `{k}` | {v:.3f} | {100 * v / tot:.1f}% |")
    lines += ["", "## Top kernels (instantiations)", "",
              "| kernel | calls/step | avg us | ms/step | share | VGPR | LDS B |",
              "|---|---|---|---|---|---|---|"]
    for k, (n, us, grids, vg, lds) in sorted(inst.items(), key=lambda x: -x[1][1])[:30]:
        lines.append(f"| `{k}` | {n / steps:.1f} | {us / n:.1f} | {us / 1e3 / steps:.3f} | "
                     f"{100 * us / 1e3 / steps / tot:.1f}% | {vg} | {lds} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
