#!/usr/bin/env python3
"""Merge several rocprofv3 `--pmc ... --output-format csv` passes of the SAME command into
one markdown table per kernel (rocprofv3 collects one counter block set per pass).

Per pass, every dispatch's counters are averaged per (kernel, grid); passes are joined on
(kernel, grid).  Derived columns:
  dur us        mean dispatch duration (first pass that has the kernel)
  MFMA TF/s     512 * SQ_INSTS_VALU_MFMA_MOPS_BF16 / duration
  VALU/MFMA     SQ_INSTS_VALU / SQ_INSTS_MFMA (vector instructions per matrix instruction)
  wait% issue%  SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  LDS conf/inst SQ_LDS_BANK_CONFLICT cycles per SQ_INSTS_LDS
  HBM GB/s      (FETCH_SIZE + WRITE_SIZE) [KB] / duration
usage: pmc_merge.py TITLE OUT_MD PASS_CSV [PASS_CSV ...] [--only SUBSTR]"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name).replace("void ", "").replace("dtr::", "")
    m = re.match(r"_ZN3dtr\d+(\w+?)E", n)
    return m.group(1) if m else n[:90]


def load(path, only):
    disp = collections.defaultdict(dict)
    meta = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Kernel_Name"])
            if only and only not in k:
                continue
            d = int(r["Dispatch_Id"])
            disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = (k, int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = collections.defaultdict(lambda: [0, 0.0, collections.defaultdict(float)])
    for d, (k, grid, dur) in meta.items():
        e = out[(k, grid)]
        e[0] += 1
        e[1] += dur
        for c, v in disp[d].items():
            e[2][c] += v
    return {key: (n, dur / n / 1e3, {c: v / n for c, v in cs.items()}) for key, (n, dur, cs) in out.items()}


def main():
    args = sys.argv[1:]
    only = None
    if "--only" in args:
        i = args.index("--only")
        only = args[i + 1]
        del args[i:i + 2]
    title, out_md, paths = args[0], args[1], args[2:]
    merged = {}
    for p in paths:
        for key, (n, dur, cs) in load(p, only).items():
            if key not in merged:
                merged[key] = [n, dur, {}]
            merged[key][2].update(cs)
    rows = []
    for (k, grid), (n, dur, c) in merged.items():
        g = c.get
        wc = g("SQ_WAVE_CYCLES", 0) or 1
        tf = 512 * g("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) / (dur * 1e-6) / 1e12 if dur else 0.0
        vm = g("SQ_INSTS_VALU", 0) / g("SQ_INSTS_MFMA", 0) if g("SQ_INSTS_MFMA") else float("nan")
        lc = g("SQ_LDS_BANK_CONFLICT", 0) / g("SQ_INSTS_LDS", 0) if g("SQ_INSTS_LDS") else float("nan")
        kb = g("FETCH_SIZE", 0) + g("WRITE_SIZE", 0)
        bw = kb * 1e3 / (dur * 1e3) if dur and kb else float("nan")   # KB/us = GB/s
        rows.append((k, grid, n, dur, tf, vm, 100 * g("SQ_WAIT_ANY", 0) / wc,
                     100 * g("SQ_ACTIVE_INST_ANY", 0) / wc, lc, g("FETCH_SIZE", float("nan")) / 1e3,
                     g("WRITE_SIZE", float("nan")) / 1e3, bw))
    rows.sort(key=lambda r: -r[3] * r[2])
    with open(out_md, "w") as f:
        f.write(f"# {title}\n\n")
        f.write("| kernel | grid (threads) | n | dur us | MFMA TF/s | VALU/MFMA | wait% | issue% | "
                "LDS conf/inst | fetch MB | write MB | HBM GB/s |\n")
        f.write("|---|---|---|---|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r[0]}` | {r[1]} | {r[2]} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.1f} | {r[6]:.0f} | "
                    f"{r[7]:.0f} | {r[8]:.2f} | {r[9]:.2f} | {r[10]:.2f} | {r[11]:.0f} |\n")
    print(open(out_md).read())


if __name__ == "__main__":
    main()
