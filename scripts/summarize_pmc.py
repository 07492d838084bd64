#!/usr/bin/env python3
"""Summarise a rocprofv3 `--pmc ... --output-format csv` run into markdown.

Groups dispatches by (kernel, grid size), pivots the counters per dispatch and
reports means plus derived ratios:
  busy%      = SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
  wait%      = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (waves parked on s_waitcnt / barrier)
  issue%     = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  mfma_tf    = 512 * SQ_INSTS_VALU_MFMA_MOPS_BF16 / duration  (MOPS counted per 512 flop)
Usage: summarize_pmc.py <counter_collection.csv> [title] > out.md"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name) if not name.startswith("void at::") else "torch:" + \
        name.split("<")[0].split("::")[-1]
    return name.replace("void ", "").replace("dtr::", "")


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    disp = collections.defaultdict(dict)
    meta = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            d = int(row["Dispatch_Id"])
            disp[d][row["Counter_Name"]] = float(row["Counter_Value"])
            meta[d] = (short(row["Kernel_Name"]), int(row["Grid_Size"]),
                       int(row["End_Timestamp"]) - int(row["Start_Timestamp"]),
                       int(row["LDS_Block_Size"]), int(row["VGPR_Count"]) + int(row["Accum_VGPR_Count"]))
    groups = collections.defaultdict(list)
    for d, (k, grid, dur, lds, vgpr) in meta.items():
        groups[(k, grid, lds, vgpr)].append((dur, disp[d]))
    print(f"# {title}\n")
    print("| kernel | grid (threads) | LDS B | VGPR | n | dur us | busy% | wait% | issue% | MFMA TF/s | LDS bank-conf/wave-cyc |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    rows = []
    for (k, grid, lds, vgpr), items in groups.items():
        if k.startswith("torch:"):
            continue
        n = len(items)
        dur = sum(i[0] for i in items) / n / 1e3
        avg = collections.defaultdict(float)
        for _, c in items:
            for kk, v in c.items():
                avg[kk] += v / n
        wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
        busy = 100 * avg.get("SQ_BUSY_CYCLES", 0) / (avg.get("GRBM_GUI_ACTIVE", 0) or 1)
        tf = 512 * avg.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) / (dur * 1e-6) / 1e12 if dur else 0
        rows.append((k, grid, lds, vgpr, n, dur, busy, 100 * avg.get("SQ_WAIT_ANY", 0) / wc,
                     100 * avg.get("SQ_ACTIVE_INST_ANY", 0) / wc, tf,
                     avg.get("SQ_LDS_BANK_CONFLICT", 0) / wc))
    rows.sort(key=lambda r: -r[5] * r[4])
    for r in rows:
        print(f"| `{r[0]}` | {r[1]} | {r[2]} | {r[3]} | {r[4]} | {r[5]:.1f} | {r[6]:.0f} | {r[7]:.0f} | "
              f"{r[8]:.0f} | {r[9]:.1f} | {r[10]:.3f} |")


if __name__ == "__main__":
    main()
