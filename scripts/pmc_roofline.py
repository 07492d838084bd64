#!/usr/bin/env python3
"""Measured bytes and MFMA rate per conv layer: joins the rocprofv3 --pmc CSVs of
scripts/roofline.py (one run per counter pass) with its launch manifest.

usage: pmc_roofline.py MANIFEST OUT_MD PMC_CSV [PMC_CSV ...]

Pass A: FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
Pass B: WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT
Per (layer, pass): HBM bytes read (FETCH_SIZE) and written (WRITE_SIZE) against the
unique-byte floor of roofline.py, the L2 hit rate, MFMA TF/s from the MFMA op count,
and the share of wave cycles spent waiting (s_waitcnt / barrier)."""
import collections
import csv
import re
import sys

OURS = re.compile(r"conv_gemm_kernel|conv_ring_kernel|conv3x3_direct_kernel|conv_wgrad|wgrad_reduce")


def load(path):
    disp = collections.defaultdict(dict)
    meta = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            d = int(row["Dispatch_Id"])
            disp[d][row["Counter_Name"]] = float(row["Counter_Value"])
            meta[d] = (row["Kernel_Name"], int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    seq = [(meta[d][0], meta[d][1], disp[d]) for d in sorted(disp) if OURS.search(meta[d][0])]
    return seq


def main():
    man, out, csvs = sys.argv[1], sys.argv[2], sys.argv[3:]
    calls = []
    for line in open(man):
        name, p, n, byts, flop = line.rstrip("\n").split("|")
        calls.append((name, p, int(n), float(byts), float(flop)))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in csvs:
        seq = load(path)
        i = 0
        for name, p, n, byts, flop in calls:
            per = 2 if p == "wgrad" else 1
            for c in range(n):
                grp = seq[i:i + per]
                i += per
                if c == 0:
                    continue                       # warm-up call
                tot = collections.defaultdict(float)
                dur = 0
                for _, d, cnt in grp:
                    dur += d
                    for k, v in cnt.items():
                        tot[k] += v
                for k, v in tot.items():
                    acc[(name, p)][k].append(v)
                acc[(name, p)]["_dur"].append(dur)
        if i != len(seq):
            print(f"warning: {path}: {len(seq) - i} unattributed dispatches", file=sys.stderr)
    lines = ["| layer | pass | floor MB | HBM read MB | HBM write MB | read+write / floor | L2 hit % | "
             "MFMA TF/s | wait % |", "|---|---|---|---|---|---|---|---|---|"]
    tot_floor = tot_meas = 0.0
    for name, p, n, byts, flop in calls:
        a = acc[(name, p)]
        m = lambda k: sum(a[k]) / len(a[k]) if a.get(k) else float("nan")  # noqa: E731
        rd, wr = m("FETCH_SIZE") / 1e3, m("WRITE_SIZE") / 1e3     # KB -> MB
        hit = 100 * m("TCC_HIT_sum") / max(m("TCC_HIT_sum") + m("TCC_MISS_sum"), 1)
        dur = m("_dur") * 1e-9
        tf = 512 * m("SQ_INSTS_VALU_MFMA_MOPS_BF16") / dur / 1e12 if dur else 0
        wait = 100 * m("SQ_WAIT_ANY") / max(m("SQ_WAVE_CYCLES"), 1)
        lines.append(f"| {name} | {p} | {byts / 1e6:.0f} | {rd:.0f} | {wr:.0f} | "
                     f"{(rd + wr) / (byts / 1e6):.2f} | {hit:.0f} | {tf:.0f} | {wait:.0f} |")
        tot_floor += byts / 1e6
        tot_meas += rd + wr
    lines.append("")
    lines.append(f"All layers once: measured HBM traffic {tot_meas / 1e3:.2f} GB vs unique-byte "
                 f"floor {tot_floor / 1e3:.2f} GB ({tot_meas / tot_floor:.2f}x).")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
