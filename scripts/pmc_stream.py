#!/usr/bin/env python3
"""Measured HBM bytes per kernel dispatch group from rocprofv3 --pmc CSVs (pass A with
FETCH_SIZE, pass B with WRITE_SIZE) of a probe script: rows grouped by (kernel, grid size),
medians over the group's dispatches.  FETCH_SIZE / WRITE_SIZE are in KB (L2 <-> fabric).

usage: pmc_stream.py OUT_MD FILTER_REGEX PASS_A.csv PASS_B.csv
"""
import collections
import csv
import re
import statistics
import sys


def load(path, counter):
    vals = collections.defaultdict(dict)
    meta = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            d = int(row["Dispatch_Id"])
            if row["Counter_Name"] == counter:
                vals[d][counter] = vals[d].get(counter, 0.0) + float(row["Counter_Value"])
            grid = row.get("Grid_Size") or row.get("Grid_Size_X") or ""
            meta[d] = (row["Kernel_Name"], grid,
                       int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals, meta


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("dtr::", "")
    return n[:70]


def main():
    out, flt, pa, pb = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3], sys.argv[4]
    va, ma = load(pa, "FETCH_SIZE")
    vb, mb = load(pb, "WRITE_SIZE")
    ga, gb = collections.defaultdict(list), collections.defaultdict(list)
    for d, (k, g, _) in ma.items():
        if flt.search(k) and "FETCH_SIZE" in va[d]:
            ga[(short(k), g)].append(va[d]["FETCH_SIZE"])
    for d, (k, g, _) in mb.items():
        if flt.search(k) and "WRITE_SIZE" in vb[d]:
            gb[(short(k), g)].append(vb[d]["WRITE_SIZE"])
    lines = ["| kernel | grid | dispatches | HBM read MB | HBM write MB |", "|---|---|---|---|---|"]
    for key in sorted(set(ga) | set(gb)):
        r = statistics.median(ga[key]) / 1024 if ga.get(key) else float("nan")
        w = statistics.median(gb[key]) / 1024 if gb.get(key) else float("nan")
        n = max(len(ga.get(key, [])), len(gb.get(key, [])))
        lines.append(f"| `{key[0]}` | {key[1]} | {n} | {r:.1f} | {w:.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
