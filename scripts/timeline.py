#!/usr/bin/env python3
"""Per-step stream timeline from a rocprofv3 kernel_trace.csv: busy time per
queue, idle gaps on the main queue, and the critical-path split of one step.
A step is delimited by the `cifar_augment_kernel`/`synth_kernel` (first kernel
of every training step) -- pass another marker with --marker.
usage: timeline.py TRACE_CSV [--marker NAME] [--step K]"""
import argparse
import csv
import re


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("dtr::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="cifar_augment_kernel|synth_kernel|sgd_pack_kernel")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                  short(r["Kernel_Name"])) for r in rows), key=lambda e: e[0])
    pat = re.compile(a.marker.split("|")[-1])  # step ends at the optimizer kernel
    ends = [i for i, e in enumerate(ev) if pat.search(e[3])]
    if len(ends) < 3:
        print("not enough steps")
        return
    k = a.step
    lo, hi = ends[k - 1] + 1, ends[k] + 1
    step = ev[lo:hi]
    t0, t1 = step[0][0], step[-1][1]
    print(f"step wall (first start -> optimizer end): {(t1 - t0) / 1e3:.1f} us, kernels {len(step)}")
    queues = sorted({e[2] for e in step})
    for q in queues:
        ks = [e for e in step if e[2] == q]
        busy = sum(e[1] - e[0] for e in ks)
        gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
        gsum = sum(g for g in gaps if g > 0)
        print(f"queue {q}: {len(ks)} kernels, busy {busy / 1e3:.1f} us, gaps {gsum / 1e3:.1f} us "
              f"(median gap {sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.2f} us)")
    # union busy
    cur_s, cur_e, union = None, None, 0
    for s, e, _, _ in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    print(f"GPU busy (union of queues): {union / 1e3:.1f} us -> idle {(t1 - t0 - union) / 1e3:.1f} us")
    if a.list:
        for s, e, q, n in step:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {n}")


if __name__ == "__main__":
    main()
