#!/usr/bin/env python3
"""Per-stream kernel time of the last STEPS steps of a rocprofv3 (rocpd) trace: which
families sit on each hardware queue/stream -- the main stream's sum is the step's
critical-path floor when the side stream's work overlaps it.

usage: stream_breakdown.py RUN_RESULTS_DB STEPS [MARK_KERNEL]
MARK_KERNEL (default sgd_pack_kernel) runs once per step; the window starts after the
STEPS+1-th last occurrence."""
import collections
import re
import sqlite3
import sys


def fam(name):
    n = re.sub(r"^void ", "", name.split("(")[0])
    n = n.replace("dtr::", "")
    return n.split("<")[0]


def main():
    db, steps = sys.argv[1], int(sys.argv[2])
    mark = sys.argv[3] if len(sys.argv) > 3 else "sgd_pack_kernel"
    rows = sqlite3.connect(db).execute(
        "select name, queue_id, stream_id, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if mark in r[0]]
    lo = idx[-steps - 1] + 1 if len(idx) > steps else 0
    win = rows[lo:idx[-1] + 1]
    wall = (win[-1][4] - win[0][3]) / 1e3 / steps
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    tot = collections.defaultdict(float)
    for name, q, s, a, b in win:
        per[(q, s)][fam(name)] += (b - a) / 1e3 / steps
        tot[(q, s)] += (b - a) / 1e3 / steps
    print(f"wall per step {wall:.1f} us over {steps} steps")
    for key in sorted(tot, key=lambda k: -tot[k]):
        print(f"\n## queue {key[0]} stream {key[1]}: {tot[key]:.1f} us/step")
        for f, t in sorted(per[key].items(), key=lambda kv: -kv[1])[:14]:
            print(f"  {t:8.1f}  {f}")


if __name__ == "__main__":
    main()
