#!/usr/bin/env python3
"""Critical-path tail of one profiled training step from a rocprofv3 (rocpd) DB:
lists the kernels of the second-to-last step from the first kernel at or after
`--from` (regex) up to the optimizer, with their queue, start offset and duration,
and the main queue's idle time in that window.
usage: step_tail.py RUN_RESULTS_DB [--from REGEX] [--last K]"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"^void ", "", n.split("(")[0]).replace("dtr::", "")
    return n[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--from", dest="frm", default="maxpool_bwd")
    ap.add_argument("--opt", default="sgd_pack")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    ev = sorted(db.execute("select start, end, queue_id, name from kernels"))
    opt = [i for i, e in enumerate(ev) if re.search(a.opt, e[3])]
    end_i = opt[-2]
    beg_i = opt[-3] + 1
    step = ev[beg_i:end_i + 1]
    t0 = step[0][0]
    print(f"step span {(step[-1][1] - t0) / 1e3:.1f} us, {len(step)} kernels")
    start = next((i for i, e in enumerate(step) if re.search(a.frm, e[3])), len(step) - a.last)
    tail = step[start:]
    qmain = step[0][2]
    busy, last_end = 0, tail[0][0]
    for s, e, q, n in tail:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{q % 100:02d} {short(n)}")
        if q == qmain:
            busy += e - max(s, last_end) if e > last_end else 0
            last_end = max(last_end, e)
    span = tail[-1][1] - tail[0][0]
    print(f"tail span {span / 1e3:.1f} us, main-queue busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
