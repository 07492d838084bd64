#!/usr/bin/env python3
"""Queue-level overlap of the comm stream with the compute streams, from a rocprofv3
(rocpd SQLite) kernel trace of scripts/comm_overlap.py.

usage: overlap_summary.py RUN_RESULTS_DB STEPS TITLE OUT_MD [JSON_LINE_FILE]

Window: the last STEPS steps (one sgd_pack_kernel per step).  Reports, per
(stream, hardware queue): kernels and kernel time per step and the main kernel
families; for the comm stream (the one carrying the loopback all-reduce kernel):
the fraction of its kernel time during which a kernel of another stream was
running, and the exposed tail (last comm kernel end - last compute kernel end
before the optimizer) per step.
"""
import collections
import json
import re
import sqlite3
import sys


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("dtr::", "")
    if n.startswith("_ZN3dtr"):
        m = re.match(r"_ZN3dtr\d+(\w+?)E", n)
        n = m.group(1) if m else n
    return n.split("<")[0][:60]


def overlap_len(iv, others):
    """Length of interval iv covered by the union of `others` (sorted, merged)."""
    s, e = iv
    tot = 0
    for a, b in others:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def merge(ivs):
    out = []
    for a, b in sorted(ivs):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main():
    db, steps, title, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    extra = open(sys.argv[5]).read().strip().splitlines()[-1] if len(sys.argv) > 5 else None
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, duration, stream_id, queue_id from kernels "
                     "order by start").fetchall()
    opt = [i for i, r in enumerate(rows) if "sgd_pack_kernel" in r[0]]
    if len(opt) < steps + 1:
        raise SystemExit(f"found {len(opt)} optimizer launches, need > {steps}")
    win = rows[opt[-steps - 1] + 1:opt[-1] + 1]
    by = collections.defaultdict(list)
    for r in win:
        by[(r[4], r[5])].append(r)
    comm_key = next((k for k, v in by.items() if any("scale_inplace" in r[0] for r in v)), None)
    lines = [f"# {title}", "",
             f"Window: the last {steps} steps of the trace (rocprofv3 --kernel-trace).", "",
             "| stream id | HW queue id | kernels / step | kernel ms / step | main kernels |",
             "|---|---|---|---|---|"]
    for k, v in sorted(by.items()):
        fam = collections.Counter(short(r[0]) for r in v)
        tag = " (comm)" if k == comm_key else ""
        lines.append(f"| {k[0]}{tag} | {k[1]} | {len(v) / steps:.1f} | "
                     f"{sum(r[3] for r in v) / 1e6 / steps:.3f} | "
                     + ", ".join(f"`{n}` x{cnt / steps:.0f}" for n, cnt in fam.most_common(4)) + " |")
    queues = collections.defaultdict(set)
    for s, q in by:
        queues[q].add(s)
    shared = {q: sorted(s) for q, s in queues.items() if len(s) > 1}
    lines += ["", f"Streams sharing a hardware queue: {shared or 'none'}."]
    if comm_key is not None:
        comm = by[comm_key]
        others = merge([(r[1], r[2]) for k, v in by.items() if k != comm_key for r in v])
        ctot = sum(r[2] - r[1] for r in comm)
        cov = sum(overlap_len((r[1], r[2]), others) for r in comm)
        # exposed tail per step: from the last compute kernel before the step's optimizer
        # to the end of that step's last comm kernel
        tails = []
        opts = [r for r in win if "sgd_pack_kernel" in r[0]]
        prev = win[0][1]
        for o in opts:
            comp = [r for k, v in by.items() if k != comm_key for r in v
                    if prev <= r[1] < o[1] and "sgd_pack" not in r[0]]
            cm = [r for r in comm if prev <= r[1] < o[1]]
            if comp and cm:
                tails.append(max(0, max(r[2] for r in cm) - max(r[2] for r in comp)) / 1e3)
            prev = o[2]
        lines += ["", f"Comm-stream kernels: {len(comm) / steps:.1f} per step, "
                      f"{ctot / 1e3 / steps:.1f} us per step, of which "
                      f"**{100 * cov / max(ctot, 1):.1f} %** ran while a compute-stream kernel "
                      "was running (the rest: alone on the GPU)."]
        if tails:
            lines.append(f"Comm tail after the last compute kernel of the step: "
                         f"median {sorted(tails)[len(tails) // 2]:.1f} us.")
    if extra:
        try:
            j = json.loads(extra)
            lines += ["", "Engine phase timing (HIP events, 5 steps after the trace window):", "",
                      "```", json.dumps(j.get("phase_ms")), json.dumps(j.get("comm")), "```"]
        except ValueError:
            pass
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
