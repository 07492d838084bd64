#!/usr/bin/env python3
"""Which hardware queue every stream's kernels ran on (rocprofv3 rocpd database).

usage: queue_table.py RESULTS_DB TITLE OUT_MD"""
import collections
import re
import sqlite3
import sys


def fam(name: str) -> str:
    n = re.sub(r"\(.*$", "", name).replace("void ", "").replace("dtr::", "")
    m = re.match(r"_ZN3dtr\d+(\w+?)E", n)
    n = m.group(1) if m else n
    return n.split("<")[0][:48]


def main():
    db, title, out = sys.argv[1:4]
    c = sqlite3.connect(db)
    rows = c.execute("select stream_id, stream, queue_id, queue, name from kernels").fetchall()
    per = collections.defaultdict(collections.Counter)
    names = {}
    for sid, sname, qid, qname, kname in rows:
        per[(sid, qid)][fam(kname)] += 1
        names[(sid, qid)] = (sname, qname)
    lines = [f"# {title}", "", "| stream id | stream | queue id | queue | kernels | families (count) |",
             "|---|---|---|---|---|---|"]
    for key in sorted(per):
        cnt = per[key]
        fams = ", ".join(f"`{k}` {v}" for k, v in cnt.most_common(6))
        lines.append(f"| {key[0]} | {names[key][0]} | {key[1]} | {names[key][1]} | "
                     f"{sum(cnt.values())} | {fams} |")
    try:
        sa = c.execute("select * from stream_args limit 1").fetchall()
        if sa:
            lines += ["", f"(stream_args view present: {len(c.execute('select * from stream_args').fetchall())} rows)"]
    except sqlite3.Error:
        pass
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
