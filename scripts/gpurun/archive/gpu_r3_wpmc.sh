#!/bin/bash
# Round 3: counters of the 7x7 512->512 3x3 weight gradient (register loop vs ring).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/wpmc$r -o run -- python3 scripts/wgrad_probe.py 128 7 512 512 3 1 10 $r > gpurun_out/wpmc$r.log 2>&1 || { tail -5 gpurun_out/wpmc$r.log; exit 1; }
done
for r in 0 1; do
  f=$(find gpurun_out/wpmc$r -name '*counter_collection.csv' | head -1)
  python3 - "$f" $r <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r['Kernel_Name'].split('(')[0][-60:]
    if 'wgrad' not in k or 'reduce' in k: continue
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    cnt = max(v for (kk, c), v in n.items() if kk == k)
    print('ring', sys.argv[2], k, {c: round(v / cnt) for c, v in d.items()})
PY
done
