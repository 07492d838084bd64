#!/bin/bash
# PMC counters of the persistent CIFAR launches (bs16, 10 steps): one counter set per pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
mkdir -p gpurun_out/pmc
timeout -k 10 200 python3 -u scripts/prn_probe.py 16 50 > gpurun_out/prn_probe16.txt 2>&1 || { tail -5 gpurun_out/prn_probe16.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/prn_probe16.txt | tail -40
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  tag=$(echo $set | cut -c1-20 | tr ' ' '_')
  DTR_TUNE=persist=1 timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/$tag -- python3 bench.py --batch 16 --steps 10 --warmup 3 --phase-steps 0 > /dev/null 2> gpurun_out/pmc/$tag.err || { tail -5 gpurun_out/pmc/$tag.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob("gpurun_out/pmc/*/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "prn_" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        n = max(c for (kk, _), c in cnt.items() if kk == k)
        print(k[:40], {c: round(v / n) for c, v in sorted(d.items())})
PY
