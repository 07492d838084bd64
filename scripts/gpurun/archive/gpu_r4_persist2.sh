#!/bin/bash
# Persistent CIFAR step v2 (row slices): numerics tests, then bs16/32 A/B (P = 4, 2, per-layer).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python3 -u -m pytest tests/test_persist_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/persist_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|worst|persistent|rel" gpurun_out/persist_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
for b in 16 32; do
  for t in "persist=1,persist_slices=4" "persist=1,persist_slices=2" "persist=0"; do
    DTR_TUNE=$t timeout -k 10 200 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $b $t
  done
done
timeout -k 10 120 python3 scripts/prn_probe.py 16 50 > gpurun_out/prn_probe16.log 2>&1 && cat gpurun_out/prn_probe16.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prn16 -o prn16 -- python3 bench.py --batch 16 --steps 50 --warmup 10 > gpurun_out/prof_prn16.log 2>&1 && find gpurun_out/prof_prn16 -name "*kernel_stats.csv" | head -3
