#!/bin/bash
# Persistent step: all numerics tests (P = 4, 2, 1), then bs96/128 persistent vs per-layer.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python3 -u -m pytest tests/test_persist_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/persist_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/persist_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for b in 96 128; do
  for t in "persist=1" "persist=0"; do
    DTR_TUNE=$t timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $b $t
  done
done
