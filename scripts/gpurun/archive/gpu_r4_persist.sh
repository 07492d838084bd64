#!/bin/bash
# Persistent CIFAR step: numerics tests, then bs16/32 A/B against the per-layer engine.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python3 -u -m pytest tests/test_persist_gpu.py tests/test_plan_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/persist_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|worst|persistent|rel" gpurun_out/persist_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
for b in 16 32; do
  for p in 1 0; do
    DTR_TUNE=persist=$p timeout -k 10 200 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], 'persist', sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $b $p
  done
done
