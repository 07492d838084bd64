#!/bin/bash
# Persistent step quick check: gradient tests, then bs16/32/64/96/128 bench (auto slices).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread -k "autograd or deterministic or forward or auto" > gpurun_out/prnq_tests.log 2>&1
rc=$?
tail -3 gpurun_out/prnq_tests.log
[ $rc -eq 0 ] || exit $rc
for b in ${BATCHES:-16 32 64 96 128}; do
  timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
