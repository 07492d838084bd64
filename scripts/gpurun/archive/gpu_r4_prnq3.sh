#!/bin/bash
# Persistent step: deferred forward publishes at one slice + shared weight-gradient queue.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python3 -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prnq_tests.log 2>&1
rc=$?
tail -2 gpurun_out/prnq_tests.log
[ $rc -eq 0 ] || exit $rc
for b in 16 32 64 128; do
  timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
