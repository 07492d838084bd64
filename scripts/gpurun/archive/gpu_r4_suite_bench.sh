#!/bin/bash
# Full GPU test suite, then the per-layer CIFAR selection A/B (persist=0) at bs16/32/64/128
# and the default bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_full.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/gpu_full.log | head -20
tail -1 gpurun_out/gpu_full.log
[ $rc -eq 0 ] || exit $rc
for b in 16 32 64 128; do
  for t in persist=0 persist=-1; do
    DTR_TUNE=$t timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'])" $b $t
  done
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cat gpurun_out/bench_default.json
