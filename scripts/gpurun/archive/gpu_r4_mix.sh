#!/bin/bash
# Forward/backward slice split + stage-3 split-K across idle waves: persistent tests and
# ring8 tests, bs16-128 bench; then the ring8 probe and the RN50 kernel-trace A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python3 -u -m pytest tests/test_persist_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "persist or ring8" > gpurun_out/prnq_tests.log 2>&1
rc=$?
tail -2 gpurun_out/prnq_tests.log
[ $rc -eq 0 ] || exit $rc
for b in 16 32 64 96 128; do
  timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
bash scripts/gpurun/gpu_r4_ring8probe.sh
