#!/bin/bash
# 8-wave ring conv: numerics vs the 4-wave ring and the reference, then ImageNet RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "ring" > gpurun_out/ring8_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/ring8_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for t in ring8=1 ring8=0; do
  DTR_TUNE=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 20 --warmup 5 > gpurun_out/bi.json 2> gpurun_out/bi.err || { tail -20 gpurun_out/bi.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bi.json')); print('RN50', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $t
done
