#!/bin/bash
# Round 3: BN-backward apply in a recomputed dgrad epilogue (tune bap_maxc): numerics, then
# ImageNet RN50 bs128 A/B back to back (bap_maxc=0 = dgrad + separate apply).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/bap_tests.log 2>&1 \
  || { tail -40 gpurun_out/bap_tests.log; exit 1; }
tail -2 gpurun_out/bap_tests.log
for t in 0 2048 0 2048; do
  DTR_TUNE=bap_maxc=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/bap.json 2> gpurun_out/bap.err || { tail -20 gpurun_out/bap.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bap.json')); print('bap_maxc', sys.argv[1], j['value'], j['ms_per_step'])" $t
done
