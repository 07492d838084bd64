#!/bin/bash
# Round 5: conv_wide (256x128 tile, 128x64 per wave) -- numerics, per-shape timing, RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "wide" > gpurun_out/r5w_tests.log 2>&1 || { tail -40 gpurun_out/r5w_tests.log; exit 1; }
tail -1 gpurun_out/r5w_tests.log
timeout -k 10 300 python -u scripts/wide_probe.py 3 > gpurun_out/r5w_probe.txt 2>&1 || { tail -20 gpurun_out/r5w_probe.txt; exit 1; }
cat gpurun_out/r5w_probe.txt
for t in "wide=1" "wide=0" "wide=1" "wide=0"; do
  DTR_TUNE=$t timeout -k 10 300 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 > gpurun_out/r5w_in.json 2> gpurun_out/r5w_err.log || { tail -20 gpurun_out/r5w_err.log; exit 1; }
  echo "RN50 [$t] $(python -c "import json;d=json.load(open('gpurun_out/r5w_in.json'));print(d['ms_per_step'], d['value'])")"
done
