#!/bin/bash
# Kernel trace of the ImageNet RN50 bs128 step with and without the 8-wave ring.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for t in 1 0; do
  DTR_TUNE=ring8=$t timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r8_$t -o run -- python3 bench.py --model imagenet_resnet50 --steps 6 --warmup 3 --phase-steps 0 > gpurun_out/prof_r8_$t.log 2>&1 || { tail -20 gpurun_out/prof_r8_$t.log; exit 1; }
done
