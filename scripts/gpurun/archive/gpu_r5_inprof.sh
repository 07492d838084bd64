#!/bin/bash
# ImageNet RN50 bs128 kernel statistics (round 5).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_in5 -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/prof_in5.log 2>&1 || { tail -20 gpurun_out/prof_in5.log; exit 1; }
ls gpurun_out/prof_in5 | head
