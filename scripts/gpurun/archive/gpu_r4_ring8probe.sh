#!/bin/bash
# ring8 per-shape timing + workgroup-0 timeline, then the RN50 kernel trace A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 200 python3 scripts/ring8_probe.py > gpurun_out/ring8_probe.log 2>&1 || { tail -20 gpurun_out/ring8_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ring8_probe.log
for t in 1 0; do
  DTR_TUNE=ring8=$t timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r8_$t -o run -- python3 bench.py --model imagenet_resnet50 --steps 6 --warmup 3 --phase-steps 0 > gpurun_out/prof_r8_$t.log 2>&1 || { tail -20 gpurun_out/prof_r8_$t.log; exit 1; }
done
