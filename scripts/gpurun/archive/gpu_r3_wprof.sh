#!/bin/bash
# Round 3: engine kernel totals with the ring weight gradient on / off (ImageNet RN50 bs128).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for t in "ring_wgrad=1" "ring_wgrad=0"; do
  DTR_TUNE="$t" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_w -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 5 > gpurun_out/prof_w.log 2>&1 || { tail -20 gpurun_out/prof_w.log; exit 1; }
  db=$(find gpurun_out/prof_w -name '*.db' | head -1)
  python3 scripts/rocpd_summary.py "$db" 10 "RN50 $t" gpurun_out/w_$t.md > /dev/null && sed -n '3,3p;/By kernel family/,/^$/p' gpurun_out/w_$t.md | head -12; grep "wgrad" gpurun_out/w_$t.md | head -12
  rm -rf gpurun_out/prof_w
done
