#!/bin/bash
# ImageNet RN50 at the final defaults: fork cadence 2 / 3 and tail fraction 1 / 0.5.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_in_tail.txt; : > $out
for cfg in "2 1" "3 1" "2 0.5" "2 1" "3 1" "2 0.5"; do
  set -- $cfg
  r=$(DTR_FORK_EVERY=$1 DTR_TAIL_MAIN=$2 timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric) || exit 1
  echo "imagenet fork_every=$1 tail_main=$2 $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
done
