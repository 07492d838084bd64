#!/bin/bash
# Fork cadence re-check with the backward-tail split (DTR_FORK_EVERY 1/2/3/4), CIFAR bs16/bs128.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_fork2.txt; : > $out
for b in 16 128; do
  for f in 2 1 3 4 2; do
    r=$(DTR_FORK_EVERY=$f timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b fork_every=$f $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
  done
done
