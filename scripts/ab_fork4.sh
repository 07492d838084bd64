#!/bin/bash
# Fork cadence 2 vs 4 at the 2- and 4-GPU per-rank shares (bs64, bs32).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_fork4.txt; : > $out
for b in 64 32; do
  for f in 2 4 2 4; do
    r=$(DTR_FORK_EVERY=$f timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b fork_every=$f $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
  done
done
