#!/bin/bash
# Tail fraction at the final defaults (fork every 4, reduces on main): DTR_TAIL_MAIN 1 / 0.75 / 0.5.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_tail3.txt; : > $out
for b in 16 128; do
  for f in 1 0.75 0.5 1 0.75 0.5; do
    r=$(DTR_TAIL_MAIN=$f timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b tail_main=$f $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
  done
done
