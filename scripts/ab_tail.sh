#!/bin/bash
# A/B of DTR_TAIL_MAIN (share of the backward tail's weight gradients run on the main
# stream) at the CIFAR per-rank batches of the 1/2/4/8-GPU strong-scaling run.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_tail.txt; : > $out
for b in 16 32 64 128; do
  for f in 0 0.5 0.75 1; do
    r=$(DTR_TAIL_MAIN=$f timeout -k 10 120 python bench.py --batch $b --steps 300 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b tail_main=$f $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out
  done
done
