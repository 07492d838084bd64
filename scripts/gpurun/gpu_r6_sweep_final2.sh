#!/bin/bash
# Round 6: second knob re-sweep on the RN50 bs128 step after the write-through default.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
CFGS="base plan_event_scope=1 wgrad_xcd=0 nbuf1_kt=0 nbuf1_kt=2 base dgrad_splitk=0 parity_dgrad=0 bwd_apply_fin=0 fin_v=0 base reduce_main_tail=0 fork_every=1 fork_every=3 tail_main=0.25 tail_main=0.75 base wgrad_target_wg=512 wgrad_target_wg=1024 wgrad_slab_mb=8 wgrad_slab_mb=24 base"
for r in 1 2; do for c in $CFGS; do
  if [ $c = base ]; then unset DTR_TUNE; else export DTR_TUNE=$c; fi
  timeout -k 10 200 python -u bench.py --model imagenet_resnet50 --steps 150 --warmup 10 --phase-steps 0 > gpurun_out/sw.json 2>/dev/null || { echo "r$r $c failed"; continue; }
  echo "r$r $c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done; done
