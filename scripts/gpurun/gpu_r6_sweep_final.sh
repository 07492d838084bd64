#!/bin/bash
# Round 6: re-sweep of native / engine knobs not re-measured since the weight-gradient
# ring fix, on the RN50 bs128 step (bench, 100 timed steps), two interleaved rounds with
# the default between every few configurations.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
CFGS="base splitk=1 splitk=4 splitk_tiles=128 splitk_tiles=512 base bm128_min=2048 bm128_min=8192 ring_kt=4 ring_kt=6 base ring_kt_dgrad=3 ring_kt_dgrad=5 reduce_mb=2 reduce_mb=8 base bap_maxc=256 bap_maxc=1024 wt_store=0 wt_store=1 base"
for r in 1 2; do for c in $CFGS; do
  if [ $c = base ]; then unset DTR_TUNE; else export DTR_TUNE=$c; fi
  timeout -k 10 200 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 10 --phase-steps 0 > gpurun_out/sw.json 2>/dev/null || { echo "$c failed"; continue; }
  echo "r$r $c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json)"
done; done
