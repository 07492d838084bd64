#!/bin/bash
# Round 3: CIFAR per-rank shares under wgrad_slab_mb 32 / 16, back to back.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for b in 128 32; do
  for cfg in wgrad_slab_mb=32 wgrad_slab_mb=16 wgrad_slab_mb=32 wgrad_slab_mb=16; do
    DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/c.json 2> gpurun_out/c.err || { tail -20 gpurun_out/c.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/c.json')); print('bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'])" $b $cfg
  done
done
