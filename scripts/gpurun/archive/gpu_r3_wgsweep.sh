#!/bin/bash
# Round 3: split-K wgrad sizing re-tuned after the ring wgrad + streaming kernels (RN50 bs128).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in wgrad_slab_mb=32 wgrad_slab_mb=16 wgrad_slab_mb=12 wgrad_slab_mb=8 wgrad_slab_mb=16,wgrad_target_wg=1024 wgrad_slab_mb=16,wgrad_target_wg=384 wgrad_slab_mb=32 wgrad_slab_mb=16; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/wg.json 2> gpurun_out/wg.err || { tail -20 gpurun_out/wg.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/wg.json')); print(sys.argv[1], j['ms_per_step'], j['phase_ms']['backward'])" $cfg
done
