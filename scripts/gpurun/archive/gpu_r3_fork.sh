#!/bin/bash
# Round 3 late: ImageNet fork cadence / tail re-check after the streaming kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in tail_main=1.0 tail_main=0.5 tail_main=0.25 tail_main=0.75 tail_main=0.0 tail_main=1.0 tail_main=0.5 tail_main=0.25; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 > gpurun_out/f.json 2> gpurun_out/f.err || { tail -20 gpurun_out/f.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/f.json')); print('rn50', sys.argv[1], j['ms_per_step'], j['phase_ms']['backward'])" $cfg
done
