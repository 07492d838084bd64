#!/bin/bash
# Round 3 end: stage-3 BN-backward recompute (bap_maxc 1024) and wgrad slab re-check under tail_main auto.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in bap_maxc=512 bap_maxc=1024 wgrad_slab_mb=32 bap_maxc=512 bap_maxc=1024 wgrad_slab_mb=32; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 > gpurun_out/f.json 2> gpurun_out/f.err || { tail -20 gpurun_out/f.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/f.json')); print('rn50', sys.argv[1], j['ms_per_step'], j['phase_ms']['backward'])" $cfg
done
