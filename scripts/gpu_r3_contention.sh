#!/bin/bash
# Round 3 (diagnostic, wrong math): ImageNet RN50 bs128 step with the weight gradients skipped,
# i.e. the main stream without side-stream contention; and with the ring off for reference.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for s in "" "wgrad"; do
  DTR_DIAG_SKIP="$s" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/ct.json 2> gpurun_out/ct.err || { tail -20 gpurun_out/ct.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/ct.json')); print('skip=', sys.argv[1], j['ms_per_step'], j['phase_ms'])" "$s"
done
