#!/bin/bash
# Round 3 (diagnostic, wrong math): ImageNet RN50 bs128 step phases with the weight gradients
# skipped (the main stream without side-stream contention) vs the full step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for s in "" "wgrad"; do
  DTR_DIAG_SKIP="$s" timeout -k 10 300 python3 scripts/comm_overlap.py --model imagenet_resnet50 --batch 128 > gpurun_out/ct.json 2> gpurun_out/ct.err || { tail -20 gpurun_out/ct.err; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/ct.json').read().strip().splitlines()[-1]); print('skip=', sys.argv[1], j['phase_ms'])" "$s"
done
