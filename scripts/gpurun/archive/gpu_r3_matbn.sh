#!/bin/bash
# Round 3: which inner bottleneck BN outputs to materialize now that non-PRE convs run on the ring.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for t in "" "mat_bn_minc=128,mat_bn_elems=13000000" "mat_bn_minc=64,mat_bn_elems=26000000" "mat_bn_minc=128,mat_bn_elems=13000000,ring=0"; do
  DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/mb.json 2> gpurun_out/mb.err || { tail -20 gpurun_out/mb.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/mb.json')); print(repr(sys.argv[1]), j['ms_per_step'], j['phase_ms'])" "$t"
done
