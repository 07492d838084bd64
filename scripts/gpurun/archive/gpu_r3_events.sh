#!/bin/bash
# Round 3: release scope of the plan's fork/join events (CIFAR bs128 / bs16, ImageNet bs128).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rnd in 1 2; do
for t in "plan_event_scope=0" "plan_event_scope=1" "plan_event_scope=2"; do
  for b in 128 16; do
    DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/ev.json 2> gpurun_out/ev.err || { tail -20 gpurun_out/ev.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/ev.json')); print(sys.argv[1], 'bs', sys.argv[2], j['ms_per_step'])" "$t" $b
  done
done
done
for t in "plan_event_scope=0" "plan_event_scope=1"; do
  DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/ev.json 2> gpurun_out/ev.err || { tail -20 gpurun_out/ev.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/ev.json')); print(sys.argv[1], 'imagenet', j['ms_per_step'])" "$t"
done
