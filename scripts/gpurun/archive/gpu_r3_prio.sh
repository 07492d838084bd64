#!/bin/bash
# Round 3: high-priority main stream (tune stream_prio) A/B: ImageNet RN50, CIFAR bs128 / bs16.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in stream_prio=0 stream_prio=1 stream_prio=2 stream_prio=0 stream_prio=1 stream_prio=2; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 > gpurun_out/p.json 2> gpurun_out/p.err || { tail -20 gpurun_out/p.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/p.json')); print('rn50', sys.argv[1], j['ms_per_step'], j['phase_ms']['backward'])" $cfg
done
for b in 128 16; do
  for cfg in stream_prio=0 stream_prio=1 stream_prio=0 stream_prio=1; do
    DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/p.json 2> gpurun_out/p.err || { tail -20 gpurun_out/p.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/p.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['ms_per_step'])" $b $cfg
  done
done
