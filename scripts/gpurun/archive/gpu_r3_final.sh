#!/bin/bash
# Round 3 end: full GPU suite + smoke, CIFAR benches, ImageNet RN50 tail_main A/B
# (after the streaming kernels), RN101, and the default bench.py line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -2 gpurun_out/full_gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/default.json 2> gpurun_out/default.err || { tail -20 gpurun_out/default.err; exit 1; }
cat gpurun_out/default.json
for cfg in tail_main=1.0 tail_main=0.5 tail_main=0.25 tail_main=1.0 tail_main=0.5 tail_main=0.25; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 > gpurun_out/f.json 2> gpurun_out/f.err || { tail -20 gpurun_out/f.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/f.json')); print('rn50', sys.argv[1], j['ms_per_step'], j['phase_ms']['backward'])" $cfg
done
for cfg in tail_main=1.0 tail_main=0.5; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet101 --steps 20 --warmup 5 > gpurun_out/f.json 2> gpurun_out/f.err || { tail -20 gpurun_out/f.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/f.json')); print('rn101', sys.argv[1], j['ms_per_step'], j['config']['peak_mem_gb'])" $cfg
done
for b in 128 32 16; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'])" $b
done
