#!/bin/bash
# Round 3: one-launch optimizer (tune fused_opt): tests, then CIFAR / RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_engine_gpu.py -k "optimizer" > gpurun_out/opt_tests.log 2>&1 || { tail -40 gpurun_out/opt_tests.log; exit 1; }
tail -1 gpurun_out/opt_tests.log
for b in 128 16; do
  for cfg in fused_opt=0 fused_opt=1 fused_opt=0 fused_opt=1; do
    DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/o.json 2> gpurun_out/o.err || { tail -20 gpurun_out/o.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/o.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['ms_per_step'], j['phase_ms']['optimizer'])" $b $cfg
  done
done
for cfg in fused_opt=0 fused_opt=1 fused_opt=0 fused_opt=1; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 > gpurun_out/o.json 2> gpurun_out/o.err || { tail -20 gpurun_out/o.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/o.json')); print('rn50', sys.argv[1], j['ms_per_step'], j['phase_ms']['optimizer'])" $cfg
done
