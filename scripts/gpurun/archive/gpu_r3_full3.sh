#!/bin/bash
# Round 3: full GPU suite + smoke after the BN-backward fusion, CIFAR shares, ImageNet RN50 /
# RN101 benches, and a kernel trace of the RN50 default step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -2 gpurun_out/full_gpu_tests.log
for b in 128 64 32 16; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('bs', sys.argv[1], j['value'], j['ms_per_step'])" $b
done
for m in imagenet_resnet50 imagenet_resnet50 imagenet_resnet101; do
  timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 > gpurun_out/bi.json 2> gpurun_out/bi.err || { tail -20 gpurun_out/bi.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bi.json')); print(sys.argv[1], j['value'], j['ms_per_step'], j['config']['per_gpu_batch'], j['config']['peak_mem_gb'])" $m
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_in50 -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 5 > gpurun_out/prof_in50.log 2>&1 || { tail -20 gpurun_out/prof_in50.log; exit 1; }
db=$(find gpurun_out/prof_in50 -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" 10 "ImageNet ResNet-50 v2, bs128/GPU, 1x MI355X (round 3 late: streaming narrow-K 1x1 forward and dgrad + BN backward)" gpurun_out/in50_kernels.md > /dev/null || exit 1
rm -rf gpurun_out/prof_in50
head -12 gpurun_out/in50_kernels.md
