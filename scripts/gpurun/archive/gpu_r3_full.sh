#!/bin/bash
# Round 3: full GPU test suite, then the 1-GPU benches (CIFAR headline, ImageNet RN50/RN101).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -3 gpurun_out/full_gpu_tests.log
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > gpurun_out/bench_cifar.json 2> gpurun_out/bench_cifar.err || { tail -20 gpurun_out/bench_cifar.err; exit 1; }
cat gpurun_out/bench_cifar.json
timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/bench_in50.json 2> gpurun_out/bench_in50.err || { tail -20 gpurun_out/bench_in50.err; exit 1; }
cat gpurun_out/bench_in50.json
timeout -k 10 300 python3 bench.py --model imagenet_resnet101 --steps 30 --warmup 10 > gpurun_out/bench_in101.json 2> gpurun_out/bench_in101.err || { tail -20 gpurun_out/bench_in101.err; exit 1; }
cat gpurun_out/bench_in101.json
