#!/bin/bash
# Round 6 final build: kernel tables of the CIFAR persistent step (bs16, bs128) and the
# RN50 bs128 step (rocprofv3 --kernel-trace, summarized by scripts/rocpd_summary.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/tab6_*
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tab6_c16 -o run -- python3 bench.py --batch 16 --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/tab6_c16.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tab6_c128 -o run -- python3 bench.py --batch 128 --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/tab6_c128.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tab6_in -o run -- python3 bench.py --model imagenet_resnet50 --steps 12 --warmup 5 --phase-steps 0 > gpurun_out/tab6_in.log 2>&1
