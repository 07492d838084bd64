#!/bin/bash
# Round 3: kernel trace of the ImageNet RN50 bs128 step (after the ring) + CIFAR bs128.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_in50 -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 5 > gpurun_out/prof_in50.log 2>&1 || { tail -20 gpurun_out/prof_in50.log; exit 1; }
db=$(ls gpurun_out/prof_in50/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(find gpurun_out/prof_in50 -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" 10 "ImageNet ResNet-50 v2, bs128/GPU, 1x MI355X (round 3: LDS-DMA ring)" gpurun_out/in50_kernels.md > /dev/null && head -40 gpurun_out/in50_kernels.md
rm -rf gpurun_out/prof_in50
