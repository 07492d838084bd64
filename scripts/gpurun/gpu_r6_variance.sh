#!/bin/bash
# Round 6: box-to-box spread of the bench numbers -- run on several fresh boxes: CIFAR
# RN50 global 128 (x3), the per-rank shares 64 / 32 / 16, ImageNet RN50 bs128.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && tag=${1:-x} &&
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py > gpurun_out/var.json 2>/dev/null || exit 1
  echo "$tag cifar128 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var.json)"
done
for b in 64 32 16; do
  timeout -k 10 120 python -u bench.py --batch $b --steps 400 --warmup 40 --phase-steps 0 > gpurun_out/var.json 2>/dev/null || exit 1
  echo "$tag cifar$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var.json)"
done
timeout -k 10 240 python -u bench.py --model imagenet_resnet50 > gpurun_out/var.json 2>/dev/null || exit 1
echo "$tag imagenet $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var.json)"
