#!/bin/bash
# Soak, part A: the persistent CIFAR RN50 step on one GPU for 10 min at the headline
# batch 128 and 4 min at the 8-GPU per-rank share 16 (scripts/soak.py)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 660 python -u scripts/soak.py --seconds 600 --batch 128 --out gpurun_out/soak_cifar_bs128.jsonl &&
timeout -k 10 300 python -u scripts/soak.py --seconds 240 --batch 16 --out gpurun_out/soak_cifar_bs16.jsonl
