#!/bin/bash
# Soak, part B: ImageNet RN50 bs128 for 5 min, then two ranks on CU halves of one GPU
# (shm transport, persistent step + overlap plan) at 16 and 64 images per rank
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 380 python -u scripts/soak.py --model imagenet_resnet50 --seconds 300 --batch 128 --chunk 200 --out gpurun_out/soak_imagenet_bs128.jsonl &&
export DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm DTR_CU_PARTITION=2 HSA_ENABLE_IPC_MODE_LEGACY=0 &&
timeout -k 10 330 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29821 scripts/soak.py --seconds 270 --batch 16 --out gpurun_out/soak_w2_bs16.jsonl &&
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29822 scripts/soak.py --seconds 150 --batch 64 --out gpurun_out/soak_w2_bs64.jsonl
