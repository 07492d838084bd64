#!/bin/bash
# Soak, part C: the world > 1 paths the scaling run takes, two ranks on CU halves of one
# GPU (shm transport): CIFAR persistent + overlap plan at 32 images per rank (the 4-GPU
# share) for 8 min, and the ImageNet RN50 per-layer plan (side stream + comm-stream
# buckets) at 32 images per rank for 5 min; replicas compared bit for bit at the end.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
export DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm DTR_CU_PARTITION=2 HSA_ENABLE_IPC_MODE_LEGACY=0 &&
timeout -k 10 560 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29841 scripts/soak.py --seconds 480 --batch 32 --out gpurun_out/soak_w2_bs32.jsonl &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29842 scripts/soak.py --model imagenet_resnet50 --seconds 300 --batch 32 --chunk 100 --out gpurun_out/soak_w2_in_bs32.jsonl
