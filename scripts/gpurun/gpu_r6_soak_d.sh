#!/bin/bash
# Soak, part D: two ranks on CU halves at the 8-GPU (16 images) and 2-GPU (64 images)
# per-rank shares, persistent step (overlap plan at 16, after-backward buckets at 64 per
# the reserve rule on 128 CUs), 9 + 7 minutes, replicas compared bit for bit at the end.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
export DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm DTR_CU_PARTITION=2 HSA_ENABLE_IPC_MODE_LEGACY=0 &&
timeout -k 10 620 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29851 scripts/soak.py --seconds 540 --batch 16 --out gpurun_out/soak_w2_bs16_long.jsonl &&
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29852 scripts/soak.py --seconds 420 --batch 64 --out gpurun_out/soak_w2_bs64_long.jsonl
