#!/bin/bash
# World > 1 stream-set rehearsal on one GPU: c10d NCCL group (device_id) + forced native
# RCCL Comm + bf16 exchange; rocprofv3 kernel + HIP runtime trace; queue id of every
# stream.  "late": the engine streams created after the process group (the round-3 order).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for order in early late; do
  for cfg in "cifar_resnet50 32" "imagenet_resnet50 64"; do
    set -- $cfg
    timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/queues_${order}_$1 -o run -- python3 scripts/stream_rehearsal.py $1 $2 6 $order > gpurun_out/queues_${order}_$1.log 2>&1 || { tail -20 gpurun_out/queues_${order}_$1.log; exit 1; }
    echo "$order $1: $(grep -E 'STREAMS' gpurun_out/queues_${order}_$1.log)"
  done
done
