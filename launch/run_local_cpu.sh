#!/usr/bin/env bash
# Localhost pseudo-cluster on the CPU (the reference's fake multi-node backend:
# mkl-scripts/run_dist_tf_local.sh, 1 PS + 2 workers on localhost, batch 10, 100 steps):
# NPROC CPU ranks over gloo, synchronous DP, restart-on-failure, foreground.
#   NPROC=2 STEPS=100 launch/run_local_cpu.sh
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
NPROC="${NPROC:-2}"
RUN_DIR="${RUN_DIR:-/tmp/resnet_cpu_run}"
"$PY" -m distributed_tensorflow_resnet_amd.parallel.launch --nproc "$NPROC" \
  --master_port "${MASTER_PORT:-29542}" --max_restarts "${MAX_RESTARTS:-1}" \
  "$REPO/resnet_cifar_main.py" --device cpu --dtype fp32 --synthetic \
  --resnet_size "${RESNET_SIZE:-8}" --batch_size "${BATCH:-10}" --train_steps "${STEPS:-100}" \
  --variable_update horovod --log_every "${LOG_EVERY:-10}" --train_dir "$RUN_DIR/ckpt" \
  --save_checkpoint_steps "${SAVE_STEPS:-50}" ${EXTRA_ARGS:-}
