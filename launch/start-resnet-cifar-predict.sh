#!/usr/bin/env bash
# Predict 100 test images from the latest checkpoint (reference: start-resnet-cifar-predict.sh).
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
RUN_DIR="${RUN_DIR:?set RUN_DIR to the training run directory}"
exec_args=(--train_dir "$RUN_DIR/ckpt")
[[ -n "${DATA:-}" ]] && exec_args+=(--eval_data_path "$DATA")
"$PY" "$REPO/resnet_cifar_predict.py" "${exec_args[@]}" ${EXTRA_ARGS:-}
