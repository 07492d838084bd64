#!/usr/bin/env bash
# ImageNet side-car evaluator only (reference: start-resnet-imagenet-eval.sh).
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
RUN_DIR="${RUN_DIR:?set RUN_DIR to the training run directory}"
data_args=(--synthetic)
[[ -n "${DATA:-}" ]] && data_args=(--eval_data_path "$DATA")
run_bg eval "$RUN_DIR/logs/eval.log" "$PY" "$REPO/resnet_imagenet_eval.py" \
  --resnet_size "${RESNET_SIZE:-50}" --device "${EVAL_DEVICE:-auto}" \
  --train_dir "$RUN_DIR/ckpt" --eval_dir "$RUN_DIR/log/validation" "${data_args[@]}" \
  ${EVAL_ONCE:+--eval_once}
