#!/usr/bin/env bash
# ImageNet ResNet v2 training, 128 images per GPU (the reference's
# start-resnet-imagenet-main.sh / start-resnet-imagenet-horovod-train.sh).
#   GPUS=8 RESNET_SIZE=50 DATA=/data/imagenet-tfrecords RUN_DIR=/tmp/in_run \
#   launch/start-resnet-imagenet-main.sh
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
GPUS="${GPUS:-8}"
BATCH="${BATCH:-128}"
RESNET_SIZE="${RESNET_SIZE:-50}"
TRAIN_STEPS="${TRAIN_STEPS:-112590}"
RUN_DIR="${RUN_DIR:-/tmp/resnet_imagenet_run}"
DATA="${DATA:-}"
EVAL="${EVAL:-1}"
PORT="${MASTER_PORT:-29541}"
RESTARTS="${MAX_RESTARTS:-3}"
data_args=(--synthetic)
if [[ -z "${SYNTHETIC:-}" && -n "$DATA" ]]; then
  data_args=(--train_data_path "$DATA" --eval_data_path "$DATA")
fi
run_bg train "$RUN_DIR/logs/train.log" "$PY" -m distributed_tensorflow_resnet_amd.parallel.launch \
  --nproc "$GPUS" --master_port "$PORT" --max_restarts "$RESTARTS" \
  "$REPO/resnet_imagenet_main.py" --mode train --resnet_size "$RESNET_SIZE" \
  --batch_size "$BATCH" --train_steps "$TRAIN_STEPS" --variable_update horovod \
  --train_dir "$RUN_DIR/ckpt" --log_dir "$RUN_DIR/log/train" "${data_args[@]}" ${EXTRA_ARGS:-}
if [[ "$EVAL" == 1 ]]; then
  run_bg eval "$RUN_DIR/logs/eval.log" "$PY" "$REPO/resnet_imagenet_main.py" --mode eval \
    --resnet_size "$RESNET_SIZE" --device "${EVAL_DEVICE:-cpu}" --train_dir "$RUN_DIR/ckpt" \
    --eval_dir "$RUN_DIR/log/validation" "${data_args[@]}"
fi
echo "[launch] stop with: launch/stop.sh $RUN_DIR"
