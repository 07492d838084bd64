#!/usr/bin/env bash
# CIFAR-10/100 ResNet v2 training on N GPUs + side-car evaluator (the reference's
# start-resnet-cifar-main.sh: PS or Horovod containers + eval container).
#   GPUS=4 GLOBAL_BATCH=128 RESNET_SIZE=50 TRAIN_STEPS=200000 \
#   DATA=/data/cifar-10-batches-bin RUN_DIR=/tmp/cifar_run launch/start-resnet-cifar-main.sh
# SYNTHETIC=1 trains on synthetic data; EVAL=0 skips the evaluator; DEVICE=cpu runs the
# gloo CPU path (the reference's localhost pseudo-cluster).
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
GPUS="${GPUS:-1}"
GLOBAL_BATCH="${GLOBAL_BATCH:-128}"
RESNET_SIZE="${RESNET_SIZE:-50}"
DATASET="${DATASET:-cifar10}"
TRAIN_STEPS="${TRAIN_STEPS:-200000}"
RUN_DIR="${RUN_DIR:-/tmp/resnet_${DATASET}_run}"
DATA="${DATA:-}"
EVAL="${EVAL:-1}"
DEVICE="${DEVICE:-auto}"
PORT="${MASTER_PORT:-29540}"
RESTARTS="${MAX_RESTARTS:-3}"
if (( GLOBAL_BATCH % GPUS )); then echo "GLOBAL_BATCH must divide by GPUS" >&2; exit 2; fi
BATCH=$(( GLOBAL_BATCH / GPUS ))
data_args=(--synthetic)
if [[ -z "${SYNTHETIC:-}" && -n "$DATA" ]]; then
  data_args=(--train_data_path "$DATA" --eval_data_path "$DATA")
fi
run_bg train "$RUN_DIR/logs/train.log" "$PY" -m distributed_tensorflow_resnet_amd.parallel.launch \
  --nproc "$GPUS" --master_port "$PORT" --max_restarts "$RESTARTS" \
  "$REPO/resnet_cifar_main.py" --mode train --dataset "$DATASET" --resnet_size "$RESNET_SIZE" \
  --batch_size "$BATCH" --train_steps "$TRAIN_STEPS" --variable_update horovod --device "$DEVICE" \
  --train_dir "$RUN_DIR/ckpt" --log_dir "$RUN_DIR/log/train" "${data_args[@]}" ${EXTRA_ARGS:-}
if [[ "$EVAL" == 1 ]]; then
  # the side-car polls train_dir every 60 s and records Precision / Best Precision
  run_bg eval "$RUN_DIR/logs/eval.log" "$PY" "$REPO/resnet_cifar_main.py" --mode eval \
    --dataset "$DATASET" --resnet_size "$RESNET_SIZE" --device "${EVAL_DEVICE:-cpu}" \
    --train_dir "$RUN_DIR/ckpt" --eval_dir "$RUN_DIR/log/validation" "${data_args[@]}"
fi
echo "[launch] stop with: launch/stop.sh $RUN_DIR"
