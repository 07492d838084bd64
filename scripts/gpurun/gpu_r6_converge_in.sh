#!/bin/bash
# Round 6: ImageNet ResNet-50 v2 trained end to end through the reference's CLI on a
# learnable task in the real ImageNet input format (data/learnable.py --imagenet: JPEG
# TFRecord shards, 100 classes, 25.6k train / 5k held out), the real-data pipeline (CPU
# workers decode + VGG resize / crop to uint8, device flip / mean / pack), 3000 steps at
# batch 128 (schedule boundaries x 0.03, LR values x 0.125: the linear scaling rule for
# 128 instead of the reference's 8 x 128 images), then the side-car evaluator.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/converge_in && W=/tmp/dtr_converge_in && rm -rf $W && mkdir -p $W &&
timeout -k 10 300 python -u -m distributed_tensorflow_resnet_amd.data.learnable $W/data --imagenet \
  --train 25600 --test 5000 --classes 100 --workers 12 > gpurun_out/converge_in/data.log 2>&1 || { tail gpurun_out/converge_in/data.log; exit 1; }
timeout -k 10 900 python -u resnet_imagenet_main.py --device gpu --resnet_size 50 --batch_size 128 \
  --train_steps 3000 --lr_schedule_scale 0.03 --lr_value_scale 0.125 --train_data_path $W/data \
  --train_dir $W/train --log_every 250 --save_checkpoint_steps 3000 --num_parallel_calls 12 \
  --num_epochs 100 > gpurun_out/converge_in/train.log 2>&1 || { tail -20 gpurun_out/converge_in/train.log; exit 1; }
timeout -k 10 300 python -u resnet_imagenet_eval.py --device gpu --resnet_size 50 --train_dir $W/train \
  --eval_dir $W/eval --eval_data_path $W/data --eval_once --eval_batch_size 100 \
  --eval_batch_count 50 --num_parallel_calls 12 > gpurun_out/converge_in/eval.log 2>&1 || { tail -20 gpurun_out/converge_in/eval.log; exit 1; }
grep -h "step =\|training done\|global_step/sec\|precision:" gpurun_out/converge_in/train.log gpurun_out/converge_in/eval.log | tail -16
