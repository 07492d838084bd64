#!/bin/bash
# Round 6: (a) the hard learnable CIFAR task on the reference's FULL schedule (0.1 / 0.01 /
# 0.001 / 1e-4 from steps 40k / 60k / 80k, 90k steps, batch 128, persistent step);
# (b) a harder ImageNet-format task (300 classes, 60k train / 10k held out, noise 45) for
# 6000 steps of RN50 through the real-data pipeline.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/converge && W=/tmp/dtr_converge_long && rm -rf $W && mkdir -p $W &&
timeout -k 10 300 python -u -m distributed_tensorflow_resnet_amd.data.learnable $W/cdata --train 50000 \
  --test 10000 --separation 0.2 --noise 70 --shift 5 > /dev/null 2>&1 &&
timeout -k 10 400 python -u resnet_cifar_main.py --device gpu --resnet_size 50 --batch_size 128 \
  --train_steps 90000 --train_data_path $W/cdata --train_dir $W/ct --log_every 10000 \
  --save_checkpoint_steps 30000 > gpurun_out/converge/long_cifar.log 2>&1 &&
timeout -k 10 300 python -u resnet_cifar_eval.py --device gpu --resnet_size 50 --train_dir $W/ct \
  --eval_dir $W/ce --eval_data_path $W/cdata --eval_once --eval_batch_size 100 \
  --eval_batch_count 100 > gpurun_out/converge/long_cifar_eval.log 2>&1 || exit 1
grep -h "training done\|precision:" gpurun_out/converge/long_cifar.log gpurun_out/converge/long_cifar_eval.log | tail -2
timeout -k 10 400 python -u -m distributed_tensorflow_resnet_amd.data.learnable $W/idata --imagenet \
  --train 60000 --test 10000 --classes 300 --noise 45 --workers 12 > gpurun_out/converge/long_in_data.log 2>&1 &&
timeout -k 10 700 python -u resnet_imagenet_main.py --device gpu --resnet_size 50 --batch_size 128 \
  --train_steps 6000 --lr_schedule_scale 0.06 --lr_value_scale 0.125 --train_data_path $W/idata \
  --train_dir $W/it --log_every 500 --save_checkpoint_steps 6000 --num_parallel_calls 12 \
  --num_epochs 100 > gpurun_out/converge/long_in.log 2>&1 &&
timeout -k 10 300 python -u resnet_imagenet_eval.py --device gpu --resnet_size 50 --train_dir $W/it \
  --eval_dir $W/ie --eval_data_path $W/idata --eval_once --eval_batch_size 100 \
  --eval_batch_count 100 --num_parallel_calls 12 > gpurun_out/converge/long_in_eval.log 2>&1 || exit 1
grep -h "step = \|training done\|precision:" gpurun_out/converge/long_in.log gpurun_out/converge/long_in_eval.log | tail -14
