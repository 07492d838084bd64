#!/bin/bash
# Round 6: the flagship configuration (CIFAR ResNet-50 v2, batch 128) trained end to end
# through the reference's CLI on a HARD learnable CIFAR-format task (data/learnable.py:
# 50k train / 10k held out, class templates 80 % common field, noise 70, shift 5 -- an
# oracle matched filter gets ~69 %), schedule compressed 10x (0.1 / 0.01 / 0.001 / 1e-4
# from steps 4000 / 6000 / 8000), then the side-car evaluator on the held-out split --
# once on the persistent step and once on the per-layer plan (DTR_TUNE=persist=0).
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/converge && W=/tmp/dtr_converge && rm -rf $W && mkdir -p $W &&
timeout -k 10 300 python -u -m distributed_tensorflow_resnet_amd.data.learnable $W/data --train 50000 \
  --test 10000 --separation 0.2 --noise 70 --shift 5 > gpurun_out/converge/data.log 2>&1 || exit 1
for path in persist layer; do
  if [ $path = layer ]; then export DTR_TUNE=persist=0; else unset DTR_TUNE; fi
  timeout -k 10 600 python -u resnet_cifar_main.py --device gpu --resnet_size 50 --batch_size 128 \
    --train_steps 9000 --lr_schedule_scale 0.1 --train_data_path $W/data --train_dir $W/train_$path \
    --log_every 250 --save_checkpoint_steps 3000 > gpurun_out/converge/train_$path.log 2>&1 || exit 1
  timeout -k 10 300 python -u resnet_cifar_eval.py --device gpu --resnet_size 50 --train_dir $W/train_$path \
    --eval_dir $W/eval_$path --eval_data_path $W/data --eval_once --eval_batch_size 100 \
    --eval_batch_count 100 > gpurun_out/converge/eval_$path.log 2>&1 || exit 1
  cp $W/train_$path/metrics.jsonl gpurun_out/converge/metrics_$path.jsonl 2>/dev/null
  echo "$path: $(grep -h 'step_path' $W/train_$path/metrics.jsonl | head -1 | cut -c1-200)"
  grep -h "step = 9000\|precision:" gpurun_out/converge/train_$path.log gpurun_out/converge/eval_$path.log
done
