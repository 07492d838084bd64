#!/bin/bash
# Round 6: the hard learnable CIFAR task (gpu_r6_converge.sh) with two more init seeds per
# step path -- the held-out precision spread of the persistent step vs the per-layer plan.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/converge && W=/tmp/dtr_converge && rm -rf $W && mkdir -p $W &&
timeout -k 10 300 python -u -m distributed_tensorflow_resnet_amd.data.learnable $W/data --train 50000 \
  --test 10000 --separation 0.2 --noise 70 --shift 5 > /dev/null 2>&1 || exit 1
for seed in 1 2; do for path in persist layer; do
  if [ $path = layer ]; then export DTR_TUNE=persist=0; else unset DTR_TUNE; fi
  timeout -k 10 300 python -u resnet_cifar_main.py --device gpu --resnet_size 50 --batch_size 128 \
    --train_steps 9000 --lr_schedule_scale 0.1 --train_data_path $W/data --train_dir $W/t_${path}_$seed \
    --log_every 3000 --save_checkpoint_steps 9000 --seed $seed > gpurun_out/converge/seed_${path}_$seed.log 2>&1 || exit 1
  timeout -k 10 300 python -u resnet_cifar_eval.py --device gpu --resnet_size 50 --train_dir $W/t_${path}_$seed \
    --eval_dir $W/e_${path}_$seed --eval_data_path $W/data --eval_once --eval_batch_size 100 \
    --eval_batch_count 100 > gpurun_out/converge/seed_eval_${path}_$seed.log 2>&1 || exit 1
  echo "seed $seed $path: $(grep -h 'precision:' gpurun_out/converge/seed_eval_${path}_$seed.log | tail -1)"
done; done
