# A/B of HIP runtime launch knobs on the eager CIFAR step (bs128 and the 8-GPU per-rank bs16)
set -o pipefail
for B in 128 16; do
  timeout -k 10 120 python3 bench.py --batch $B > gpurun_out/env_base_$B.log 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python3 bench.py --batch $B > gpurun_out/env_kernarg_$B.log 2>&1 || exit $?
  GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python3 bench.py --batch $B > gpurun_out/env_hwq2_$B.log 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=1 GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python3 bench.py --batch $B > gpurun_out/env_both_$B.log 2>&1 || exit $?
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python3 bench.py --model imagenet_resnet50 --steps 60 --warmup 10 > gpurun_out/env_kernarg_in.log 2>&1 || exit $?
grep -H -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/env_*.log
