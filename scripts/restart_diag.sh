#!/bin/bash
# Launcher restart of a 2-rank native (shm) job on one GPU, output streamed to a log
# (diagnosis of tests/test_dp_gpu.py::test_launcher_restarts_native_job_from_checkpoint).
set -o pipefail
out=${1:-gpurun_out/restart.log}
td=$(mktemp -d)
DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1 \
  timeout -k 10 240 python -u -m distributed_tensorflow_resnet_amd.parallel.launch --nproc 2 \
  --master_port 29751 --max_restarts 1 resnet_cifar_main.py --device gpu --resnet_size 8 \
  --batch_size 8 --synthetic --train_steps 6 --train_dir "$td" --save_checkpoint_steps 2 \
  --variable_update horovod --log_every 1 --comm_timeout_secs 120 --fault_kill_step 3 \
  --fault_kill_rank 1 > "$out" 2>&1
rc=$?
echo "rc=$rc" >> "$out"
ls -la "$td" >> "$out"
exit $rc
