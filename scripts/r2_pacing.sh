cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 100 "python -u scripts/host_pacing.py 16 > gpurun_out/pace16.log 2>&1" \
 100 "python -u scripts/host_pacing.py 128 > gpurun_out/pace128.log 2>&1" \
 100 "HSA_KERNARG_POOL_SIZE=67108864 python -u scripts/host_pacing.py 16 > gpurun_out/pace16_kp.log 2>&1" \
 100 "ROC_AQL_QUEUE_SIZE=65536 python -u scripts/host_pacing.py 16 > gpurun_out/pace16_aq.log 2>&1" \
 100 "ROC_SIGNAL_POOL_SIZE=65536 python -u scripts/host_pacing.py 16 > gpurun_out/pace16_sp.log 2>&1" \
 100 "HSA_KERNARG_POOL_SIZE=67108864 python -u scripts/host_pacing.py 128 > gpurun_out/pace128_kp.log 2>&1"
