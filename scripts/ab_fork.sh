# fork cadence of the wgrad side stream (DTR_FORK_EVERY residual blocks per fork)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "DTR_FORK_EVERY=1 $B --batch 16 > gpurun_out/fk1_16.log 2>&1" \
 100 "DTR_FORK_EVERY=2 $B --batch 16 > gpurun_out/fk2_16.log 2>&1" \
 100 "DTR_FORK_EVERY=4 $B --batch 16 > gpurun_out/fk4_16.log 2>&1" \
 100 "DTR_FORK_EVERY=8 $B --batch 16 > gpurun_out/fk8_16.log 2>&1" \
 100 "DTR_FORK_WGRAD=0 $B --batch 16 > gpurun_out/fk0_16.log 2>&1" \
 100 "DTR_FORK_EVERY=4 $B > gpurun_out/fk4_128.log 2>&1" \
 100 "DTR_FORK_EVERY=2 $B > gpurun_out/fk2_128.log 2>&1" \
 100 "DTR_FORK_EVERY=4 $B --batch 32 > gpurun_out/fk4_32.log 2>&1" \
 100 "DTR_FORK_EVERY=2 $B --batch 32 > gpurun_out/fk2_32.log 2>&1"
