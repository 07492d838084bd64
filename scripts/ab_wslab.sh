# split-K slab budget of the generic wgrad in the full ImageNet step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 150 "$B > gpurun_out/ws32.log 2>&1" \
 150 "DTR_WGRAD_SLAB_MB=8 $B > gpurun_out/ws8.log 2>&1" \
 150 "DTR_WGRAD_SLAB_MB=16 $B > gpurun_out/ws16.log 2>&1" \
 150 "DTR_WGRAD_SLAB_MB=4 $B > gpurun_out/ws4.log 2>&1" \
 150 "DTR_WGRAD_TARGET_WG=384 $B > gpurun_out/wt384.log 2>&1" \
 150 "DTR_WGRAD_TARGET_WG=384 DTR_WGRAD_SLAB_MB=8 $B > gpurun_out/wt384s8.log 2>&1" \
 150 "$B > gpurun_out/ws32b.log 2>&1"
