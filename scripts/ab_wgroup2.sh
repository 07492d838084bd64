# grouped wgrads: group size / channel-count sweep at bs16 and bs128
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "DTR_WGRAD_GROUP=1 $B --batch 16 > gpurun_out/wgA_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP=2 $B --batch 16 > gpurun_out/wgB_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP_C=1 $B --batch 16 > gpurun_out/wgC_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP_C=6 $B --batch 16 > gpurun_out/wgD_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP=1 $B --batch 16 > gpurun_out/wgA2_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP=1 $B > gpurun_out/wgA_128.log 2>&1" \
 100 "DTR_WGRAD_GROUP=2 $B > gpurun_out/wgB_128.log 2>&1" \
 100 "DTR_WGRAD_GROUP_C=1 $B > gpurun_out/wgC_128.log 2>&1" \
 100 "$B > gpurun_out/wgE_128.log 2>&1"
