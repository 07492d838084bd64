cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "DTR_WG_WT=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 250 --timeout-method thread > gpurun_out/t_wgwt.log 2>&1" \
 150 "$B > gpurun_out/gwt0_a.log 2>&1" \
 150 "DTR_WG_WT=1 $B > gpurun_out/gwt1_a.log 2>&1" \
 150 "$B > gpurun_out/gwt0_b.log 2>&1" \
 150 "DTR_WG_WT=1 $B > gpurun_out/gwt1_b.log 2>&1" \
 150 "DTR_WT_STORE=1 $B > gpurun_out/gwt2_a.log 2>&1" \
 150 "DTR_WT_STORE=1 DTR_WG_WT=1 $B > gpurun_out/gwt3_a.log 2>&1"
