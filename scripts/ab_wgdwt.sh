cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "DTR_WGD_WT=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 250 --timeout-method thread > gpurun_out/t_wgdwt.log 2>&1" \
 100 "$C > gpurun_out/gw0_a.log 2>&1" \
 100 "DTR_WGD_WT=1 $C > gpurun_out/gw1_a.log 2>&1" \
 100 "$C > gpurun_out/gw0_b.log 2>&1" \
 100 "DTR_WGD_WT=1 $C > gpurun_out/gw1_b.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/gw0_16.log 2>&1" \
 100 "DTR_WGD_WT=1 $C --batch 16 > gpurun_out/gw1_16.log 2>&1"
