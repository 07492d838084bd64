cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_wt3.log 2>&1" \
 100 "$C > gpurun_out/wt3_d_a.log 2>&1" \
 100 "DTR_WT_STORE=0 $C > gpurun_out/wt3_0_a.log 2>&1" \
 100 "$C > gpurun_out/wt3_d_b.log 2>&1" \
 100 "DTR_WT_STORE=0 $C > gpurun_out/wt3_0_b.log 2>&1" \
 100 "$C --batch 32 > gpurun_out/wt3_d_32.log 2>&1" \
 100 "$C --batch 96 > gpurun_out/wt3_d_96.log 2>&1" \
 100 "DTR_WT_STORE=0 $C --batch 96 > gpurun_out/wt3_0_96.log 2>&1"
