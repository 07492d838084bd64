cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_engine_gpu.py tests/test_determinism_gpu.py tests/test_golden_gpu.py tests/test_racecheck_gpu.py tests/test_driver_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_fo.log 2>&1" \
 100 "$C > gpurun_out/fo1_128.log 2>&1" \
 100 "DTR_FUSED_OHWI=0 $C > gpurun_out/fo0_128.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/fo1_16.log 2>&1" \
 100 "DTR_FUSED_OHWI=0 $C --batch 16 > gpurun_out/fo0_16.log 2>&1" \
 100 "$C > gpurun_out/fo1b_128.log 2>&1" \
 100 "DTR_FUSED_OHWI=0 $C > gpurun_out/fo0b_128.log 2>&1"
