cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fuzz_gpu.py tests/test_determinism_gpu.py tests/test_racecheck_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_mid.log 2>&1" \
 100 "$B --batch 64 > gpurun_out/d_64.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/d_32.log 2>&1" \
 100 "$B --batch 48 > gpurun_out/d_48.log 2>&1" \
 100 "DTR_C16_MID=-1 $B --batch 48 > gpurun_out/d0_48.log 2>&1" \
 100 "$B --batch 96 > gpurun_out/d_96.log 2>&1" \
 100 "DTR_C16_MID=-1 $B --batch 96 > gpurun_out/d0_96.log 2>&1"
