cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fuzz_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_def.log 2>&1" \
 100 "$B > gpurun_out/f_128.log 2>&1" \
 100 "$B --batch 64 > gpurun_out/f_64.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/f_32.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/f_16.log 2>&1" \
 100 "$B > gpurun_out/f_128b.log 2>&1"
