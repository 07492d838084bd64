# grouped same-shape direct wgrads on the side stream (DTR_WGRAD_GROUP, 1 = per layer)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_racecheck_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_wg.log 2>&1" \
 100 "DTR_WGRAD_GROUP=1 $B --batch 16 > gpurun_out/wg1_16.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/wg8_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP=4 $B --batch 16 > gpurun_out/wg4_16.log 2>&1" \
 100 "DTR_WGRAD_GROUP=1 $B --batch 32 > gpurun_out/wg1_32.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/wg8_32.log 2>&1" \
 100 "DTR_WGRAD_GROUP=1 $B > gpurun_out/wg1_128.log 2>&1" \
 100 "$B > gpurun_out/wg8_128.log 2>&1" \
 200 "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlg16 -- python3 bench.py --batch 16 --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/tlg16.log 2>&1"
