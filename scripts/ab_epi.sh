# epilogue: DPP/permlane column sums + prefetched BN-backward coefficients (direct dgrad)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_epi.log 2>&1" \
 100 "$B > gpurun_out/epi_128a.log 2>&1" \
 100 "$B > gpurun_out/epi_128b.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/epi_16.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/epi_32.log 2>&1" \
 200 "python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 5 --phase-steps 0 > gpurun_out/epi_in50.log 2>&1" \
 100 "python -u scripts/probe_direct.py 128 > gpurun_out/probe128.log 2>&1" \
 100 "python -u scripts/probe_direct.py 16 > gpurun_out/probe16.log 2>&1"
