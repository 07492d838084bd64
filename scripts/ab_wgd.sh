# batch-adaptive direct-wgrad tiles (DTR_WGD_TARGET) A/B, CIFAR RN50, 1 GPU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_wgd.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 --batch 16 > gpurun_out/wgd_b16.log 2>&1" \
 120 "DTR_WGD_TARGET=1 python -u bench.py --steps 300 --warmup 30 --batch 16 > gpurun_out/wgd0_b16.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 --batch 32 > gpurun_out/wgd_b32.log 2>&1" \
 120 "DTR_WGD_TARGET=1 python -u bench.py --steps 300 --warmup 30 --batch 32 > gpurun_out/wgd0_b32.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 > gpurun_out/wgd_b128.log 2>&1" \
 120 "DTR_WGD_TARGET=192 python -u bench.py --steps 300 --warmup 30 > gpurun_out/wgd192_b128.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wgd16 -o run -- python3 bench.py --steps 20 --warmup 5 --batch 16 > gpurun_out/prof_wgd16.log 2>&1"
