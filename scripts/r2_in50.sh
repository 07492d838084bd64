cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_in50.log 2>&1" \
 200 "python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/in50_a.log 2>&1" \
 200 "python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/in50_b.log 2>&1"
