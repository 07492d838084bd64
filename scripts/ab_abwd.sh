# fused BN backward in the implicit-GEMM dgrad (DTR_GEMM_ABWD) A/B, ImageNet, 1 GPU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'gemm_dgrad_fused or direct_dgrad' --timeout 200 --timeout-method thread > gpurun_out/t_abwd.log 2>&1" \
 300 "python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_imagenet_feed_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_abwd2.log 2>&1" \
 300 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_abwd -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 > gpurun_out/prof_abwd.log 2>&1"
