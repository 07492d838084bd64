cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_imagenet_feed_gpu.py tests/test_determinism_gpu.py -x -v -s --timeout 250 --timeout-method thread > gpurun_out/t_feed.log 2>&1" \
 600 "python -u -m pytest tests/test_convergence_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/t_conv.log 2>&1" \
 300 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn101 -o run -- python3 bench.py --model imagenet_resnet101 --steps 8 --warmup 3 > gpurun_out/prof_rn101.log 2>&1"
