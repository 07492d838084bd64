cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_rl.log 2>&1" \
 100 "python -u scripts/reduce_bw.py > gpurun_out/rl_bw.log 2>&1" \
 100 "$C > gpurun_out/rl_128a.log 2>&1" \
 100 "$C > gpurun_out/rl_128b.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/rl_16.log 2>&1" \
 150 "python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0 > gpurun_out/rl_in50.log 2>&1"
