cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_perm.log 2>&1" \
 100 "$C > gpurun_out/perm_128a.log 2>&1" \
 100 "$C > gpurun_out/perm_128b.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/perm_16.log 2>&1" \
 100 "$C --batch 64 > gpurun_out/perm_64.log 2>&1" \
 150 "python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0 > gpurun_out/perm_in50.log 2>&1" \
 100 "python -u scripts/probe_direct.py 16 > gpurun_out/perm_probe16.log 2>&1"
