cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_engine_gpu.py tests/test_racecheck_gpu.py tests/test_driver_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_mp.log 2>&1" \
 150 "$B > gpurun_out/mp1_a.log 2>&1" \
 150 "DTR_WGRAD_MATPRE=0 $B > gpurun_out/mp0_a.log 2>&1" \
 150 "$B > gpurun_out/mp1_b.log 2>&1" \
 150 "DTR_WGRAD_MATPRE=0 $B > gpurun_out/mp0_b.log 2>&1" \
 250 "python -u bench.py --model imagenet_resnet101 --steps 15 --warmup 5 --phase-steps 0 > gpurun_out/mp1_101.log 2>&1"
