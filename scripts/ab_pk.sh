cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 --phase-steps 0"
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_pk.log 2>&1" \
 200 "python -u scripts/dgrad_fusion_cost.py > gpurun_out/pk_dfc.log 2>&1" \
 200 "python -u scripts/fwd_fusion_cost.py > gpurun_out/pk_ffc.log 2>&1" \
 150 "$B > gpurun_out/pk_in50.log 2>&1" \
 150 "$B > gpurun_out/pk_in50b.log 2>&1" \
 100 "$C > gpurun_out/pk_c128.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/pk_c16.log 2>&1"
