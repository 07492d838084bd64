cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -v -k 'splitk' --timeout 250 --timeout-method thread > gpurun_out/t_sk3.log 2>&1" \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_sk4.log 2>&1" \
 200 "python -u scripts/dgrad_fusion_cost.py > gpurun_out/sk_dfc.log 2>&1" \
 200 "DTR_DGRAD_SPLITK=0 python -u scripts/dgrad_fusion_cost.py > gpurun_out/sk_dfc0.log 2>&1" \
 150 "DTR_DGRAD_SPLITK=0 $B > gpurun_out/dsk0_in50.log 2>&1" \
 150 "$B > gpurun_out/dsk1_in50.log 2>&1" \
 150 "DTR_DGRAD_SPLITK=0 $B > gpurun_out/dsk0b_in50.log 2>&1" \
 150 "$B > gpurun_out/dsk1b_in50.log 2>&1"
