cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -v -k 'splitk' --timeout 250 --timeout-method thread > gpurun_out/t_sk.log 2>&1" \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_sk2.log 2>&1" \
 200 "DTR_SPLITK=1 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/sk1.log 2>&1" \
 200 "python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/sk2.log 2>&1" \
 200 "DTR_SPLITK=4 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/sk4.log 2>&1" \
 150 "DTR_SPLITK=1 $B > gpurun_out/sk1_in50.log 2>&1" \
 150 "$B > gpurun_out/sk2_in50.log 2>&1" \
 150 "DTR_SPLITK=4 $B > gpurun_out/sk4_in50.log 2>&1"
