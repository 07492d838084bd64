cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_nb.log 2>&1" \
 200 "DTR_NBUF1_KT=0 python -u scripts/bench_kernels.py in_56 in_28 > gpurun_out/nb0.log 2>&1" \
 200 "python -u scripts/bench_kernels.py in_56 in_28 > gpurun_out/nb1.log 2>&1" \
 150 "DTR_NBUF1_KT=0 $B > gpurun_out/nb0_in50.log 2>&1" \
 150 "$B > gpurun_out/nb1_in50.log 2>&1" \
 150 "DTR_NBUF1_KT=0 $B > gpurun_out/nb0b_in50.log 2>&1" \
 150 "$B > gpurun_out/nb1b_in50.log 2>&1" \
 100 "python -u scripts/reduce_bw.py > gpurun_out/rbw.log 2>&1"
