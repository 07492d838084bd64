# CIFAR stage-1 (16-channel) tile height: 256 (default) vs 128 rows
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "DTR_SMALLC_BM=128,128 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_c16.log 2>&1" \
 100 "$B > gpurun_out/c16_256a.log 2>&1" \
 100 "DTR_SMALLC_BM=128,128 $B > gpurun_out/c16_128a.log 2>&1" \
 100 "$B > gpurun_out/c16_256b.log 2>&1" \
 100 "DTR_SMALLC_BM=128,128 $B > gpurun_out/c16_128b.log 2>&1" \
 100 "DTR_SMALLC_BM=128,128 $B --batch 64 > gpurun_out/c16_128_64.log 2>&1" \
 100 "$B --batch 64 > gpurun_out/c16_256_64.log 2>&1"
