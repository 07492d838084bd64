# direct conv: weights staged through LDS (DTR_DIRECT_LDSW bitmask: 1 C16, 2 C32, 4 C64)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "DTR_DIRECT_LDSW=7 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_ldsw.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/lw0_16.log 2>&1" \
 100 "DTR_DIRECT_LDSW=4 $B --batch 16 > gpurun_out/lw4_16.log 2>&1" \
 100 "DTR_DIRECT_LDSW=6 $B --batch 16 > gpurun_out/lw6_16.log 2>&1" \
 100 "DTR_DIRECT_LDSW=7 $B --batch 16 > gpurun_out/lw7_16.log 2>&1" \
 100 "$B > gpurun_out/lw0_128.log 2>&1" \
 100 "DTR_DIRECT_LDSW=7 $B > gpurun_out/lw7_128.log 2>&1" \
 100 "DTR_DIRECT_LDSW=4 $B > gpurun_out/lw4_128.log 2>&1" \
 100 "DTR_DIRECT_LDSW=7 python -u scripts/probe_direct.py 16 > gpurun_out/probe16_lw7.log 2>&1"
