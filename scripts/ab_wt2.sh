cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "DTR_WT_STORE=1 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_wt2.log 2>&1" \
 100 "$C > gpurun_out/wt2_0a.log 2>&1" \
 100 "DTR_WT_STORE=1 $C > gpurun_out/wt2_1a.log 2>&1" \
 100 "$C > gpurun_out/wt2_0b.log 2>&1" \
 100 "DTR_WT_STORE=1 $C > gpurun_out/wt2_1b.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/wt2_0_16.log 2>&1" \
 100 "DTR_WT_STORE=1 $C --batch 16 > gpurun_out/wt2_1_16.log 2>&1" \
 100 "$C --batch 64 > gpurun_out/wt2_0_64.log 2>&1" \
 100 "DTR_WT_STORE=1 $C --batch 64 > gpurun_out/wt2_1_64.log 2>&1" \
 100 "DTR_WT_STORE=1 python -u scripts/probe_direct.py 128 > gpurun_out/wt2_probe.log 2>&1"
