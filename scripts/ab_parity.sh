cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
C="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -v -k 'parity' --timeout 250 --timeout-method thread > gpurun_out/t_par.log 2>&1" \
 400 "python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_determinism_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t_par2.log 2>&1" \
 200 "python -u scripts/stride2_cost.py > gpurun_out/par_s2c.log 2>&1" \
 150 "$B > gpurun_out/par1_in50.log 2>&1" \
 150 "DTR_PARITY_DGRAD=0 $B > gpurun_out/par0_in50.log 2>&1" \
 100 "$C > gpurun_out/par1_c128.log 2>&1" \
 100 "DTR_PARITY_DGRAD=0 $C > gpurun_out/par0_c128.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/par1_c16.log 2>&1" \
 100 "DTR_PARITY_DGRAD=0 $C --batch 16 > gpurun_out/par0_c16.log 2>&1"
