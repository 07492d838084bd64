# A/B of the per-stream issue threads of Plan::run (DTR_PLAN_THREADS), CIFAR RN50, 1 GPU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_comm_gpu.py tests/test_dp_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_thr.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 --batch 16 > gpurun_out/thr_b16.log 2>&1" \
 120 "DTR_PLAN_THREADS=0 python -u bench.py --steps 300 --warmup 30 --batch 16 > gpurun_out/nothr_b16.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 --batch 32 > gpurun_out/thr_b32.log 2>&1" \
 120 "DTR_PLAN_THREADS=0 python -u bench.py --steps 300 --warmup 30 --batch 32 > gpurun_out/nothr_b32.log 2>&1" \
 120 "python -u bench.py --steps 300 --warmup 30 > gpurun_out/thr_b128.log 2>&1" \
 120 "DTR_PLAN_THREADS=0 python -u bench.py --steps 300 --warmup 30 > gpurun_out/nothr_b128.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_thr16 -o run -- python3 bench.py --steps 20 --warmup 5 --batch 16 > gpurun_out/prof_thr16.log 2>&1"
