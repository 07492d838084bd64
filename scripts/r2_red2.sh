cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'reduce or wgrad' --timeout 250 --timeout-method thread > gpurun_out/t_red2.log 2>&1" \
 100 "python -u scripts/reduce_bw.py > gpurun_out/rbw3.log 2>&1" \
 150 "$B > gpurun_out/red2_in50.log 2>&1" \
 150 "$B > gpurun_out/red2_in50b.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/fprof_in2 -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/fprof_in2.log 2>&1"
