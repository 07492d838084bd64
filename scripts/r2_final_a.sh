# round-2 refresh: benches for the docs + kernel-trace profiles
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30"
I="python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
 100 "$C > gpurun_out/fa_c128.log 2>&1" \
 100 "$C --batch 64 > gpurun_out/fa_c64.log 2>&1" \
 100 "$C --batch 32 > gpurun_out/fa_c32.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/fa_c16.log 2>&1" \
 200 "$I > gpurun_out/fa_in50.log 2>&1" \
 300 "python -u bench.py --model imagenet_resnet101 --steps 20 --warmup 5 > gpurun_out/fa_in101.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/fprof_c -- python3 bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/fprof_c.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/fprof_in -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/fprof_in.log 2>&1"
