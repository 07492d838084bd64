cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 120 "python -u bench.py --steps 200 --warmup 20 > gpurun_out/b128.log 2>&1" \
 120 "python -u bench.py --steps 200 --warmup 20 --batch 32 > gpurun_out/b32.log 2>&1" \
 120 "python -u bench.py --steps 200 --warmup 20 --batch 16 > gpurun_out/b16.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b16 -o run -- python3 bench.py --steps 20 --warmup 5 --batch 16 > gpurun_out/prof_b16.log 2>&1" \
 200 "python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 5 > gpurun_out/in50.log 2>&1" \
 300 "python -u bench.py --model imagenet_resnet101 --steps 20 --warmup 5 > gpurun_out/in101.log 2>&1"
