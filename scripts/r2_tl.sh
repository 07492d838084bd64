# kernel traces for the stream timeline at bs128 and bs16
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 200 "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl128 -- python3 bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/tl128.log 2>&1" \
 200 "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl16 -- python3 bench.py --batch 16 --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/tl16.log 2>&1"
