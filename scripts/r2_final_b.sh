# round-2 end refresh: benches + probes + kernel traces
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="python -u bench.py --steps 300 --warmup 30"
I="python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
 100 "$C > gpurun_out/fb_c128.log 2>&1" \
 100 "$C > gpurun_out/fb_c128b.log 2>&1" \
 100 "$C --batch 64 > gpurun_out/fb_c64.log 2>&1" \
 100 "$C --batch 32 > gpurun_out/fb_c32.log 2>&1" \
 100 "$C --batch 16 > gpurun_out/fb_c16.log 2>&1" \
 200 "$I > gpurun_out/fb_in50.log 2>&1" \
 300 "python -u bench.py --model imagenet_resnet101 --steps 20 --warmup 5 > gpurun_out/fb_in101.log 2>&1" \
 100 "python -u scripts/probe_direct.py 16 > gpurun_out/fb_probe16.log 2>&1" \
 100 "python -u scripts/probe_direct.py 128 > gpurun_out/fb_probe128.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/fbprof_c -- python3 bench.py --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/fbprof_c.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/fbprof_in -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/fbprof_in.log 2>&1"
