# write-through epilogue stores (DTR_WT_STORE) + threaded issue A/B, CIFAR RN50; epilogue probes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "$B > gpurun_out/wt_def_a.log 2>&1" \
 100 "DTR_WT_STORE=1 $B > gpurun_out/wt_1_a.log 2>&1" \
 100 "DTR_PLAN_THREADS=0 $B > gpurun_out/wt_nothr.log 2>&1" \
 100 "$B > gpurun_out/wt_def_b.log 2>&1" \
 100 "DTR_WT_STORE=1 $B > gpurun_out/wt_1_b.log 2>&1" \
 100 "DTR_WT_STORE=1 $B --batch 16 > gpurun_out/wt_1_16.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/wt_def_16.log 2>&1" \
 200 "DTR_WT_STORE=1 python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 5 --phase-steps 0 > gpurun_out/wt_1_in50.log 2>&1" \
 100 "python -u scripts/probe_direct.py 128 > gpurun_out/probe128.log 2>&1" \
 100 "python -u scripts/probe_direct.py 16 > gpurun_out/probe16.log 2>&1"
