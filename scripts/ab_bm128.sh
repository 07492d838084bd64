cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
 200 "$B > gpurun_out/bm0_in50.log 2>&1" \
 200 "DTR_BM128_MIN=4096 $B > gpurun_out/bm1_in50.log 2>&1" \
 200 "$B > gpurun_out/bm0b_in50.log 2>&1" \
 200 "DTR_BM128_MIN=4096 $B > gpurun_out/bm1b_in50.log 2>&1"
