cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 150 "$B > gpurun_out/w0_in50.log 2>&1" \
 150 "DTR_WIDE_128x64=1 $B > gpurun_out/w1_in50.log 2>&1" \
 150 "DTR_WIDE_128x64=2 $B > gpurun_out/w2_in50.log 2>&1" \
 150 "DTR_WIDE_128x64=3 $B > gpurun_out/w3_in50.log 2>&1" \
 150 "DTR_XCD_SWZ=1 $B > gpurun_out/w4_in50.log 2>&1" \
 150 "DTR_NBUF1_KT=2 $B > gpurun_out/w5_in50.log 2>&1" \
 150 "$B > gpurun_out/w0b_in50.log 2>&1"
