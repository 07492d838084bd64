cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "$B > gpurun_out/e0_128.log 2>&1" \
 100 "DTR_C32_MID=32768 $B > gpurun_out/e1_128.log 2>&1" \
 100 "$B --batch 64 > gpurun_out/e0_64.log 2>&1" \
 100 "DTR_C32_MID=16384 $B --batch 64 > gpurun_out/e1_64.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=3 $B --batch 64 > gpurun_out/e2_64.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=2 $B --batch 32 > gpurun_out/e2_32.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/e0_32.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=6 $B --batch 16 > gpurun_out/e3_16.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/e0_16.log 2>&1"
