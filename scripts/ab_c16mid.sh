cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "$B --batch 64 > gpurun_out/m0_64.log 2>&1" \
 100 "DTR_C16_MID=0 $B --batch 64 > gpurun_out/m1_64.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/m0_32.log 2>&1" \
 100 "DTR_C16_MID=0 $B --batch 32 > gpurun_out/m1_32.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/m0_16.log 2>&1" \
 100 "DTR_C16_MID=0 $B --batch 16 > gpurun_out/m1_16.log 2>&1" \
 100 "$B --batch 64 > gpurun_out/m0b_64.log 2>&1" \
 100 "DTR_C16_MID=0 $B --batch 64 > gpurun_out/m1b_64.log 2>&1"
