cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "DTR_DIRECT_SPLITN=3 $B --batch 16 > gpurun_out/s3_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=7 $B --batch 16 > gpurun_out/s7_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=6 $B --batch 16 > gpurun_out/s6_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=2 $B --batch 16 > gpurun_out/s2_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=3 $B --batch 32 > gpurun_out/s3_32.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=7 $B --batch 32 > gpurun_out/s7_32.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=6 $B --batch 32 > gpurun_out/s6_32.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=6 $B --batch 16 > gpurun_out/s6b_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=3 $B --batch 16 > gpurun_out/s3b_16.log 2>&1" \
 100 "DTR_C32_MID=32768 DTR_DIRECT_SPLITN=6 $B --batch 128 > gpurun_out/s6_128.log 2>&1" \
 100 "DTR_C32_MID=32768 $B --batch 128 > gpurun_out/s2_128.log 2>&1"
