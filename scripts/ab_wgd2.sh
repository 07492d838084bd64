cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 100 "$B --batch 64 > gpurun_out/g0_64.log 2>&1" \
 100 "DTR_WGD_BMP=256,256,128 $B --batch 64 > gpurun_out/g1_64.log 2>&1" \
 100 "DTR_WGD_BMP=1024,512,256 $B --batch 64 > gpurun_out/g2_64.log 2>&1" \
 100 "DTR_WGD_TARGET=192 $B --batch 64 > gpurun_out/g3_64.log 2>&1" \
 100 "DTR_WGD_BMP=256,256,128 $B > gpurun_out/g1_128.log 2>&1" \
 100 "DTR_WGD_BMP=1024,512,256 $B > gpurun_out/g2_128.log 2>&1" \
 100 "$B > gpurun_out/g0_128.log 2>&1" \
 100 "DTR_WGD_TARGET=48 $B --batch 32 > gpurun_out/g4_32.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/g0_32.log 2>&1"
