cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --model imagenet_resnet50 --steps 30 --warmup 8 --phase-steps 0"
scripts/gpu_steps.sh \
 200 "DTR_SPLITK_TILES=512 python -u scripts/bench_kernels.py in_14 in_28 > gpurun_out/skt512.log 2>&1" \
 200 "DTR_SPLITK_TILES=512 python -u scripts/dgrad_fusion_cost.py > gpurun_out/skt512_dfc.log 2>&1" \
 150 "DTR_SPLITK_TILES=512 $B > gpurun_out/skt512_in50.log 2>&1" \
 150 "$B > gpurun_out/skt256_in50.log 2>&1" \
 150 "DTR_SPLITK_TILES=512 $B > gpurun_out/skt512b_in50.log 2>&1" \
 150 "DTR_SPLITK_TILES=1024 $B > gpurun_out/skt1024_in50.log 2>&1"
