# CIFAR direct-conv tile sweep: rows per workgroup (DTR_SMALLC_BM) and column splits
# (DTR_DIRECT_SPLITN) at the 1-GPU (bs128) and 8-GPU (bs16) per-rank batch
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u bench.py --steps 300 --warmup 30 --phase-steps 0"
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'gemm_dgrad_fused' --timeout 200 --timeout-method thread > gpurun_out/t_sw.log 2>&1" \
 100 "$B > gpurun_out/sw_def_128.log 2>&1" \
 100 "DTR_SMALLC_BM=256,64 $B > gpurun_out/sw_b32_128.log 2>&1" \
 100 "DTR_SMALLC_BM=64,128 $B > gpurun_out/sw_b16_128.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=4 $B > gpurun_out/sw_s4_128.log 2>&1" \
 100 "DTR_SMALLC_BM=256,64 DTR_DIRECT_SPLITN=4 $B > gpurun_out/sw_b32s4_128.log 2>&1" \
 100 "$B --batch 16 > gpurun_out/sw_def_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=5 $B --batch 16 > gpurun_out/sw_s5_16.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=4 $B --batch 16 > gpurun_out/sw_s4_16.log 2>&1" \
 100 "$B --batch 32 > gpurun_out/sw_def_32.log 2>&1" \
 100 "DTR_DIRECT_SPLITN=5 $B --batch 32 > gpurun_out/sw_s5_32.log 2>&1"
