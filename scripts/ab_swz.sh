# XCD-grouped tile order of conv_gemm (DTR_XCD_SWZ) A/B on the ImageNet shapes, 1 GPU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "DTR_XCD_SWZ=1 python -u -m pytest tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_swz.log 2>&1" \
 200 "DTR_XCD_SWZ=0 python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/swz0_in50.log 2>&1" \
 200 "DTR_XCD_SWZ=1 python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/swz1_in50.log 2>&1" \
 200 "DTR_XCD_SWZ=0 python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/swz0b_in50.log 2>&1" \
 200 "DTR_XCD_SWZ=1 python -u bench.py --model imagenet_resnet50 --steps 40 --warmup 10 > gpurun_out/swz1b_in50.log 2>&1" \
 200 "DTR_XCD_SWZ=1 python -u bench.py --steps 300 --warmup 30 > gpurun_out/swz1_c128.log 2>&1"
