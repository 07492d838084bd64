#!/bin/bash
# Round 6: write-through output stores in the streaming BN / 1x1 kernels (build switch
# DTR_WT_STREAM=1) vs the default build, .so files alternated on one box: RN50 bs128 step.
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
SO=distributed_tensorflow_resnet_amd/_C.cpython-310-x86_64-linux-gnu.so &&
for r in 1 2 3 4; do for v in base wt; do
  cp ab/_C_$v.so $SO || exit 1
  timeout -k 10 200 python -u bench.py --model imagenet_resnet50 --steps 150 --warmup 10 --phase-steps 0 > gpurun_out/sw.json 2>/dev/null || exit 1
  echo "r$r $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw.json) $(grep -o '"final_loss": [0-9.]*' gpurun_out/sw.json)"
done; done
cp ab/_C_wt.so $SO && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "bn or 1x1 or stream or engine" > gpurun_out/r6_wts_tests.log 2>&1; tail -1 gpurun_out/r6_wts_tests.log
