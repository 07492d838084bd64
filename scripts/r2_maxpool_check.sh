#!/bin/bash
# maxpool_bwd row-grid rewrite: kernel tests + ImageNet engine tests, bench, kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_stem_s2d_gpu.py tests/test_driver_gpu.py > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("imagenet", d["ms_per_step"])' || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_in_mp -o run -- python3 bench.py --model imagenet_resnet50 --steps 6 --warmup 3 > gpurun_out/prof_in_mp.log 2>&1
