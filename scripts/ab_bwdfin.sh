#!/bin/bash
# Finalize-fused BN-backward apply (DTR_BWD_APPLY_FIN 0 / 1 / 2): tests, then A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_bn_apply_acc_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
out=gpurun_out/ab_bwdfin.txt; : > $out
for m in 0 1 2 1 0; do
  r=$(DTR_BWD_APPLY_FIN=$m timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric) || exit 1
  echo "imagenet bwd_apply_fin=$m $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out
done
for b in 16 128; do
  for m in 0 1 0 1; do
    r=$(DTR_BWD_APPLY_FIN=$m timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b bwd_apply_fin=$m $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out
  done
done
