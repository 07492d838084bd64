#!/bin/bash
# New-kernel tests, ImageNet A/B (tail split x fused apply-finalize), CIFAR tail 0.5 vs 1,
# then an ImageNet kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_bn_apply_acc_gpu.py tests/test_stem_s2d_gpu.py > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
out=gpurun_out/ab_tail2.txt; : > $out
for cfg in "1 1" "0 1" "0.5 1" "1 0"; do
  set -- $cfg
  r=$(DTR_TAIL_MAIN=$1 DTR_FUSED_APPLY_FIN=$2 timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric) || exit 1
  echo "imagenet tail_main=$1 fused_apply_fin=$2 $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out
done
for b in 32 128; do
  for f in 0.5 1 0.5 1; do
    r=$(DTR_TAIL_MAIN=$f timeout -k 10 120 python bench.py --batch $b --steps 500 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b tail_main=$f $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_in2 -o run -- python3 bench.py --model imagenet_resnet50 --steps 6 --warmup 3 > gpurun_out/prof_in2.log 2>&1
