#!/bin/bash
# s2d stem + narrow gather + backward-tail split: tests, then ImageNet A/B, then tail A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_stem_s2d_gpu.py tests/test_imagenet_feed_gpu.py tests/test_engine_gpu.py > gpurun_out/s2d_tests.log 2>&1 || { tail -30 gpurun_out/s2d_tests.log; exit 1; }
tail -2 gpurun_out/s2d_tests.log
DTR_TAIL_MAIN=0.5 timeout -k 10 300 $T tests/test_racecheck_gpu.py tests/test_plan_gpu.py > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
for v in 0 1; do
  r=$(DTR_STEM_S2D=$v timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric) || exit 1
  echo "imagenet s2d=$v $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/ab_s2d.txt
done
scripts/ab_tail.sh
