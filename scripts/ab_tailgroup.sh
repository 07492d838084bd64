#!/bin/bash
# Grouped same-shape weight gradients in the main-stream tail (DTR_TAIL_GROUP 1 vs 8).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
DTR_TAIL_GROUP=8 timeout -k 10 300 $T tests/test_racecheck_gpu.py tests/test_plan_gpu.py tests/test_determinism_gpu.py > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -1 gpurun_out/t6.log
out=gpurun_out/ab_tailgroup.txt; : > $out
for b in 16 32 128; do
  for g in 1 8 1 8; do
    r=$(DTR_TAIL_GROUP=$g timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b tail_group=$g $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
  done
done
