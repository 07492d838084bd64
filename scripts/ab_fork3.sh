#!/bin/bash
# Tail reduce on main (DTR_REDUCE_MAIN_TAIL) x fork cadence (DTR_FORK_EVERY): tests, then A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_racecheck_gpu.py tests/test_plan_gpu.py tests/test_engine_gpu.py tests/test_dp_gpu.py tests/test_comm_gpu.py > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
out=gpurun_out/ab_fork3.txt; : > $out
for b in 16 128; do
  for cfg in "2 0" "2 1" "4 0" "4 1" "8 1" "4 1"; do
    set -- $cfg
    r=$(DTR_FORK_EVERY=$1 DTR_REDUCE_MAIN_TAIL=$2 timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric) || exit 1
    echo "bs$b fork_every=$1 reduce_main=$2 $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
  done
done
for cfg in "2 1" "4 1" "2 0"; do
  set -- $cfg
  r=$(DTR_FORK_EVERY=$1 DTR_REDUCE_MAIN_TAIL=$2 timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric) || exit 1
  echo "imagenet fork_every=$1 reduce_main=$2 $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
done
