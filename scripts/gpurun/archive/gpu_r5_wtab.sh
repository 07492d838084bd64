#!/bin/bash
# Round 5: overlap-mode weight-gradient slabs staged in LDS and stored write-through as
# 16-B units -- the comm / persist pins, then the world-1 forced-RCCL step times of the
# previous build (ab_old/) and this one, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_comm_gpu.py tests/test_persist_gpu.py > gpurun_out/r5w_tests.log 2>&1 || { tail -60 gpurun_out/r5w_tests.log; exit 1; }
tail -1 gpurun_out/r5w_tests.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cmd="python scripts/ab_run.py ab_old scripts/comm_step_time.py"; else cmd="python scripts/comm_step_time.py"; fi
    timeout -k 10 300 $cmd 16,32,64,128 200 2 > gpurun_out/r5w_${v}_$r.txt 2>&1 || { tail -20 gpurun_out/r5w_${v}_$r.txt; exit 1; }
    echo "== round $r $v"; grep -v amdgpu.ids gpurun_out/r5w_${v}_$r.txt
  done
done
