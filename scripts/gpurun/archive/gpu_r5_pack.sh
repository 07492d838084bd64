#!/bin/bash
# Round 5: persistent exchange (pack + all-reduce + early updates beside the backward):
# comm tests, step-time A/B, kernel traces.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_comm_gpu.py tests/test_persist_gpu.py tests/test_engine_gpu.py > gpurun_out/r5p_tests.log 2>&1 || { tail -60 gpurun_out/r5p_tests.log; exit 1; }
tail -1 gpurun_out/r5p_tests.log
timeout -k 10 400 python -u scripts/comm_step_time.py 16,32,64,128 200 3 > gpurun_out/r5p_time.log 2>&1 || { tail -30 gpurun_out/r5p_time.log; exit 1; }
grep bs gpurun_out/r5p_time.log
for m in ov0 ov1; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_p$m -o run -- \
    python3 scripts/comm_step_trace.py $m 32 60 > gpurun_out/r5p_$m.log 2>&1 || { tail -30 gpurun_out/r5p_$m.log; exit 1; }
done
echo traces done
