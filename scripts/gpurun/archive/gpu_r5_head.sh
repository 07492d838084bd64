#!/bin/bash
# Round 5: head batch folds inside the backward launch vs a launch behind it (same process).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py tests/test_golden_gpu.py tests/test_comm_gpu.py > gpurun_out/r5h2_tests.log 2>&1 || { tail -60 gpurun_out/r5h2_tests.log; exit 1; }
tail -1 gpurun_out/r5h2_tests.log
timeout -k 10 500 python -u scripts/persist_engine_ab.py "persist_head_in_bwd=0;persist_head_in_bwd=1" 128,32,16 200 3 > gpurun_out/r5h2_ab.log 2>&1; rc=$?; grep bs gpurun_out/r5h2_ab.log; exit $rc
