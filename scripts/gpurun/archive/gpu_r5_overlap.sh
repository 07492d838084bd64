#!/bin/bash
# Round 5: persistent backward with the bucket all-reduces overlapped on the comm stream.
# Correctness (plan identity, loopback doubling under jitter, persistent pins), then the
# world-1 forced-RCCL step-time A/B against the no-comm step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_comm_gpu.py tests/test_persist_gpu.py > gpurun_out/r5o_tests.log 2>&1 || { tail -60 gpurun_out/r5o_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5o_tests.log | tail -2
timeout -k 10 400 python -u scripts/comm_step_time.py 16,32,128 200 3 > gpurun_out/r5o_time.log 2>&1 || { tail -30 gpurun_out/r5o_time.log; exit 1; }
cat gpurun_out/r5o_time.log
