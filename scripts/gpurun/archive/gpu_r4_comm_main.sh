#!/bin/bash
# Persistent step's all-reduce on the main stream: comm/persist tests + world-1 comm step time.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_comm_gpu.py tests/test_persist_gpu.py tests/test_plan_gpu.py > gpurun_out/comm_main_tests.log 2>&1 || { tail -40 gpurun_out/comm_main_tests.log; exit 1; }
tail -2 gpurun_out/comm_main_tests.log
timeout -k 10 200 python scripts/comm_step_time.py 16 300 && timeout -k 10 200 python scripts/comm_step_time.py 128 200
