#!/bin/bash
# Round 5: same-process A/B of the BN barrier scheme (prn_fx 0 = fp64 + counter, 1 = fixed point).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 240 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py > gpurun_out/r5fxab_tests.log 2>&1 || { tail -60 gpurun_out/r5fxab_tests.log; exit 1; }
tail -1 gpurun_out/r5fxab_tests.log
timeout -k 10 600 python -u scripts/persist_tune_ab.py prn_fx 0,1 128,64,32,16 200 3 > gpurun_out/r5fxab.log 2>&1; rc=$?; cat gpurun_out/r5fxab.log; exit $rc
