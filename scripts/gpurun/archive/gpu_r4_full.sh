#!/bin/bash
# Full GPU test suite (one process), summary to stdout.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1080 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_full.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_full.log | grep -v PASSED | head -40
tail -3 gpurun_out/gpu_full.log
exit $rc
