#!/bin/bash
# Persistent-step GPU tests + smoke (after the fused optimizer change).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_persist_gpu.py tests/test_comm_gpu.py > gpurun_out/persist_tests.log 2>&1 || { tail -40 gpurun_out/persist_tests.log; exit 1; }
tail -3 gpurun_out/persist_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
