#!/bin/bash
# Round 3: persistent multi-layer prototype -- numerics, then the probe vs per-layer launches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_persist_gpu.py > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 1; }
tail -2 gpurun_out/persist_tests.log
timeout -k 10 300 python3 scripts/persist_probe.py 16 32 64 > gpurun_out/persist_probe.md 2>&1 || { tail -20 gpurun_out/persist_probe.md; exit 1; }
cat gpurun_out/persist_probe.md
