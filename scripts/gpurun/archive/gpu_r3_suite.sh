#!/bin/bash
# Round 3 end: smoke + the whole GPU suite on the final tree.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -1 gpurun_out/full_gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/default.json 2> gpurun_out/default.err || { tail -20 gpurun_out/default.err; exit 1; }
cat gpurun_out/default.json
