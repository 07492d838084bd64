#!/bin/bash
# Round 3: streaming narrow-K 1x1 forward (bn_fwd1x1.hip): numerics + per-shape timing.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming_narrow_fwd" > gpurun_out/bnf_tests.log 2>&1 \
  || { tail -40 gpurun_out/bnf_tests.log; exit 1; }
tail -1 gpurun_out/bnf_tests.log
timeout -k 10 300 python3 scripts/fwd1x1_probe.py 20 > gpurun_out/fwd1x1_probe.md 2>&1; ec=$?; cat gpurun_out/fwd1x1_probe.md; exit $ec
