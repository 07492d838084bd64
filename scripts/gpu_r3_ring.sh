#!/bin/bash
# Round 3: LDS-DMA ring implicit GEMM -- numerics, then in-process roofline A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "ring or splitk or parity or conv_fwd or conv_dgrad" \
  > gpurun_out/ring_tests.log 2>&1 || { tail -30 gpurun_out/ring_tests.log; exit 1; }
tail -3 gpurun_out/ring_tests.log
timeout -k 10 600 python3 scripts/roofline.py 5 --ab "ring=0" "ring=1,ring_slots=4" \
  "ring=1,ring_slots=5" > gpurun_out/roof_ab.md 2>&1 || { tail -20 gpurun_out/roof_ab.md; exit 1; }
tail -4 gpurun_out/roof_ab.md
