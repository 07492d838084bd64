#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/fwd1x1_diag.py > gpurun_out/diag.log 2>&1; ec=$?; cat gpurun_out/diag.log | head -120; exit $ec
