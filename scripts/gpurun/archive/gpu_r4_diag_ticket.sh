#!/bin/bash
# Diagnostic build (ticket disabled): sgd_tiles duration without the global_step ticket.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_diag -o run -- python3 bench.py --batch 128 --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/prof_diag.log 2>&1 || { tail -20 gpurun_out/prof_diag.log; exit 1; }
echo done
