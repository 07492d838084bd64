#!/bin/bash
# Kernel traces of the persistent step: no comm / comm after the backward / comm overlapped.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for m in nocomm ov0 ov1; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_$m -o run -- \
    python3 scripts/comm_step_trace.py $m 32 60 > gpurun_out/r5t_$m.log 2>&1 || { tail -30 gpurun_out/r5t_$m.log; exit 1; }
done
ls -R gpurun_out/prof_ov1 | head -20
