#!/bin/bash
# Phase probes of the persistent step at bs16 (4 slices) and bs128 (1 slice).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 16 128; do
  timeout -k 10 120 python3 scripts/prn_probe.py $b 50 > gpurun_out/prn_probe$b.log 2>&1 || { tail -20 gpurun_out/prn_probe$b.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/prn_probe$b.log
done
