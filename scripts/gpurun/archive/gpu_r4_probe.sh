#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 200 python3 -u scripts/prn_probe.py 16 50 2>&1 | tee gpurun_out/prn_probe16.txt | grep -v amdgpu.ids
