#!/bin/bash
# In-kernel phase probe of the final persistent step at bs128 and bs16.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 200 python scripts/prn_probe.py 128 > gpurun_out/probe_final128.txt 2>&1 && timeout -k 10 200 python scripts/prn_probe.py 16 > gpurun_out/probe_final16.txt 2>&1 && echo done
