#!/bin/bash
# Round 5 (spill-free build): forward slices per image, auto vs the alternative, same process.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u scripts/persist_ab.py 128,96,64 200 3 > gpurun_out/r5_fwdp.log 2>&1; rc=$?; grep bs gpurun_out/r5_fwdp.log; exit $rc
