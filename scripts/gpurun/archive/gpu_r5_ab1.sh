#!/bin/bash
# Round 5: same-process A/B of barrier shards (1 vs 8) x forward slices, bs128/64/32/16.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 500 python -u scripts/persist_ab.py 128,64,32,16 200 3 > gpurun_out/r5_ab1.txt 2>&1; rc=$?
cat gpurun_out/r5_ab1.txt; exit $rc
