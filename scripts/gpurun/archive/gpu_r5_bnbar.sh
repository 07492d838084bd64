#!/bin/bash
# Round 5: BatchNorm grid-barrier schemes microbenchmark (microbench/bn_barrier.hip).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 ./microbench/bn_barrier > gpurun_out/bn_barrier.md 2>&1 || { cat gpurun_out/bn_barrier.md; exit 1; }
cat gpurun_out/bn_barrier.md
