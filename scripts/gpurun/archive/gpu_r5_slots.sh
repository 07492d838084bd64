#!/bin/bash
# BatchNorm barrier: atomics + counter vs tagged slots microbenchmark.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 ./microbench/bn_slots > gpurun_out/bn_slots.md 2>&1; rc=$?; cat gpurun_out/bn_slots.md; exit $rc
