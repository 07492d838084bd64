#!/bin/bash
# BN barrier microbenchmark with pipelined polls (round 5).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 ./microbench/bn_barrier > gpurun_out/bn_barrier2.md 2>&1; rc=$?; cat gpurun_out/bn_barrier2.md; exit $rc
