#!/bin/bash
# Round 3: grid-barrier microbenchmark + comm-stream overlap traces (ImageNet RN50 bs128,
# CIFAR RN50 bs32 = the 4-GPU per-rank share).  Each GPU step bounded; stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 microbench/grid_barrier.hip -o /tmp/grid_barrier && timeout -k 10 150 /tmp/grid_barrier > gpurun_out/grid_barrier.md 2> gpurun_out/grid_barrier.err || exit $?
cat gpurun_out/grid_barrier.md
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_overlap_in -- python3 scripts/comm_overlap.py \
  --model imagenet_resnet50 --batch 128 > gpurun_out/overlap_in.log 2>&1 || exit $?
tail -1 gpurun_out/overlap_in.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_overlap_c -- python3 scripts/comm_overlap.py \
  --model cifar_resnet50 --batch 32 > gpurun_out/overlap_c.log 2>&1 || exit $?
tail -1 gpurun_out/overlap_c.log
