#!/bin/bash
# Kernel tables of the final persistent step at bs16 and bs128 + a default bench check.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 16 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_fin$b -o run -- python3 bench.py --batch $b --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/prof_fin$b.log 2>&1 || { tail -20 gpurun_out/prof_fin$b.log; exit 1; }
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cat gpurun_out/bench_default.json
