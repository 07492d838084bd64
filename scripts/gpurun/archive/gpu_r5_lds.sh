#!/bin/bash
# Round 5: last-released weight-gradient items at N/64 images (bs128: 2, bs64: 1) instead of N/32 -- pins, then the previous build
# (ab_old/) vs this one, same box, alternating runs; then the LDS conflict counter.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py tests/test_golden_gpu.py > gpurun_out/r5l_tests.log 2>&1 || { tail -60 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
for r in 1 2 3; do
  for b in 128 64; do
    for v in old new; do
      case $v in old) cmd="python scripts/ab_run.py ab_old bench.py";; *) cmd="python bench.py";; esac
      case $v in d4) export DTR_PRN_TAIL_READY=43;; s0) export DTR_PRN_TAIL_READY=35;; *) unset DTR_PRN_TAIL_READY;; esac
      timeout -k 10 200 $cmd --batch $b --steps 250 --warmup 30 > gpurun_out/r5l_${v}_b$b.json 2> gpurun_out/r5l_err.log || { tail -20 gpurun_out/r5l_err.log; exit 1; }
      echo "round $r bs$b $v $(python -c "import json;d=json.load(open('gpurun_out/r5l_${v}_b$b.json'));print(d['ms_per_step'])")"
    done
  done
done
