#!/bin/bash
# Round 5: persistent kernels without VGPR spills (opaque weight-staging addresses) against
# the previous build (ab_old/), same box, alternating runs; then the persistent pins.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for r in 1 2; do
  for b in 128 32 16; do
    for v in old new; do
      if [ $v = old ]; then cmd="python scripts/ab_run.py ab_old bench.py"; else cmd="python bench.py"; fi
      timeout -k 10 200 $cmd --batch $b --steps 300 --warmup 30 > gpurun_out/r5s_${v}_b$b.json 2> gpurun_out/r5s_err.log || { tail -20 gpurun_out/r5s_err.log; exit 1; }
      echo "round $r bs$b $v $(python -c "import json;d=json.load(open('gpurun_out/r5s_${v}_b$b.json'));print(d['ms_per_step'])")"
    done
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py tests/test_golden_gpu.py > gpurun_out/r5s_tests.log 2>&1 || { tail -60 gpurun_out/r5s_tests.log; exit 1; }
tail -1 gpurun_out/r5s_tests.log
