#!/bin/bash
# Head folds inside the persistent backward launch: persist/comm tests, smoke, bench bs128/bs16, kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_persist_gpu.py tests/test_comm_gpu.py > gpurun_out/persist_tests.log 2>&1 || { tail -40 gpurun_out/persist_tests.log; exit 1; }
tail -2 gpurun_out/persist_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for b in 128 16 128 16; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/hf_b$b.json 2> gpurun_out/hf_err.log || { tail -20 gpurun_out/hf_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/hf_b$b.json'));print(d['ms_per_step'], d['value'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_hf128 -o run -- python3 bench.py --batch 128 --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/prof_hf128.log 2>&1 || { tail -20 gpurun_out/prof_hf128.log; exit 1; }
echo done
