#!/bin/bash
# Round 5: persistent-step failure handling + headline-instance pins, then the baseline bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  \
  tests/test_golden_gpu.py tests/test_persist_gpu.py > gpurun_out/r5h_tests.log 2>&1 || { tail -40 gpurun_out/r5h_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5h_tests.log | tail -2
grep -E "stage[0-9]|stem:|head:|persistent-vs" gpurun_out/r5h_tests.log | head -20
for b in 128 32 16; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/r5b_b$b.json 2> gpurun_out/r5b_err.log || { tail -20 gpurun_out/r5b_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/r5b_b$b.json'));print(d['ms_per_step'], d['value'], d['config'].get('step_path'))")"
done
timeout -k 10 300 python bench.py --model imagenet_resnet50 > gpurun_out/r5b_in.json 2> gpurun_out/r5b_err.log || { tail -20 gpurun_out/r5b_err.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5b_in.json'));print('imagenet', d['value'], d['ms_per_step'])"
