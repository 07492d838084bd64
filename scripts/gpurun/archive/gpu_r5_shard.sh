#!/bin/bash
# Round 5: sharded arrival counters in the persistent kernels -- tests, then step times.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py > gpurun_out/r5s_tests.log 2>&1 || { tail -40 gpurun_out/r5s_tests.log; exit 1; }
tail -1 gpurun_out/r5s_tests.log
b() {  # batch, DTR_TUNE
  DTR_TUNE="$2" timeout -k 10 200 python bench.py --batch $1 --steps 300 --warmup 30 > gpurun_out/r5s.json 2> gpurun_out/r5s_err.log || { tail -20 gpurun_out/r5s_err.log; exit 1; }
  echo "bs$1 [$2] $(python -c "import json;d=json.load(open('gpurun_out/r5s.json'));print(d['ms_per_step'], d['value'], d['config'].get('step_path'))")"
}
b 128 "" && b 32 "" && b 16 "" && b 64 "" && b 128 "persist_slices=2" && b 64 "persist_slices=4" && b 32 "persist_slices=2" && b 128 ""
