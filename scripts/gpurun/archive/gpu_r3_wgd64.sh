#!/bin/bash
# Round 3 end: stage-3 direct wgrad auto rule (implicit-GEMM wgrad at <= 1024 pixels).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wgd_tests.log 2>&1 || { tail -30 gpurun_out/wgd_tests.log; exit 1; }
tail -1 gpurun_out/wgd_tests.log
for b in 16 128 32 16 128 32; do
for cfg in none wgd_bmp64=256; do
  t=$cfg; [ "$cfg" = none ] && t=""
  DTR_TUNE=$t timeout -k 10 120 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/c.json 2> gpurun_out/c.err || { tail -20 gpurun_out/c.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/c.json')); print('bs', sys.argv[2], sys.argv[1], j['ms_per_step'])" $cfg $b
done
done
