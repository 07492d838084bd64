#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "ring or splitk or parity or conv_ or engine" \
  > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
python3 -c "import json; j=json.load(open('gpurun_out/rb.json')); print(j['ms_per_step'], j['phase_ms'])"
