#!/bin/bash
# Round 3: full GPU suite with the no-fence plan events, then the CIFAR headline bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -2 gpurun_out/full_gpu_tests.log
for b in 128 64 32 16; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('bs', sys.argv[1], j['value'], j['ms_per_step'])" $b
done
