#!/bin/bash
# ring8 with interleaved DMA halves: numerics, probe; CIFAR bs96/128 with the forward rule.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ring8" > gpurun_out/r8_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r8_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ring8_probe.py > gpurun_out/ring8_probe.log 2>&1 || { tail -20 gpurun_out/ring8_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ring8_probe.log
for b in 96 128; do
  timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
