#!/bin/bash
# Persistent step quick loop: gradient tests, bs16/32 bench (auto slices), phase probes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread -k "autograd or deterministic or forward" > gpurun_out/prnq_tests.log 2>&1
rc=$?
tail -3 gpurun_out/prnq_tests.log
[ $rc -eq 0 ] || exit $rc
for b in 16 32; do
  DTR_TUNE=persist=1 timeout -k 10 200 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
timeout -k 10 120 python3 scripts/prn_probe.py 16 50 > gpurun_out/prn_probe16.log 2>&1 && cat gpurun_out/prn_probe16.log && \
PRN_WGRAD_WGS=1 timeout -k 10 120 python3 scripts/prn_probe.py 16 50 > gpurun_out/prn_probe16_w1.log 2>&1 && cat gpurun_out/prn_probe16_w1.log
