#!/bin/bash
# Persistent step at larger per-rank batches (P = 2) vs the per-layer engine, plus a
# per-stage phase probe at bs16.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 48 64; do
  for t in "persist=1" "persist=0"; do
    DTR_TUNE=$t timeout -k 10 200 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $b $t
  done
done
timeout -k 10 120 python3 scripts/prn_probe.py 16 50 > gpurun_out/prn_probe16.log 2>&1 && cat gpurun_out/prn_probe16.log
