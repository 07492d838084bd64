#!/bin/bash
# Round 4 baseline: CIFAR bench at 16/32/128 with per-phase timing (same box).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 16 32 128; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms'])" $b
done
