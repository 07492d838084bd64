#!/bin/bash
# Quick bench: bs128 and bs16 persistent step, twice each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 128 16 128 16; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/q_b$b.json 2> gpurun_out/q_err.log || { tail -20 gpurun_out/q_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/q_b$b.json'));print(d['ms_per_step'], d['value'])")"
done
