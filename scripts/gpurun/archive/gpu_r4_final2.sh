#!/bin/bash
# Round-4 evidence refresh after the fused optimizer / head-fold changes: full GPU suite,
# smoke, default bench, per-rank batch sweep of the persistent step, kernel traces.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final2_suite.log 2>&1 || { tail -30 gpurun_out/final2_suite.log; exit 1; }
tail -2 gpurun_out/final2_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python bench.py > gpurun_out/final2_bench.json 2> gpurun_out/final2_bench.err || { tail -20 gpurun_out/final2_bench.err; exit 1; }
cat gpurun_out/final2_bench.json
for b in 16 32 64 128; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/final2_b$b.json 2> gpurun_out/final2_err.log || { tail -20 gpurun_out/final2_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/final2_b$b.json'));print(d['ms_per_step'], d['value'])")"
done
for b in 16 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_fin$b -o run -- python3 bench.py --batch $b --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/prof_fin$b.log 2>&1 || { tail -20 gpurun_out/prof_fin$b.log; exit 1; }
done
echo done
