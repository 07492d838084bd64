#!/bin/bash
# Final round-4 check after the accumulator-replica change: full GPU suite, smoke, default
# bench, per-rank sweep, ImageNet RN50 bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final3_suite.log 2>&1 || { tail -30 gpurun_out/final3_suite.log; exit 1; }
tail -1 gpurun_out/final3_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python bench.py > gpurun_out/final3_bench.json 2> gpurun_out/final3_bench.err || { tail -20 gpurun_out/final3_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final3_bench.json'));print('default bench', d['value'], d['ms_per_step'], d['vs_baseline'])"
for b in 16 32 64 128; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/final3_b$b.json 2> gpurun_out/final3_err.log || { tail -20 gpurun_out/final3_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/final3_b$b.json'));print(d['ms_per_step'], d['value'])")"
done
timeout -k 10 300 python bench.py --model imagenet_resnet50 > gpurun_out/final3_in.json 2> gpurun_out/final3_err.log || { tail -20 gpurun_out/final3_err.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final3_in.json'));print('imagenet', d['value'], d['ms_per_step'], d['vs_baseline'])"
