#!/bin/bash
# Round 5: bench.py per-rank batches (the 2/4/8-GPU shares on one GPU) and ImageNet RN50.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 128 64 32 16; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/r5b2_b$b.json 2> gpurun_out/r5b2_err.log || { tail -20 gpurun_out/r5b2_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/r5b2_b$b.json'));print(d['ms_per_step'], d['value'], d['config'].get('step_path'))")"
done
timeout -k 10 300 python bench.py --model imagenet_resnet50 > gpurun_out/r5b2_in.json 2> gpurun_out/r5b2_err.log || { tail -20 gpurun_out/r5b2_err.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5b2_in.json'));print('imagenet', d['value'], d['ms_per_step'])"
