#!/bin/bash
# Round-5 baseline on a fresh box: persistent step bs128/32/16, ImageNet RN50 bs128.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for b in 128 32 16; do
  timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/r5b_b$b.json 2> gpurun_out/r5b_err.log || { tail -20 gpurun_out/r5b_err.log; exit 1; }
  echo "bs$b $(python -c "import json;d=json.load(open('gpurun_out/r5b_b$b.json'));print(d['ms_per_step'], d['value'])")"
done
timeout -k 10 300 python bench.py --model imagenet_resnet50 > gpurun_out/r5b_in.json 2> gpurun_out/r5b_err.log || { tail -20 gpurun_out/r5b_err.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5b_in.json'));print('imagenet', d['value'], d['ms_per_step'])"
