#!/bin/bash
# A/B: the per-layer plan's optimizer as one sgd_tiles launch (ImageNet RN50 bs128, CIFAR per-layer bs128).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for f in 0 1 0 1; do
  DTR_TUNE=opt_fused_layer=$f timeout -k 10 300 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 > gpurun_out/ol_in_$f.json 2> gpurun_out/ol_err.log || { tail -20 gpurun_out/ol_err.log; exit 1; }
  echo "imagenet opt_fused_layer=$f $(python -c "import json;d=json.load(open('gpurun_out/ol_in_$f.json'));print(d['ms_per_step'], d['value'])")"
done
for f in 0 1; do
  DTR_TUNE=persist=0,opt_fused_layer=$f timeout -k 10 200 python bench.py --batch 128 --steps 200 --warmup 20 > gpurun_out/ol_c_$f.json 2> gpurun_out/ol_err.log || { tail -20 gpurun_out/ol_err.log; exit 1; }
  echo "cifar per-layer opt_fused_layer=$f $(python -c "import json;d=json.load(open('gpurun_out/ol_c_$f.json'));print(d['ms_per_step'], d['value'])")"
done
DTR_TUNE=opt_fused_layer=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ol -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/prof_ol.log 2>&1 || { tail -20 gpurun_out/prof_ol.log; exit 1; }
echo done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "optimizer_step or graph_replay" > gpurun_out/ol_tests.log 2>&1 || { tail -30 gpurun_out/ol_tests.log; exit 1; }
tail -2 gpurun_out/ol_tests.log
