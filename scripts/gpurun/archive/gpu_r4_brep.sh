#!/bin/bash
# A/B of the per-layer kernels' BN accumulator replicas (BN_ACC_REP 2/4/8 builds in
# gpurun_variants/), same box: ImageNet RN50 bs128 and the per-layer CIFAR step at bs128.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
SO=distributed_tensorflow_resnet_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO gpurun_variants/_C_tree.so
for round in 1 2; do for rep in 2 4 8; do
  cp gpurun_variants/_C_b$rep.so $SO
  timeout -k 10 300 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 > gpurun_out/brep${rep}_in.json 2> gpurun_out/brep_err.log || { tail -20 gpurun_out/brep_err.log; exit 1; }
  DTR_TUNE=persist=0 timeout -k 10 200 python bench.py --batch 128 --steps 200 --warmup 20 > gpurun_out/brep${rep}_c.json 2> gpurun_out/brep_err.log || { tail -20 gpurun_out/brep_err.log; exit 1; }
  echo "BN_ACC_REP $rep imagenet $(python -c "import json;d=json.load(open('gpurun_out/brep${rep}_in.json'));print(d['ms_per_step'])") cifar-per-layer $(python -c "import json;d=json.load(open('gpurun_out/brep${rep}_c.json'));print(d['ms_per_step'])")"
done; done
cp gpurun_variants/_C_tree.so $SO
