#!/bin/bash
# A/B of the persistent kernels' BN accumulator replicas (gpurun_variants/_C_rep{1,2,4}.so;
# the tree's build = 4; 8 and 16 measured earlier), same box: bench bs128 / bs16, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
SO=distributed_tensorflow_resnet_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO gpurun_variants/_C_tree.so
for round in 1 2; do for rep in 1 2 4; do
  cp gpurun_variants/_C_rep$rep.so $SO
  for b in 128 16; do
    timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/rep${rep}_b$b.json 2> gpurun_out/rep_err.log || { tail -20 gpurun_out/rep_err.log; exit 1; }
    echo "rep$rep bs$b $(python -c "import json;d=json.load(open('gpurun_out/rep${rep}_b$b.json'));print(d['ms_per_step'], d['value'])")"
  done
done; done
cp gpurun_variants/_C_tree.so $SO
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_persist_gpu.py > gpurun_out/rep_tests.log 2>&1 || { tail -30 gpurun_out/rep_tests.log; exit 1; }
tail -1 gpurun_out/rep_tests.log
