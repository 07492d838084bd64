#!/bin/bash
# Fused persistent-step optimizer (sgd_tiles): persist tests, A/B bench vs the three-launch
# optimizer at bs16/bs128, kernel table of the fused step at bs128.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_persist_gpu.py -k fused > gpurun_out/optf_tests.log 2>&1 || { tail -40 gpurun_out/optf_tests.log; exit 1; }
grep "rel grad" gpurun_out/optf_tests.log
for b in 128 16; do for f in 0 1 0 1; do
  DTR_TUNE=opt_fused=$f timeout -k 10 200 python bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/optf_b${b}_f$f.json 2> gpurun_out/optf_err.log || { tail -20 gpurun_out/optf_err.log; exit 1; }
  echo "bs$b opt_fused=$f $(python -c "import json;d=json.load(open('gpurun_out/optf_b${b}_f$f.json'));print(d['ms_per_step'], d['value'])")"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_optf128 -o run -- python3 bench.py --batch 128 --steps 50 --warmup 10 --phase-steps 0 > gpurun_out/prof_optf128.log 2>&1 || { tail -20 gpurun_out/prof_optf128.log; exit 1; }
echo done
