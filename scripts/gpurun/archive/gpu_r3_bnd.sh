#!/bin/bash
# Round 3: streaming narrow-K dgrad + BN backward (bn_dgrad1x1.hip): numerics, probe, RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming_narrow or bn_backward_apply" > gpurun_out/bnd_tests.log 2>&1 \
  || { tail -40 gpurun_out/bnd_tests.log; exit 1; }
tail -2 gpurun_out/bnd_tests.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_engine_gpu.py -k "bn_backward_apply" > gpurun_out/bnd_tests2.log 2>&1 \
  || { tail -40 gpurun_out/bnd_tests2.log; exit 1; }
tail -2 gpurun_out/bnd_tests2.log
timeout -k 10 300 python3 scripts/bap_probe.py 20 > gpurun_out/bap_probe2.md 2>&1 || { tail -20 gpurun_out/bap_probe2.md; exit 1; }
cat gpurun_out/bap_probe2.md
for t in 0 1024 512 0 1024 512; do
  DTR_TUNE=bap_maxc=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/bap.json 2> gpurun_out/bap.err || { tail -20 gpurun_out/bap.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bap.json')); print('bap_maxc', sys.argv[1], j['value'], j['ms_per_step'])" $t
done
