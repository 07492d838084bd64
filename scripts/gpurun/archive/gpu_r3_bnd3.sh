#!/bin/bash
# Round 3: streaming 1x1 dgrad with store + BN-backward sums (mode 2): numerics, timing, RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming" > gpurun_out/bnd3_tests.log 2>&1 \
  || { tail -40 gpurun_out/bnd3_tests.log; exit 1; }
tail -1 gpurun_out/bnd3_tests.log
timeout -k 10 300 python3 scripts/bnb_cost.py 20 > gpurun_out/bnb_cost2.md 2>&1 || { tail -20 gpurun_out/bnb_cost2.md; exit 1; }
cat gpurun_out/bnb_cost2.md
for t in 0 1 0 1; do
  DTR_TUNE=dgrad1x1_stream=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/bnd3.json 2> gpurun_out/bnd3.err || { tail -20 gpurun_out/bnd3.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bnd3.json')); print('dgrad1x1_stream', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms']['backward'])" $t
done
