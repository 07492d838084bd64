#!/bin/bash
# Round 3: streaming kernel with the LDS A tile at K = 256 (stage 3); BNB epilogue cost per dgrad.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming_narrow" > gpurun_out/bnd_tests.log 2>&1 \
  || { tail -40 gpurun_out/bnd_tests.log; exit 1; }
tail -1 gpurun_out/bnd_tests.log
timeout -k 10 300 python3 scripts/bap_probe.py 20 > gpurun_out/bap_probe3.md 2>&1 || { tail -20 gpurun_out/bap_probe3.md; exit 1; }
cat gpurun_out/bap_probe3.md
for t in 512 1024 512 1024; do
  DTR_TUNE=bap_maxc=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/bap.json 2> gpurun_out/bap.err || { tail -20 gpurun_out/bap.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bap.json')); print('bap_maxc', sys.argv[1], j['value'], j['ms_per_step'])" $t
done
timeout -k 10 300 python3 scripts/bnb_cost.py 20 > gpurun_out/bnb_cost.md 2>&1; cat gpurun_out/bnb_cost.md
