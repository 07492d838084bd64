#!/bin/bash
# Round 3: streaming 1x1 forward, narrowing convs too: numerics, per-shape timing, RN50 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming_narrow" > gpurun_out/bnf_tests.log 2>&1 \
  || { tail -40 gpurun_out/bnf_tests.log; exit 1; }
tail -1 gpurun_out/bnf_tests.log
timeout -k 10 300 python3 scripts/fwd1x1_probe.py 20 > gpurun_out/fwd1x1_probe.md 2>&1 || { tail -20 gpurun_out/fwd1x1_probe.md; exit 1; }
cat gpurun_out/fwd1x1_probe.md
for t in 0 1 0 1; do
  DTR_TUNE=fwd1x1_stream=$t timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/bnf.json 2> gpurun_out/bnf.err || { tail -20 gpurun_out/bnf.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bnf.json')); print('fwd1x1_stream', sys.argv[1], j['value'], j['ms_per_step'], j['phase_ms']['forward'])" $t
done
