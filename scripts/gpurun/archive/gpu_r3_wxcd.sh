#!/bin/bash
# Round 3: XCD-aware block order of the split-K weight gradients -- numerics, A/B, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/wx_tests.log 2>&1 || { tail -30 gpurun_out/wx_tests.log; exit 1; }
tail -2 gpurun_out/wx_tests.log
timeout -k 10 600 python3 scripts/roofline.py 5 --ab "wgrad_xcd=0" "wgrad_xcd=1" > gpurun_out/roof_wx.md 2>&1 || { tail -20 gpurun_out/roof_wx.md; exit 1; }
grep wgrad gpurun_out/roof_wx.md | tail -24
for r in 1 2; do
for t in "" "wgrad_xcd=0"; do
  DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/rb.json')); print(repr(sys.argv[1]), j['ms_per_step'], j['phase_ms'])" "$t"
done
done
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
python3 -c "import json; j=json.load(open('gpurun_out/rb.json')); print('cifar', j['ms_per_step'])"
