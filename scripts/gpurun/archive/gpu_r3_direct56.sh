#!/bin/bash
# Round 3: direct halo conv for the ImageNet 56x56x64 3x3 layers -- numerics, A/B, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "direct or imagenet_stage1" \
  > gpurun_out/d56_tests.log 2>&1 || { tail -30 gpurun_out/d56_tests.log; exit 1; }
tail -2 gpurun_out/d56_tests.log
timeout -k 10 600 python3 scripts/roofline.py 5 --ab "direct_conv=0" "direct_conv=1" "direct_conv=1,direct_ldsw=12" > gpurun_out/roof_d56.md 2>&1 || { tail -20 gpurun_out/roof_d56.md; exit 1; }
grep "56x56 64->64 3x3" gpurun_out/roof_d56.md
for t in "" "direct_conv=0" "direct_ldsw=12"; do
  DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/rb.json')); print(repr(sys.argv[1]), j['ms_per_step'], j['phase_ms'])" "$t"
done
