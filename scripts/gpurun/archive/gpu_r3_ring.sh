#!/bin/bash
# Round 3: LDS-DMA ring implicit GEMM -- numerics, in-process roofline A/B, engine bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "ring or splitk or parity or conv_fwd or conv_dgrad" \
  > gpurun_out/ring_tests.log 2>&1 || { tail -30 gpurun_out/ring_tests.log; exit 1; }
tail -3 gpurun_out/ring_tests.log
timeout -k 10 600 python3 scripts/roofline.py 5 --ab "ring=0" "ring=1" > gpurun_out/roof_ab.md 2>&1 || { tail -20 gpurun_out/roof_ab.md; exit 1; }
tail -4 gpurun_out/roof_ab.md
for t in "" "ring=0"; do
  DTR_TUNE="$t" timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 50 --warmup 10 > gpurun_out/rb.json 2> gpurun_out/rb.err || { tail -20 gpurun_out/rb.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/rb.json')); print(repr(sys.argv[1]), j['ms_per_step'], j['phase_ms'])" "$t"
done
