#!/bin/bash
# Round 3: streaming kernels with 128-column slices at K = 512 (stage 4): numerics; RN50 with
# the wgrad slab cap re-tuned.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "streaming" > gpurun_out/cw_tests.log 2>&1 \
  || { tail -40 gpurun_out/cw_tests.log; exit 1; }
tail -1 gpurun_out/cw_tests.log
for cfg in wgrad_slab_mb=32 wgrad_slab_mb=16 wgrad_slab_mb=12 wgrad_slab_mb=8 wgrad_slab_mb=16,wgrad_target_wg=1024 wgrad_slab_mb=16,wgrad_target_wg=384 wgrad_slab_mb=32 wgrad_slab_mb=16 bap_maxc=2048,wgrad_slab_mb=16; do
  DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/wg.json 2> gpurun_out/wg.err || { tail -20 gpurun_out/wg.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/wg.json')); print(sys.argv[1], j['ms_per_step'], j['phase_ms']['forward'], j['phase_ms']['backward'])" $cfg
done
