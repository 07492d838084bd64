#!/bin/bash
# Round 3: kernel traces of ImageNet RN50 bs128 with bap_maxc=0 / 2048; then ring_xcd A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for t in 0 2048; do
  DTR_TUNE=bap_maxc=$t timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bap$t -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 5 > gpurun_out/prof_bap$t.log 2>&1 || { tail -20 gpurun_out/prof_bap$t.log; exit 1; }
  db=$(find gpurun_out/prof_bap$t -name '*.db' | head -1)
  python3 scripts/rocpd_summary.py "$db" 10 "ImageNet RN50 bs128 bap_maxc=$t" gpurun_out/bap${t}_kernels.md > /dev/null || exit 1
  rm -rf gpurun_out/prof_bap$t
done
for x in 0 1 2 0 1 2; do
  DTR_TUNE=ring_xcd=$x timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 40 --warmup 5 \
    > gpurun_out/xcd.json 2> gpurun_out/xcd.err || { tail -20 gpurun_out/xcd.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/xcd.json')); print('ring_xcd', sys.argv[1], j['value'], j['ms_per_step'])" $x
done
