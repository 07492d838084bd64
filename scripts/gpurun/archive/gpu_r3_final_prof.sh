#!/bin/bash
# Round 3 late: CIFAR slab-cap A/B; refreshed CIFAR RN50 bs128 and ImageNet RN101 bs256 kernel tables.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for b in 128 32; do
  for cfg in wgrad_slab_mb=32 wgrad_slab_mb=16 wgrad_slab_mb=32 wgrad_slab_mb=16; do
    DTR_TUNE=$cfg timeout -k 10 300 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/c.json 2> gpurun_out/c.err || { tail -20 gpurun_out/c.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/c.json')); print('bs', sys.argv[1], sys.argv[2], j['value'], j['ms_per_step'])" $b $cfg
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_c128 -o run -- python3 bench.py --steps 30 --warmup 10 > gpurun_out/prof_c128.log 2>&1 || { tail -20 gpurun_out/prof_c128.log; exit 1; }
db=$(find gpurun_out/prof_c128 -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" 20 "CIFAR-10 ResNet-50 v2, bs128, 1x MI355X (round 3 late)" gpurun_out/c128_kernels.md > /dev/null || exit 1
rm -rf gpurun_out/prof_c128
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r101 -o run -- python3 bench.py --model imagenet_resnet101 --steps 6 --warmup 3 > gpurun_out/prof_r101.log 2>&1 || { tail -20 gpurun_out/prof_r101.log; exit 1; }
db=$(find gpurun_out/prof_r101 -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" 6 "ImageNet ResNet-101 v2, bs256/GPU, 1x MI355X (round 3 late)" gpurun_out/r101_kernels.md > /dev/null || exit 1
rm -rf gpurun_out/prof_r101
head -5 gpurun_out/c128_kernels.md; head -5 gpurun_out/r101_kernels.md
