#!/bin/bash
# Round 3 end: CIFAR bs128 / bs16 knob re-check on the current code (back to back).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for b in 128 16; do
for cfg in none direct_ldsw=7 direct_ldsw=6 wgd_bmp64=512 wgd_bmp32=1024 wgd_target=128 wgd_target=64 fork_every=2 none direct_ldsw=7 direct_ldsw=6 wgd_bmp64=512 wgd_bmp32=1024 wgd_target=128 wgd_target=64 fork_every=2; do
  t=$cfg; [ "$cfg" = none ] && t=""
  DTR_TUNE=$t timeout -k 10 120 python3 bench.py --batch $b --steps 300 --warmup 30 > gpurun_out/c.json 2> gpurun_out/c.err || { tail -20 gpurun_out/c.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/c.json')); print('bs', sys.argv[2], sys.argv[1], j['ms_per_step'])" $cfg $b
done
done
