#!/bin/bash
# Slice-count A/B at the 4-GPU per-rank share (bs32) and bs48 after the round-4 changes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for cfg in "32 -1" "32 4" "32 2" "48 -1" "48 4" "24 -1" "24 4"; do
  set -- $cfg
  DTR_TUNE=persist_slices=$2 timeout -k 10 200 python3 bench.py --batch $1 --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], 'slices', sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $1 $2
done
timeout -k 10 300 python3 bench.py --model imagenet_resnet50 --steps 30 --warmup 5 > gpurun_out/bi.json 2> gpurun_out/bi.err || { tail -20 gpurun_out/bi.err; exit 1; }
python3 -c "import json; j=json.load(open('gpurun_out/bi.json')); print('RN50', j['value'], j['ms_per_step'], j['phase_ms'])"
