#!/bin/bash
# Slice-count A/B of the persistent step (P = 1, 2, 4) per per-rank batch, then rocprof
# kernel tables of the bs16 and bs128 steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
for bp in 16:4 16:2 32:2 32:1 64:2 64:1 96:2 96:1 128:1; do
  b=${bp%%:*}; p=${bp##*:}
  DTR_TUNE=persist=1,persist_slices=$p timeout -k 10 200 python3 bench.py --batch $b --steps 200 --warmup 20 > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/bc.json')); print('cifar bs', sys.argv[1], 'P', sys.argv[2], j['value'], j['ms_per_step'], j['phase_ms'])" $b $p
done
for b in 16 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_prn$b -o run -- python3 bench.py --batch $b --steps 50 --warmup 10 > gpurun_out/prof_prn$b.log 2>&1 || { tail -20 gpurun_out/prof_prn$b.log; exit 1; }
done
timeout -k 10 120 python3 scripts/prn_probe.py 128 50 > gpurun_out/prn_probe128.log 2>&1 && grep -A30 "mean us per phase" gpurun_out/prn_probe128.log
