#!/bin/bash
# Round-2 late check: full GPU tests + smoke, benches, kernel traces for profiles/.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_late.log 2>&1 || { tail -40 gpurun_out/gputest_late.log; exit 1; }
tail -1 gpurun_out/gputest_late.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
out=gpurun_out/bench_late.jsonl; : > $out
timeout -k 10 120 python bench.py 2>/dev/null | grep metric >> $out || exit 1
for b in 64 32 16; do timeout -k 10 120 python bench.py --batch $b --steps 400 --warmup 30 2>/dev/null | grep metric >> $out || exit 1; done
timeout -k 10 150 python bench.py --model imagenet_resnet50 --steps 30 --warmup 5 2>/dev/null | grep metric >> $out || exit 1
timeout -k 10 200 python bench.py --model imagenet_resnet101 --steps 10 --warmup 3 2>/dev/null | grep metric >> $out || exit 1
python -c "
import json
for l in open('$out'):
    d=json.loads(l); c=d['config']
    print(c['model'], c['per_gpu_batch'], d['ms_per_step'], d['value'], c.get('peak_mem_gb'))"
scripts/ab_fork4.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_c_late -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_c_late.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_in_late -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 > gpurun_out/prof_in_late.log 2>&1
