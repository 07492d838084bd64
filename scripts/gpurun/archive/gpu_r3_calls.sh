#!/bin/bash
# Round 3: per-call main-stream timeline of the ImageNet RN50 bs128 step, labelled by layer.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_calls -o run -- python3 scripts/step_calls.py --dump gpurun_out/calls.json > gpurun_out/calls_run.log 2>&1 || { tail -20 gpurun_out/calls_run.log; exit 1; }
db=$(find gpurun_out/prof_calls -name '*.db' | head -1)
python3 scripts/step_calls.py --report "$db" gpurun_out/calls.json > gpurun_out/in50_calls.md || exit 1
cp "$db" gpurun_out/calls.db && rm -rf gpurun_out/prof_calls
sed -n '/^Main stream/,$p' gpurun_out/in50_calls.md | head -60
