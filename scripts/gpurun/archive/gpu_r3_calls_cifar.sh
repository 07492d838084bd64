#!/bin/bash
# Round 3: per-call main-stream timeline of the CIFAR RN50 bs128 step, labelled by layer.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_cc -o run -- python3 scripts/step_calls.py --model cifar_resnet50 --batch 128 --steps 10 --dump gpurun_out/ccalls.json > gpurun_out/ccalls_run.log 2>&1 || { tail -20 gpurun_out/ccalls_run.log; exit 1; }
db=$(find gpurun_out/prof_cc -name '*.db' | head -1)
python3 scripts/step_calls.py --report "$db" gpurun_out/ccalls.json > gpurun_out/cifar_calls.md || exit 1
cp "$db" gpurun_out/ccalls.db && rm -rf gpurun_out/prof_cc
sed -n '/^Main stream/,$p' gpurun_out/cifar_calls.md | head -40
