#!/bin/bash
# Round 3: comm-path tests + CIFAR bs32 / ImageNet overlap timing after the no-join fork.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_comm_gpu.py tests/test_dp_gpu.py tests/test_racecheck_gpu.py tests/test_plan_gpu.py \
  > gpurun_out/comm_tests2.log 2>&1 || { tail -30 gpurun_out/comm_tests2.log; exit 1; }
tail -3 gpurun_out/comm_tests2.log
for b in 16 32 64; do
  timeout -k 10 120 python3 scripts/comm_overlap.py --model cifar_resnet50 --batch $b > gpurun_out/ov_c$b.log 2>&1 || exit $?
  tail -1 gpurun_out/ov_c$b.log
done
