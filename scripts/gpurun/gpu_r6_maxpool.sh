#!/bin/bash
# Fixed-window 3x3/2 max-pool kernels: numerics, then the RN50 bs128 step and a kernel
# trace of it (maxpool_fwd / maxpool_bwd per-call times).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k maxpool > gpurun_out/r6_maxpool_test.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --model imagenet_resnet50 > gpurun_out/r6_mp_in$r.json 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_mp_in$r.json
done
rm -rf gpurun_out/prof_mp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mp -o run -- \
  python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 5 > gpurun_out/r6_mp_prof.log 2>&1 || exit 1
f=$(ls gpurun_out/prof_mp/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && grep -i "maxpool" "$f"
exit 0
