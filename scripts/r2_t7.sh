cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 200 "python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/t7a.log 2>&1" \
 200 "DTR_WIDE_128x64=3 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/t7b.log 2>&1"
