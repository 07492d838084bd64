cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 200 "python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/bkt0.log 2>&1" \
 200 "DTR_BM128_MIN=0 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/bkt1.log 2>&1" \
 200 "DTR_XCD_SWZ=1 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/bkt2.log 2>&1" \
 200 "DTR_CONV_PIPE=0 python -u scripts/bench_kernels.py in_7 in_14 > gpurun_out/bkt3.log 2>&1"
