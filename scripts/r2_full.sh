cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 900 "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1" \
 120 "python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1" \
 120 "python -u bench.py > gpurun_out/bench_default.log 2>&1"
