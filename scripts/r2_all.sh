# full GPU suite + smoke
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 900 "python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/t_all.log 2>&1" \
 200 "python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1"
