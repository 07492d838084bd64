cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 400 "python -u -m pytest tests/test_determinism_gpu.py tests/test_driver_gpu.py tests/test_engine_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_det.log 2>&1" \
 600 "python -u -m pytest tests/test_convergence_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/t_conv.log 2>&1"
