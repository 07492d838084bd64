cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_comm_gpu.py tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_comm.log 2>&1" \
 120 "python -u scripts/launch_floor.py 200 > gpurun_out/launch_floor.log 2>&1" \
 120 "python -u scripts/plan_host_profile.py 16 > gpurun_out/host16.log 2>&1" \
 700 "python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1"
