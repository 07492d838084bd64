# round 6: CU-mask partition probe, then the world-2 persistent overlap path on CU halves
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 180 python -u scripts/cu_mask_probe.py > gpurun_out/cu_mask_probe.json 2> gpurun_out/cu_mask_probe.err &&
cat gpurun_out/cu_mask_probe.json &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_dp_gpu.py -k "cu_partition" > gpurun_out/dp_cupart.log 2>&1
EC=$?; tail -30 gpurun_out/dp_cupart.log; exit $EC
