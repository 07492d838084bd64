set -o pipefail
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1 &&
timeout -k 10 180 python -u bench.py > gpurun_out/bench2.log 2>&1
EC=$?; tail -25 gpurun_out/gpu_tests2.log; tail -3 gpurun_out/smoke2.log; cat gpurun_out/bench2.log; exit $EC
