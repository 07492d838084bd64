set -o pipefail
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u bench.py > gpurun_out/bench1.log 2>&1 &&
timeout -k 10 240 python -u bench.py --model imagenet_resnet50 > gpurun_out/bench_in.log 2>&1
EC=$?; tail -3 gpurun_out/gpu_tests.log; cat gpurun_out/bench1.log gpurun_out/bench_in.log | grep metric; exit $EC
