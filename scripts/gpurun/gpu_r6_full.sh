# round 6: the whole GPU suite + smoke + 1-GPU benches on the current tree
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u bench.py > gpurun_out/bench1.json 2>/dev/null &&
timeout -k 10 240 python -u bench.py --model imagenet_resnet50 > gpurun_out/bench_in.json 2>/dev/null
EC=$?; tail -3 gpurun_out/gpu_tests.log; cut -c1-200 gpurun_out/bench1.json gpurun_out/bench_in.json; exit $EC
