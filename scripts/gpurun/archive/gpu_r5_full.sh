#!/bin/bash
# Round 5: the whole GPU test suite, smoke, and the driver's bench command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_tests.log 2>&1 || { tail -60 gpurun_out/r5f_tests.log; exit 1; }
tail -2 gpurun_out/r5f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f_smoke.log 2>&1 || { tail -30 gpurun_out/r5f_smoke.log; exit 1; }
tail -1 gpurun_out/r5f_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { tail -20 gpurun_out/r5f_bench.err; exit 1; }
cat gpurun_out/r5f_bench.json
