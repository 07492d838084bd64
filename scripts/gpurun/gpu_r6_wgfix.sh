# round 6: wgrad ring with incremental DMA addressing + inline-asm DMAs (no compiler vmcnt(0)
# between the issue and the MFMAs): numerics, RN50 step, kernel table
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_engine_gpu.py -k "wgrad or imagenet or stem" > gpurun_out/r6_wgfix_test.log 2>&1 || { tail -30 gpurun_out/r6_wgfix_test.log; exit 1; }
tail -2 gpurun_out/r6_wgfix_test.log &&
timeout -k 10 200 python -u bench.py --model imagenet_resnet50 > gpurun_out/r6_in2.json 2> gpurun_out/r6_in2.err &&
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_in2.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_in7 -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/prof_in7.log 2>&1
