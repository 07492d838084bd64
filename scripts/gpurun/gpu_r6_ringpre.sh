# round 6: ring forwards with the BN+ReLU prologue in LDS (tune ring_pre): numerics,
# engine tests, RN50 step A/B (interleaved), RN101
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_stem_s2d_gpu.py -k "ring or imagenet or stem or bottleneck" > gpurun_out/r6_rp_test.log 2>&1 || { tail -40 gpurun_out/r6_rp_test.log; exit 1; }
tail -2 gpurun_out/r6_rp_test.log
for rep in 1 2 3; do for rp in 0 1; do
  DTR_TUNE=ring_pre=$rp timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_rp.json 2>/dev/null || exit 1
  echo "ring_pre=$rp rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_rp.json)"
done; done
