# round 6: deep-ring weight gradients (tune ring_wgrad_deep): numerics, standalone deep-K
# wgrads and the RN50 bs128 step, same box, interleaved
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "ring_wgrad" > gpurun_out/r6_wgdeep_test.log 2>&1 || { tail -30 gpurun_out/r6_wgdeep_test.log; exit 1; }
tail -2 gpurun_out/r6_wgdeep_test.log
for rep in 1 2; do for d in 0 3 4; do
  DTR_TUNE=ring_wgrad_deep=$d CALIB_ONLY=wgrad timeout -k 10 120 python -u scripts/gemm_calibration_deepk.py > gpurun_out/r6_wgd_$d.$rep.md 2>&1 || exit 1
  DTR_TUNE=ring_wgrad_deep=$d timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_ind_$d.$rep.json 2>/dev/null || exit 1
  echo "deep=$d rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_ind_$d.$rep.json)"
done; done
for d in 0 3 4; do echo "== $d"; grep "|" gpurun_out/r6_wgd_$d.2.md; done
