# round 6: wgrad ring column tiles in (channel block, tap) order: numerics on the
# new build, then RN50 bs128 step + standalone wgrads, old vs new .so alternated (same box)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
SO=distributed_tensorflow_resnet_amd/_C.cpython-310-x86_64-linux-gnu.so &&
cp ab/_C_new.so $SO &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fuzz_gpu.py tests/test_stem_s2d_gpu.py -k "wgrad" > gpurun_out/r6_wr_test.log 2>&1 || { tail -30 gpurun_out/r6_wr_test.log; exit 1; }
tail -2 gpurun_out/r6_wr_test.log
for rep in 1 2; do for v in old new; do
  cp ab/_C_$v.so $SO
  timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_wr.json 2>/dev/null || exit 1
  echo "$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_wr.json)"
  CALIB_ONLY=wgrad timeout -k 10 120 python -u scripts/gemm_calibration_deepk.py 2>/dev/null | cat
done; done
