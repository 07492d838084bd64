# round 6: per-layer plan optimizer as ONE sgd_tiles launch (tune opt_fused) vs sgd_update_pack
# + ohwi_pack: numerics (engine tests), RN50 / RN101 / CIFAR per-layer step A/B
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_determinism_gpu.py tests/test_stem_s2d_gpu.py > gpurun_out/r6_of_test.log 2>&1 || { tail -30 gpurun_out/r6_of_test.log; exit 1; }
tail -2 gpurun_out/r6_of_test.log
for rep in 1 2; do for of in 0 1; do
  DTR_TUNE=opt_fused=$of timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_of_$of.$rep.json 2>/dev/null || exit 1
  echo "opt_fused=$of rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_of_$of.$rep.json)"
done; done
for of in 0 1; do
  DTR_TUNE=opt_fused=$of,persist=0 timeout -k 10 150 python -u bench.py --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_ofc_$of.json 2>/dev/null || exit 1
  echo "cifar per-layer opt_fused=$of $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_ofc_$of.json)"
done
