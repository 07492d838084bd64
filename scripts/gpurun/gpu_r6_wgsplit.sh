# round 6: split-K slab cap of the weight gradients (tune wgrad_slab_mb): standalone deep-K
# wgrads and the RN50 bs128 step, same box, each setting twice (interleaved)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
for rep in 1 2; do for mb in 16 32 64 128; do
  DTR_TUNE=wgrad_slab_mb=$mb CALIB_ONLY=wgrad timeout -k 10 120 python -u scripts/gemm_calibration_deepk.py > gpurun_out/r6_wg_$mb.$rep.md 2>&1 || exit 1
  DTR_TUNE=wgrad_slab_mb=$mb timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_in_$mb.$rep.json 2>/dev/null || exit 1
  echo "mb=$mb rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_in_$mb.$rep.json)"
done; done
for mb in 16 32 64 128; do echo "== $mb"; cat gpurun_out/r6_wg_$mb.2.md; done
