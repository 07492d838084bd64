# round 6: re-sweep of ImageNet schedule knobs on the new wgrad ring (RN50 bs128, 2 rounds)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
for rep in 1 2; do for cfg in "" mat_bn_minc=128 mat_bn_minc=128,mat_bn_elems=20000000 wgrad_slab_mb=24 wgrad_slab_mb=12 wgrad_target_wg=512 wgrad_target_wg=1024 tail_main=0.25 tail_main=0.75 fork_every=1 fork_every=3; do
  DTR_TUNE=$cfg timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_sw.json 2>/dev/null || exit 1
  echo "cfg=[$cfg] rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_sw.json)"
done; done
