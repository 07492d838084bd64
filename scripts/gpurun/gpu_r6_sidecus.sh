# round 6: weight-gradient side stream on a CU subset (tune side_cus), RN50 bs128 step A/B
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
for rep in 1 2; do for n in 0 224 192 160 128; do
  DTR_TUNE=side_cus=$n timeout -k 10 150 python -u bench.py --model imagenet_resnet50 --steps 100 --warmup 15 --phase-steps 0 > gpurun_out/r6_sc_$n.$rep.json 2>/dev/null || exit 1
  echo "side_cus=$n rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_sc_$n.$rep.json)"
done; done
