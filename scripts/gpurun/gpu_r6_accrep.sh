# round 6: fp64 accumulator replicas of the persistent step's BN sums (PRN_ACC_REP 2 / 4 / 8,
# three builds alternated on one box), CIFAR RN50 step at bs16-128
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
SO=distributed_tensorflow_resnet_amd/_C.cpython-310-x86_64-linux-gnu.so
for rep in 1 2; do for b in 16 32 64 128; do for r in 2 4 8; do
  cp ab/_C_r$r.so $SO
  timeout -k 10 120 python -u bench.py --batch $b --steps 300 --warmup 30 --phase-steps 0 > gpurun_out/r6_ar.json 2>/dev/null || exit 1
  echo "bs$b rep=$r round=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_ar.json)"
done; done; done
cp ab/_C_r4.so $SO
