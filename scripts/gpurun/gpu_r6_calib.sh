# round 6: deep-K vendor-GEMM calibration + ImageNet RN50 bs128 bench
# and kernel table on the current build
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u scripts/gemm_calibration_deepk.py > gpurun_out/r6_calib.md 2>&1 &&
timeout -k 10 200 python -u bench.py --model imagenet_resnet50 > gpurun_out/r6_in.json 2> gpurun_out/r6_in.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_in6 -o run -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 --phase-steps 0 > gpurun_out/prof_in6.log 2>&1
EC=$?; tail -12 gpurun_out/r6_calib.md; cut -c1-300 gpurun_out/r6_in.json; exit $EC
